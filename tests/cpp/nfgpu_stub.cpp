// nfgpu_stub.cpp — TEST DOUBLE of the C-ABI (include/nfgpu.h) for CPU tests of the reference-side
// adapter (tests/test_adapter.py): built as tests/cpp/_stub/libnfgpu.so and put in front of the real
// library with LD_LIBRARY_PATH.  It runs no frame: it logs every call the adapter makes (one line per
// call to $NFGPU_STUB_LOG), keeps the values it was given so reads return what was written (last
// write wins, no change predicates, no events, no heartbeats), and reports empty frame outputs.  The
// test checks the adapter's wiring — the schema it derives from the class module, the objects and
// values it hands over, where it routes each call — not frame semantics (the GPU tests do that).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "nfgpu.h"

namespace {
struct Stub {
    nfk_config cfg{};
    int nw = 0;  // property words per object
    std::map<std::pair<int64_t, int64_t>, int> idx;
    std::vector<std::vector<uint64_t>> words;
    std::vector<std::vector<uint64_t>> used;                 // [object][rec]
    std::vector<std::vector<std::vector<uint64_t>>> cells;   // [object][rec][col * rows + row]
    std::vector<int> rows, cols;
    std::vector<std::map<int, bool>> sched;                  // [object] kind -> present
    std::vector<std::pair<int64_t, int64_t>> guid;           // [object] (head, data)
    bool committed = false;
    int n_loaded = 0;
    // objects spawned or switched in this window: the library refuses to export them until
    // nfk_execute has applied that (nfgpu_host.hip nfk_export_objects), and so does the stub
    std::set<std::pair<int64_t, int64_t>> moved;
};
FILE* g_log = nullptr;
const char* g_err = "";

// one whole line per call under a lock: the shard tests call the stub from one thread per rank
std::mutex g_log_mu;
void logf(const char* fmt, ...) {
    char line[512];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(line, sizeof(line) - 1, fmt, ap);
    va_end(ap);
    n = n < 0 ? 0 : (n > (int)sizeof(line) - 2 ? (int)sizeof(line) - 2 : n);
    line[n++] = '\n';
    std::lock_guard<std::mutex> lk(g_log_mu);
    if (!g_log) {
        const char* p = getenv("NFGPU_STUB_LOG");
        g_log = fopen(p ? p : "/dev/null", "w");
    }
    fwrite(line, 1, (size_t)n, g_log);
    fflush(g_log);
}
Stub* S(void* w) { return (Stub*)w; }
int find(Stub* s, int64_t h, int64_t d) {
    auto it = s->idx.find({h, d});
    return it == s->idx.end() ? -1 : it->second;
}
int word_of(Stub* s, int pid) {
    const int nif = s->cfg.n_int + s->cfg.n_flt;
    return pid < nif ? pid : nif + 2 * (pid - nif);
}
int add_object(Stub* s, int64_t h, int64_t d) {
    const int o = (int)s->words.size();
    s->idx[{h, d}] = o;
    s->words.emplace_back(s->nw, 0);
    s->used.emplace_back(s->rows.size(), 0);
    std::vector<std::vector<uint64_t>> c;
    for (size_t r = 0; r < s->rows.size(); r++) c.emplace_back((size_t)s->rows[r] * s->cols[r], 0);
    s->cells.push_back(c);
    s->sched.emplace_back();
    s->guid.emplace_back(h, d);
    return o;
}
}  // namespace

extern "C" {
int nfk_create(const nfk_config* cfg, void** out) {
    Stub* s = new Stub;
    s->cfg = *cfg;
    s->nw = cfg->n_int + cfg->n_flt + 2 * cfg->n_obj;
    s->rows.assign(cfg->n_rec, 0);
    s->cols.assign(cfg->n_rec, 0);
    *out = s;
    logf("create %d %d %d %d %d %d", cfg->n_int, cfg->n_flt, cfg->n_obj, cfg->n_class, cfg->n_kind, cfg->n_rec);
    return NFK_OK;
}
int nfk_destroy(void* w) {
    delete S(w);
    return NFK_OK;
}
const char* nfk_last_error(void) { return g_err; }
int nfk_set_prop_flags(void* w, int32_t cls, const uint8_t* f) {
    std::string t;
    for (int p = 0; p < S(w)->cfg.n_int + S(w)->cfg.n_flt + S(w)->cfg.n_obj; p++) t += " " + std::to_string(f[p]);
    logf("flags %d%s", cls, t.c_str());
    return NFK_OK;
}
int nfk_define_record(void* w, int32_t rec, int32_t rows, int32_t cols, const uint8_t* ct, const uint8_t* f) {
    S(w)->rows[rec] = rows;
    S(w)->cols[rec] = cols;
    std::string t;
    for (int c = 0; c < cols; c++) t += std::to_string(ct[c]);
    t += " flags";
    for (int c = 0; c < S(w)->cfg.n_class; c++) t += " " + std::to_string(f[c]);
    logf("record %d %d %d %s", rec, rows, cols, t.c_str());
    return NFK_OK;
}
int nfk_define_kind(void* w, int32_t kind, const nfk_op*, int32_t n_ops) {
    logf("kind %d %d", kind, n_ops);
    return NFK_OK;
}
int nfk_create_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* sc, const int32_t* gr,
                       const uint8_t* cl, const uint8_t* pl) {
    for (int i = 0; i < n; i++) {
        add_object(S(w), gh[i], gd[i]);
        logf("object %lld %lld %d %d %d %d", (long long)gh[i], (long long)gd[i], sc[i], gr[i], cl[i], pl[i]);
    }
    return NFK_OK;
}
int nfk_load_prop(void* w, int32_t pid, const uint64_t* bits) {
    Stub* s = S(w);
    for (size_t o = 0; o < s->words.size(); o++) s->words[o][word_of(s, pid)] = bits[o];
    logf("load_prop %d", pid);
    return NFK_OK;
}
int nfk_load_object(void* w, int32_t pid, const int64_t* head, const int64_t* data) {
    Stub* s = S(w);
    for (size_t o = 0; o < s->words.size(); o++) {
        s->words[o][word_of(s, pid)] = (uint64_t)data[o];
        s->words[o][word_of(s, pid) + 1] = (uint64_t)head[o];
    }
    logf("load_object %d", pid);
    return NFK_OK;
}
int nfk_load_record(void* w, int32_t rec, const uint64_t* cells, const uint64_t* used) {
    Stub* s = S(w);
    const size_t per = (size_t)s->rows[rec] * s->cols[rec];
    int n = 0;
    for (size_t o = 0; o < s->words.size(); o++) {
        s->used[o][rec] = used[o];
        memcpy(s->cells[o][rec].data(), cells + o * per, per * 8);
        n += used[o] != 0;
    }
    logf("load_record %d %d", rec, n);
    return NFK_OK;
}
int nfk_commit(void* w) {
    S(w)->committed = true;
    logf("commit %d", (int)S(w)->words.size());
    return NFK_OK;
}
int nfk_set_scene_props(void* w, int32_t a, int32_t b, int32_t x, int32_t y, int32_t z) {
    logf("scene_props %d %d %d %d %d", a, b, x, y, z);
    return NFK_OK;
}
int nfk_switch_scene(void* w, int64_t h, int64_t d, int32_t sc, int32_t gr, float, float, float) {
    logf("switch %lld %lld %d %d", (long long)h, (long long)d, sc, gr);
    if (find(S(w), h, d) < 0) return NFK_ERR_NOTFOUND;
    S(w)->moved.insert({h, d});
    return NFK_OK;
}
int nfk_destroy_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd) {
    for (int i = 0; i < n; i++) {
        if (find(S(w), gh[i], gd[i]) < 0) return NFK_ERR_NOTFOUND;
        S(w)->idx.erase({gh[i], gd[i]});
        logf("destroy %lld %lld", (long long)gh[i], (long long)gd[i]);
    }
    return NFK_OK;
}
int nfk_object_count(void* w, int32_t* n) {
    *n = (int32_t)S(w)->words.size();
    return NFK_OK;
}
int nfk_row_words(void* w, int32_t* n) {
    *n = S(w)->nw;
    return NFK_OK;
}
// rows = the stored property words (host memory stands for device memory here)
int nfk_export_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, uint64_t* rows) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        if (find(s, gh[i], gd[i]) < 0) return NFK_ERR_NOTFOUND;
        if (s->moved.count({gh[i], gd[i]})) {
            g_err = "export of an object whose membership already changed in this window";
            return NFK_ERR_STATE;
        }
    }
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        memcpy(rows + (size_t)i * s->nw, s->words[o].data(), (size_t)s->nw * 8);
        s->idx.erase({gh[i], gd[i]});
        logf("export %lld %lld", (long long)gh[i], (long long)gd[i]);
    }
    return NFK_OK;
}
int nfk_import_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* sc, const int32_t* gr,
                       const uint8_t* cl, const uint8_t* pl, const uint64_t* rows) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        if (find(s, gh[i], gd[i]) >= 0) return NFK_ERR_ARG;
        const int o = add_object(s, gh[i], gd[i]);
        memcpy(s->words[o].data(), rows + (size_t)i * s->nw, (size_t)s->nw * 8);
        logf("import %lld %lld %d %d %d %d", (long long)gh[i], (long long)gd[i], sc[i], gr[i], cl[i], pl[i]);
    }
    return NFK_OK;
}
int nfk_spawn_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* sc, const int32_t* gr,
                      const uint8_t* cl, const uint8_t* pl, const uint64_t* props) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = add_object(s, gh[i], gd[i]);
        s->moved.insert({gh[i], gd[i]});
        memcpy(s->words[o].data(), props + (size_t)i * s->nw, s->nw * 8);
        std::string t;
        for (int k = 0; k < s->nw; k++) t += " " + std::to_string(props[(size_t)i * s->nw + k]);
        logf("spawn %lld %lld %d %d %d %d%s", (long long)gh[i], (long long)gd[i], sc[i], gr[i], cl[i], pl[i], t.c_str());
    }
    return NFK_OK;
}
// (a batch naming an unknown object is refused whole, as the library refuses it: nothing queued)
int nfk_set_props(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, const uint64_t* bits) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++)
        if (find(s, gh[i], gd[i]) < 0) return NFK_ERR_NOTFOUND;
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        s->words[o][word_of(s, pid[i])] = bits[i];
        logf("set %lld %lld %d %llu", (long long)gh[i], (long long)gd[i], pid[i], (unsigned long long)bits[i]);
    }
    return NFK_OK;
}
// the by-object entry points log as their NFGUID forms do (object index -> NFGUID, creation order)
int nfk_set_props_obj(void* w, int32_t n, const int32_t* obj, const int32_t* pid, const uint64_t* bits) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        if (obj[i] < 0 || obj[i] >= (int)s->guid.size()) return NFK_ERR_NOTFOUND;
        const int rc = nfk_set_props(w, 1, &s->guid[obj[i]].first, &s->guid[obj[i]].second, pid + i, bits + i);
        if (rc) return rc;
    }
    return NFK_OK;
}
int nfk_set_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, const int64_t* vh,
                    const int64_t* vd) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        s->words[o][word_of(s, pid[i])] = (uint64_t)vd[i];
        s->words[o][word_of(s, pid[i]) + 1] = (uint64_t)vh[i];
        logf("set_object %lld %lld %d %lld %lld", (long long)gh[i], (long long)gd[i], pid[i], (long long)vh[i],
             (long long)vd[i]);
    }
    return NFK_OK;
}
int nfk_get_objects(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, int64_t* vh,
                    int64_t* vd) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        vd[i] = (int64_t)s->words[o][word_of(s, pid[i])];
        vh[i] = (int64_t)s->words[o][word_of(s, pid[i]) + 1];
    }
    return NFK_OK;
}
int nfk_get_props(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, uint64_t* bits) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        bits[i] = s->words[o][word_of(s, pid[i])];
    }
    return NFK_OK;
}
int nfk_set_records(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, const int32_t* row,
                    const int32_t* col, const uint8_t* is_float, const uint64_t* bits) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        if ((s->used[o][rec[i]] >> row[i]) & 1) s->cells[o][rec[i]][(size_t)col[i] * s->rows[rec[i]] + row[i]] = bits[i];
        logf("set_record %lld %lld %d %d %d %d %llu", (long long)gh[i], (long long)gd[i], rec[i], row[i], col[i],
             is_float ? is_float[i] : -1, (unsigned long long)bits[i]);
    }
    return NFK_OK;
}
int nfk_record_rows(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, const int32_t* op,
                    const int32_t* row, const uint64_t* values) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        uint64_t& u = s->used[o][rec[i]];
        int r = row[i];
        if (op[i] == 1) {
            for (int k = 0; r < 0 && k < s->rows[rec[i]]; k++)
                if (!((u >> k) & 1)) r = k;
            if (r >= 0) {
                u |= 1ull << r;
                for (int c = 0; c < s->cols[rec[i]]; c++)
                    s->cells[o][rec[i]][(size_t)c * s->rows[rec[i]] + r] = values ? values[(size_t)i * NFK_MAX_REC_COLS + c] : 0;
            }
        } else if (op[i] == 2) {
            u &= ~(1ull << r);
        } else {
            u = 0;
        }
        logf("row %lld %lld %d %d %d", (long long)gh[i], (long long)gd[i], rec[i], op[i], row[i]);
    }
    return NFK_OK;
}
int nfk_get_used_rows(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, uint64_t* masks) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        masks[i] = s->used[o][rec[i]];
    }
    return NFK_OK;
}
int nfk_get_records(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, const int32_t* row,
                    const int32_t* col, uint64_t* bits) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        bits[i] = ((s->used[o][rec[i]] >> row[i]) & 1) ? s->cells[o][rec[i]][(size_t)col[i] * s->rows[rec[i]] + row[i]] : 0;
    }
    return NFK_OK;
}
int nfk_add_schedules(void* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* kind, const float* iv,
                      const int32_t* cnt, const int64_t* now) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        const int o = find(s, gh[i], gd[i]);
        if (o < 0) return NFK_ERR_NOTFOUND;
        s->sched[o][kind[i]] = true;
        logf("add_schedule %lld %lld %d %g %d %lld", (long long)gh[i], (long long)gd[i], kind[i], iv[i], cnt[i],
             (long long)now[i]);
    }
    return NFK_OK;
}
int nfk_remove_schedule(void* w, int64_t h, int64_t d, int32_t kind) {
    const int o = find(S(w), h, d);
    if (o < 0) return NFK_ERR_NOTFOUND;
    S(w)->sched[o].erase(kind);
    logf("remove_schedule %lld %lld %d", (long long)h, (long long)d, kind);
    return NFK_OK;
}
int nfk_remove_all_schedules(void* w, int64_t h, int64_t d) {
    const int o = find(S(w), h, d);
    if (o < 0) return NFK_ERR_NOTFOUND;
    S(w)->sched[o].clear();
    logf("remove_schedules %lld %lld", (long long)h, (long long)d);
    return NFK_OK;
}
int nfk_schedule_calls(void* w, int32_t n, const int32_t* op, const int64_t* gh, const int64_t* gd, const int32_t* kind,
                       const float* iv, const int32_t* cnt, const int64_t* now) {
    for (int i = 0; i < n; i++)
        if (find(S(w), gh[i], gd[i]) < 0) return NFK_ERR_NOTFOUND;
    for (int i = 0; i < n; i++) {
        const int rc = op[i] == 1 ? nfk_add_schedules(w, 1, gh + i, gd + i, kind + i, iv + i, cnt + i, now + i)
                     : op[i] == 2 ? nfk_remove_schedule(w, gh[i], gd[i], kind[i])
                                  : nfk_remove_all_schedules(w, gh[i], gd[i]);
        if (rc) return rc;
    }
    return NFK_OK;
}
int nfk_schedule_calls_obj(void* w, int32_t n, const int32_t* op, const int32_t* obj, const int32_t* kind,
                           const float* iv, const int32_t* cnt, const int64_t* now) {
    Stub* s = S(w);
    for (int i = 0; i < n; i++) {
        if (obj[i] < 0 || obj[i] >= (int)s->guid.size()) return NFK_ERR_NOTFOUND;
        const int rc = nfk_schedule_calls(w, 1, op + i, &s->guid[obj[i]].first, &s->guid[obj[i]].second, kind + i,
                                          iv + i, cnt + i, now + i);
        if (rc) return rc;
    }
    return NFK_OK;
}
int nfk_exist_schedule(void* w, int64_t h, int64_t d, int32_t kind, int32_t* e) {
    const int o = find(S(w), h, d);
    *e = o >= 0 && S(w)->sched[o].count(kind);
    return NFK_OK;
}
int nfk_watch_props(void*, int32_t n, const int32_t* pid) {
    std::string t;
    for (int32_t i = 0; i < n; i++) t += " " + std::to_string(pid[i]);
    logf("watch%s", t.c_str());
    return NFK_OK;
}
int nfk_read_chain(void*, int32_t, int32_t* n, int32_t*, int32_t*, int32_t*, int32_t*, uint64_t*, uint64_t*) {
    *n = 0;  // (the stub runs no programs)
    return NFK_OK;
}
int nfk_read_added(void*, int32_t, int32_t* n, int64_t*, int64_t*, int32_t*) {
    *n = 0;
    return NFK_OK;
}
int nfk_execute(void* w, int64_t now) {
    logf("execute %lld", (long long)now);
    S(w)->moved.clear();
    return NFK_OK;
}
int nfk_execute_calls(void* w) {
    logf("execute_calls");
    return NFK_OK;
}
int nfk_sync(void*) { return NFK_OK; }
int nfk_get_stream(void*, void** s) {
    *s = nullptr;
    return NFK_OK;
}
int nfk_summary_get(void* w, nfk_summary* out) {
    memset(out, 0, sizeof *out);
    out->n_entities = (int64_t)S(w)->idx.size();
    return NFK_OK;
}
int nfk_outputs_get(void*, nfk_outputs* out) {
    memset(out, 0, sizeof *out);
    return NFK_OK;
}
int nfk_read_prop(void*, int32_t, uint64_t*) { return NFK_ERR_STATE; }
int nfk_read_object(void*, int32_t, int64_t*, int64_t*) { return NFK_ERR_STATE; }
int nfk_read_record(void*, int32_t, uint64_t*) { return NFK_ERR_STATE; }
int nfk_read_schedules(void*, int64_t*, int32_t*, uint8_t*) { return NFK_ERR_STATE; }
int nfk_read_events(void*, int32_t*, int32_t*, uint64_t*, uint64_t*) { return NFK_OK; }
int nfk_read_events_obj(void*, uint64_t*, uint64_t*) { return NFK_OK; }
int nfk_read_rec_events(void*, int32_t*, uint32_t*, uint64_t*, uint64_t*) { return NFK_OK; }
int nfk_read_fired(void*, int32_t*, int32_t*, int32_t*) { return NFK_OK; }
int nfk_read_fanout(void*, uint32_t* off, int32_t*) {
    off[0] = 0;
    return NFK_OK;
}
int nfk_read_frame(void*, uint32_t, nfk_frame_host* out) {
    memset(out, 0, sizeof *out);
    return NFK_OK;
}
// the live objects' top k by the property's value (ZREVRANGE order: score descending, then the
// member string "head-data" descending), as the library's nfk_rank_top answers
int nfk_rank_top(void* w, int32_t pid, int32_t k, int32_t* n, int64_t* gh, int64_t* gd, double* score) {
    Stub* s = S(w);
    struct R {
        double v;
        std::string m;
        int64_t h, d;
    };
    std::vector<R> all;
    for (const auto& kv : s->idx) {
        const uint64_t b = s->words[(size_t)kv.second][(size_t)word_of(s, pid)];
        double v;
        if (pid < s->cfg.n_int) v = (double)(int64_t)b;
        else memcpy(&v, &b, 8);
        all.push_back({v, std::to_string(kv.first.first) + "-" + std::to_string(kv.first.second), kv.first.first,
                       kv.first.second});
    }
    std::sort(all.begin(), all.end(), [](const R& a, const R& b) { return a.v != b.v ? a.v > b.v : a.m > b.m; });
    *n = (int32_t)std::min<size_t>(all.size(), (size_t)std::max(k, 0));
    for (int32_t i = 0; i < *n; i++) {
        gh[i] = all[(size_t)i].h;
        gd[i] = all[(size_t)i].d;
        score[i] = all[(size_t)i].v;
    }
    logf("rank_top %d %d %d", pid, k, *n);
    return NFK_OK;
}
}
