// ref_harness.cpp — drives the REFERENCE's own classes (built from the sources
// under /root/reference by oracle/build_ref.sh into oracle/_ref/nf_ref_harness).
//
// TEST INFRASTRUCTURE ONLY: used to pin oracle/nf_oracle.c (golden fixtures in
// tests/golden/) and as bench.py's cpu_baseline ("reference" kind).
//
// Reference classes used unmodified (flyish/NoahGameFrame):
//   NFCPropertyManager / NFCProperty   NFComm/NFCore/NFCPropertyManager.cpp, NFCProperty.cpp
//   NFCRecord                          NFComm/NFCore/NFCRecord.cpp (SetInt, AddRow, Remove, Clear)
//   NFCScheduleModule                  NFComm/NFKernelPlugin/NFCScheduleModule.cpp
//   NFCSceneInfo / NFCSceneGroupInfo   NFComm/NFPluginModule/NFISceneAOIModule.h (group maps)
// Restated here (the kernel/AOI modules need the full plugin manager to build):
//   object lookup + SetPropertyInt/Float   NFCKernelModule.cpp:323-347
//   GetBroadCastObject / OnPropertyCommonEvent recipient lists
//                                          NFCSceneAOIModule.cpp:227-258, 531-593,
//                                          NFCKernelModule.cpp:1270-1294
//   SwitchScene                            NFCKernelModule.cpp:901-951 (over the reference's
//                                          NFCSceneInfo group maps and property manager)
// NFCScheduleModule reads wall time through NFGetTime() (NFPlatform.h:367,
// std::chrono::system_clock); this harness supplies a virtual CLOCK_REALTIME
// by defining clock_gettime, so the real scheduler runs deterministically.
//
// Usage: nf_ref_harness <workload.nfio> <out.nfio>        parity outputs
//        nf_ref_harness --bench <workload.nfio> <ticks>    timing (prints JSON)
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "NFComm/NFCore/NFCDataList.h"
#include "NFComm/NFCore/NFCPropertyManager.h"
#include "NFComm/NFCore/NFCRecord.h"
#include "NFComm/NFKernelPlugin/NFCScheduleModule.h"
#include "NFComm/NFPluginModule/NFISceneAOIModule.h"
#include "../include/nfgpu.h"
#include "nfio.h"

static int64_t g_now_ms = 0;
extern "C" int clock_gettime(clockid_t clk, struct timespec* ts) {
    if (clk == CLOCK_REALTIME) {
        ts->tv_sec = g_now_ms / 1000;
        ts->tv_nsec = (g_now_ms % 1000) * 1000000;
        return 0;
    }
    return (int)syscall(SYS_clock_gettime, clk, ts);
}

static uint64_t dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static double bitsd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

// expose the scheduler's protected tables for the final-state dump
struct SchedProbe : public NFCScheduleModule {
    explicit SchedProbe(NFIPluginManager* p) : NFCScheduleModule(p) {}
    bool Probe(const NFGUID& self, const std::string& name, int64_t* next, int32_t* remain) {
        auto m = mObjectScheduleMap.GetElement(self);
        if (!m) return false;
        auto e = m->GetElement(name);
        if (!e) return false;
        *next = e->mnNextTriggerTime;
        *remain = e->mnRemainCount;
        return true;
    }
};

struct SetEv { int32_t obj, pid; uint64_t o, n, oh, nh; int64_t seq; };
struct RSetEv { int32_t obj; uint32_t rrc; uint64_t o, n; int64_t seq; };
struct Fired { int32_t obj, kind, rem; };

struct World {
    int64_t N, NI, NF, NC, NK, NR, NO;
    std::vector<std::string> pname, kname;
    std::map<std::string, int> kind_of;
    std::vector<NFGUID> id;
    std::map<NFGUID, int> obj_of;  // NFCKernelModule's NFMapEx<NFGUID, NFIObject> lookup
    std::vector<NF_SHARE_PTR<NFIPropertyManager>> pm;
    std::vector<std::vector<NF_SHARE_PTR<NFIRecord>>> rec;
    std::vector<NF_SHARE_PTR<NFIPropertyManager>> class_pm;  // class templates carry the flags
    std::vector<uint8_t> rflags;  // [NC][NR]
    std::vector<int32_t> scene, group;
    std::vector<uint8_t> cls, isplayer, alive;
    std::map<int, NF_SHARE_PTR<NFCSceneInfo>> scenes;
    nfk_op ops[NFK_MAX_KINDS][NFK_MAX_OPS];
    int32_t nops[NFK_MAX_KINDS];
    int32_t rec_rows[NFK_MAX_RECORDS], rec_cols[NFK_MAX_RECORDS];
    std::vector<SetEv> slog;
    std::vector<RSetEv> rlog;
    std::vector<Fired> fired;
    int64_t seq = 0;
    bool bench = false;
    int64_t bench_msgs = 0;
};
static World W;

// --- GetBroadCastObject (NFCSceneAOIModule.cpp:531-593) for an (object, flags) pair: public ->
// GetGroupObjectList(scene, group, "Player", self) (NFCKernelModule.cpp:1270-1294): the group's
// player map then its other map, objects of class Player except self ---
static void broadcast_list(int32_t o, uint8_t fl, NFIDataList& out) {
    if (fl & NFK_PUBLIC) {
        auto si = W.scenes[W.scene[o]];
        auto gi = si->GetElement(W.group[o]);
        if (!gi) return;
        for (int which = 0; which < 2; which++) {
            auto& lst = which == 0 ? gi->mxPlayerList : gi->mxOtherList;
            NFGUID ident;
            lst.First(ident);
            while (!ident.IsNull()) {
                if (ident != W.id[o] && W.isplayer[W.obj_of[ident]]) out.Add(ident);
                ident = NFGUID();
                lst.Next(ident);
            }
        }
    } else if ((fl & NFK_PRIVATE) && !(fl & NFK_UPLOAD)) {
        out.Add(W.id[o]);
    }
}

static uint8_t prop_flags(int32_t o, int32_t pid) {
    auto p = W.class_pm[W.cls[o]]->GetElement(W.pname[pid]);
    uint8_t f = 0;
    if (p->GetPublic()) f |= NFK_PUBLIC;
    if (p->GetPrivate()) f |= NFK_PRIVATE;
    if (p->GetUpload()) f |= NFK_UPLOAD;
    return f;
}

static int OnPropertyEvent(int32_t obj, int32_t pid, const NFIDataList::TData& oldv, const NFIDataList::TData& newv) {
    if (W.bench) {
        // the reference fans out per Set (AOI:227-258): build the recipient list now
        NFCDataList lst;
        broadcast_list(obj, prop_flags(obj, pid), lst);
        W.bench_msgs += lst.GetCount();
        return 0;
    }
    if (pid >= W.NI + W.NF) {  // TDATA_OBJECT: NFGUID (data, head)
        const NFGUID a = oldv.GetObject(), b = newv.GetObject();
        W.slog.push_back({obj, pid, (uint64_t)a.nData64, (uint64_t)b.nData64, (uint64_t)a.nHead64,
                          (uint64_t)b.nHead64, W.seq++});
        return 0;
    }
    uint64_t o = pid < W.NI ? (uint64_t)oldv.GetInt() : dbits(oldv.GetFloat());
    uint64_t n = pid < W.NI ? (uint64_t)newv.GetInt() : dbits(newv.GetFloat());
    W.slog.push_back({obj, pid, o, n, 0, 0, W.seq++});
    return 0;
}

static int OnRecordEvent(int32_t obj, int32_t r, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& oldv,
                         const NFIDataList::TData& newv) {
    if (ev.nOpType == RECORD_EVENT_DATA::Add || ev.nOpType == RECORD_EVENT_DATA::Del ||
        ev.nOpType == RECORD_EVENT_DATA::Cover) {  // row events: rrc bits 24-27 = 1 Add, 2 Del, 3 Cover
        if (W.bench) return 0;
        const uint32_t op = ev.nOpType == RECORD_EVENT_DATA::Add ? 1u : ev.nOpType == RECORD_EVENT_DATA::Del ? 2u : 3u;
        W.rlog.push_back({obj, (op << 24) | ((uint32_t)r << 16) | ((uint32_t)ev.nRow << 8) | (uint32_t)ev.nCol, 0, 0,
                          W.seq++});
        return 0;
    }
    if (ev.nOpType != RECORD_EVENT_DATA::Update) return 0;
    bool isint = newv.GetType() == TDATA_INT;
    if (W.bench) {
        NFCDataList lst;
        broadcast_list(obj, W.rflags[W.cls[obj] * W.NR + r], lst);
        W.bench_msgs += lst.GetCount();
        return 0;
    }
    uint64_t o = isint ? (uint64_t)oldv.GetInt() : dbits(oldv.GetFloat());
    uint64_t n = isint ? (uint64_t)newv.GetInt() : dbits(newv.GetFloat());
    uint32_t rrc = ((uint32_t)r << 16) | ((uint32_t)ev.nRow << 8) | (uint32_t)ev.nCol;
    W.rlog.push_back({obj, rrc, o, n, W.seq++});
    return 0;
}

// NFCKernelModule::GetPropertyInt / SetPropertyInt (KM:323-347, 401-425): object lookup then by-name
static int64_t GetInt(const NFGUID& self, int pid) {
    return W.pm[W.obj_of[self]]->GetPropertyInt(W.pname[pid]);
}
static double GetFloat(const NFGUID& self, int pid) {
    return W.pm[W.obj_of[self]]->GetPropertyFloat(W.pname[pid]);
}
static void SetInt(const NFGUID& self, int pid, int64_t v) {
    W.pm[W.obj_of[self]]->SetPropertyInt(W.pname[pid], v);
}
static void SetFloat(const NFGUID& self, int pid, double v) {
    W.pm[W.obj_of[self]]->SetPropertyFloat(W.pname[pid], v);
}

// the heartbeat functor registered with NFCScheduleModule::AddSchedule
static int OnHeartBeat(const NFGUID& self, const std::string& name, const float, const int nCount) {
    int kind = W.kind_of[name];
    int32_t obj = W.obj_of[self];
    if (!W.bench) W.fired.push_back({obj, kind, nCount});
    for (int i = 0; i < W.nops[kind]; i++) {
        const nfk_op& op = W.ops[kind][i];
        if (op.flags & NFK_GUARD) {
            const int64_t g = GetInt(self, (int)(op.guard & 0xFFFF));
            const int64_t h = (op.guard & NFK_GUARD_PROP) ? GetInt(self, (int)(op.guard >> 19))  // vs a property
                                                             : NFK_GUARD_KVAL(op.guard);   // or a constant
            const int c = (op.guard >> 16) & 3;
            if (!(c == NFK_GUARD_GT0 ? g > h : c == NFK_GUARD_LE0 ? g <= h : c == NFK_GUARD_NE0 ? g != h : g == h)) continue;
        }
        switch (op.code) {
        case NFK_OP_IADD_CLAMP: {
            int64_t cur = GetInt(self, op.dst);
            int64_t a = (op.flags & NFK_A_PROP) ? GetInt(self, (int)op.a) : op.a;
            int64_t lo = (op.flags & NFK_LO_PROP) ? GetInt(self, (int)op.b) : op.b;
            int64_t hi = (op.flags & NFK_HI_PROP) ? GetInt(self, (int)op.c) : op.c;
            int64_t v = (int64_t)((uint64_t)cur + (uint64_t)a);
            if (v < lo) v = lo;
            if (v > hi) v = hi;
            SetInt(self, op.dst, v);
            break;
        }
        case NFK_OP_FLERP: {
            double x = GetFloat(self, op.dst);
            double t = GetFloat(self, (int)op.a);
            double d = t - x;
            double m = d * bitsd((uint64_t)op.b);
            SetFloat(self, op.dst, x + m);
            break;
        }
        case NFK_OP_FAFFINE: {
            double x = GetFloat(self, op.dst);
            double m = x * bitsd((uint64_t)op.a);
            SetFloat(self, op.dst, m + bitsd((uint64_t)op.b));
            break;
        }
        case NFK_OP_ISET:
            SetInt(self, op.dst, (op.flags & NFK_A_PROP) ? GetInt(self, (int)op.a) : op.a);
            break;
        case NFK_OP_FSET:
            SetFloat(self, op.dst, (op.flags & NFK_A_PROP) ? GetFloat(self, (int)op.a) : bitsd((uint64_t)op.a));
            break;
        case NFK_OP_RIADD_CLAMP:
        case NFK_OP_RFAFFINE: {
            int r = op.dst >> 8, col = op.dst & 255;
            auto& R = W.rec[obj][r];
            for (int row = 0; row < R->GetRows(); row++) {
                if (!R->IsUsed(row)) continue;
                if (op.code == NFK_OP_RIADD_CLAMP) {
                    int64_t cur = R->GetInt(row, col);
                    int64_t v = (int64_t)((uint64_t)cur + (uint64_t)op.a);
                    if (v < op.b) v = op.b;
                    if (v > op.c) v = op.c;
                    R->SetInt(row, col, v);
                } else {
                    double x = R->GetFloat(row, col);
                    double m = x * bitsd((uint64_t)op.a);
                    R->SetFloat(row, col, m + bitsd((uint64_t)op.b));
                }
            }
            break;
        }
        default:
            break;
        }
    }
    return 0;
}

static std::string cstr(const uint8_t* p, int n) {
    std::string s((const char*)p, strnlen((const char*)p, n));
    return s;
}

#define GET(f, name) ([&]() { nfio_arr* _a = nfio_get(&f, name); if (!_a) { fprintf(stderr, "missing %s\n", name); exit(2);} return _a; }())

// Demonstrates NFCRecord::SetFloat (NFCRecord.cpp:278/285): `pVar->variantData = value` with a
// `const double` lvalue selects mapbox::util::variant's int64 alternative, so the float cell now
// holds a long and the next GetFloat() throws bad_variant_access.  Prints the variant index
// (mapbox which(): 0 = NFINT64, 1 = double) of the cell before and after one SetFloat.
static int repro_record_float() {
    NF_SHARE_PTR<NFIDataList> types(new NFCDataList()), tags(new NFCDataList());
    types->Add((NFINT64)0);
    types->Add(0.0);
    tags->Add(std::string("id"));
    tags->Add(std::string("charge"));
    NFCRecord R(NFGUID(1, 1), "rec", types, tags, 2);
    NFCDataList row;
    row.Add((NFINT64)5);
    row.Add(3.5);
    R.AddRow(0, row);
    int before = (int)R.GetRecordVec().at(1)->variantData.which();
    R.SetFloat(0, 1, 1.75);
    int after = (int)R.GetRecordVec().at(1)->variantData.which();
    bool threw = false;
    try {
        (void)R.GetFloat(0, 1);
    } catch (...) {
        threw = true;
    }
    printf("{\"which_before\": %d, \"which_after\": %d, \"getfloat_throws\": %s}\n", before, after,
           threw ? "true" : "false");
    fflush(stdout);
    _exit(0);
}

// The reference's module schedules (NFCScheduleModule, SM:123-216) driven by a script (see
// tests/cpp/module_sched.cpp for the format); prints what the functors see.
static int module_script(const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) return 2;
    SchedProbe sched(nullptr);
    auto cb = MODULE_SCHEDULE_FUNCTOR_PTR(new MODULE_SCHEDULE_FUNCTOR(
        [](const std::string& name, const float t, const int remain) {
            printf("fire %lld %s %.3f %d\n", (long long)g_now_ms, name.c_str(), t, remain);
            return 0;
        }));
    char op[16], name[64];
    long long t;
    while (fscanf(f, "%lld %15s", &t, op) == 2) {
        g_now_ms = t;
        std::string o(op);
        if (o == "add") {
            float ft;
            int cnt;
            if (fscanf(f, "%63s %f %d", name, &ft, &cnt) != 3) return 3;
            sched.AddSchedule(std::string(name), cb, ft, cnt);
        } else if (o == "remove") {
            if (fscanf(f, "%63s", name) != 1) return 3;
            sched.RemoveSchedule(std::string(name));
        } else if (o == "exist") {
            if (fscanf(f, "%63s", name) != 1) return 3;
            printf("exist %lld %s %d\n", (long long)g_now_ms, name, sched.ExistSchedule(std::string(name)) ? 1 : 0);
        } else if (o == "exec") {
            sched.Execute();
        } else {
            return 3;
        }
    }
    fclose(f);
    fflush(stdout);
    _exit(0);
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "--repro-record-float") == 0) return repro_record_float();
    if (argc == 3 && strcmp(argv[1], "--module-script") == 0) return module_script(argv[2]);
    bool bench = argc == 4 && strcmp(argv[1], "--bench") == 0;
    if (!bench && argc != 3) {
        fprintf(stderr, "usage: nf_ref_harness <workload.nfio> <out.nfio> | --bench <workload.nfio> <ticks>\n");
        return 2;
    }
    W.bench = bench;
    nfio_file wf;
    if (nfio_read(bench ? argv[2] : argv[1], &wf) != 0) { fprintf(stderr, "cannot read workload\n"); return 2; }
    int64_t* cfg = (int64_t*)GET(wf, "cfg")->data;
    W.N = cfg[0]; W.NI = cfg[1]; W.NF = cfg[2]; W.NC = cfg[3]; W.NK = cfg[4]; W.NR = cfg[5];
    int64_t NS = cfg[6], NT = cfg[7];
    nfio_arr* noa = nfio_get(&wf, "n_oprops");  // optional: object (NFGUID) properties
    W.NO = noa ? ((int64_t*)noa->data)[0] : 0;
    int64_t NP = W.NI + W.NF + W.NO;
    auto ptype = [&](int64_t p) { return p < W.NI ? TDATA_INT : p < W.NI + W.NF ? TDATA_FLOAT : TDATA_OBJECT; };
    if (bench) NT = std::min<int64_t>(NT, atoll(argv[3]));
    uint8_t* pnames = (uint8_t*)GET(wf, "prop_names")->data;
    uint8_t* knames = (uint8_t*)GET(wf, "kind_names")->data;
    for (int p = 0; p < NP; p++) W.pname.push_back(cstr(pnames + 32 * p, 32));
    for (int k = 0; k < W.NK; k++) {
        W.kname.push_back(cstr(knames + 32 * k, 32));
        W.kind_of[W.kname.back()] = k;
    }
    {
        const nfio_arr* oa = GET(wf, "ops");
        const int opk = nfio_ops_per_kind(oa);
        if (opk <= 0 || opk > NFK_MAX_OPS) {
            fprintf(stderr, "bad ops array\n");
            exit(2);
        }
        for (int k = 0; k < W.NK; k++)
            memcpy(W.ops[k], (const nfk_op*)oa->data + (size_t)k * opk, (size_t)opk * sizeof(nfk_op));
    }
    memcpy(W.nops, GET(wf, "n_ops")->data, W.NK * 4);
    for (int k = 0; k < W.NK; k++)
        for (int i = 0; i < W.nops[k]; i++)
            if (W.ops[k][i].code == NFK_OP_RFAFFINE) {
                fprintf(stderr, "nf_ref_harness: record f64 ops cannot run on the reference: "
                                "NFCRecord::SetFloat stores an int64 variant (see --repro-record-float)\n");
                return 3;
            }
    uint8_t* pflags = (uint8_t*)GET(wf, "prop_flags")->data;
    for (int c = 0; c < W.NC; c++) {
        NF_SHARE_PTR<NFIPropertyManager> cpm(new NFCPropertyManager(NFGUID()));
        for (int p = 0; p < NP; p++) {
            auto pr = cpm->AddProperty(NFGUID(), W.pname[p], ptype(p));
            uint8_t f = pflags[c * NP + p];
            pr->SetPublic(f & NFK_PUBLIC);
            pr->SetPrivate(f & NFK_PRIVATE);
            pr->SetUpload(f & NFK_UPLOAD);
        }
        W.class_pm.push_back(cpm);
    }
    std::vector<uint64_t*> rcells(W.NR), rused(W.NR);
    std::vector<uint8_t> rctype(W.NR * NFK_MAX_REC_COLS);
    if (W.NR > 0) {
        memcpy(W.rec_rows, GET(wf, "rec_rows")->data, W.NR * 4);
        memcpy(W.rec_cols, GET(wf, "rec_cols")->data, W.NR * 4);
        memcpy(rctype.data(), GET(wf, "rec_ctype")->data, W.NR * NFK_MAX_REC_COLS);
        uint8_t* rf = (uint8_t*)GET(wf, "rec_flags")->data;
        W.rflags.assign(rf, rf + W.NC * W.NR);
        for (int r = 0; r < W.NR; r++) {
            char nm[32];
            snprintf(nm, sizeof nm, "rec%d_cells", r);
            rcells[r] = (uint64_t*)GET(wf, nm)->data;
            snprintf(nm, sizeof nm, "rec%d_used", r);
            rused[r] = (uint64_t*)GET(wf, nm)->data;
        }
    }
    int64_t* gh = (int64_t*)GET(wf, "guid_head")->data;
    int64_t* gd = (int64_t*)GET(wf, "guid_data")->data;
    int32_t* sc = (int32_t*)GET(wf, "scene")->data;
    int32_t* gr = (int32_t*)GET(wf, "group")->data;
    uint8_t* cl = (uint8_t*)GET(wf, "cls")->data;
    uint8_t* ip = (uint8_t*)GET(wf, "is_player")->data;
    int64_t* init_i = (int64_t*)GET(wf, "init_i")->data;
    double* init_f = (double*)GET(wf, "init_f")->data;
    int64_t* init_oh = W.NO ? (int64_t*)GET(wf, "init_oh")->data : nullptr;
    int64_t* init_od = W.NO ? (int64_t*)GET(wf, "init_od")->data : nullptr;
    W.scene.assign(sc, sc + W.N);
    W.group.assign(gr, gr + W.N);
    W.cls.assign(cl, cl + W.N);
    W.isplayer.assign(ip, ip + W.N);

    // objects: NFCKernelModule::CreateObject (KM:101-271) property part + scene group maps; an
    // object with born[o] >= 0 is created in frame born[o]'s window (CreateObject after start)
    nfio_arr* ba = nfio_get(&wf, "born");
    int32_t* born = ba ? (int32_t*)ba->data : nullptr;
    W.alive.assign(W.N, 0);
    W.pm.resize(W.N);
    W.rec.resize(W.N);
    for (int64_t o = 0; o < W.N; o++) W.id.push_back(NFGUID(gh[o], gd[o]));
    auto create = [&](int64_t o) {
        const NFGUID id = W.id[o];
        W.obj_of[id] = (int)o;
        W.alive[o] = 1;
        NF_SHARE_PTR<NFIPropertyManager> pm(new NFCPropertyManager(id));
        for (int p = 0; p < NP; p++) {
            auto tmpl = W.class_pm[W.cls[o]]->GetElement(W.pname[p]);
            auto pr = pm->AddProperty(id, W.pname[p], ptype(p));
            pr->SetPublic(tmpl->GetPublic());
            pr->SetPrivate(tmpl->GetPrivate());
            pr->SetUpload(tmpl->GetUpload());
            if (p < W.NI) pr->SetInt(init_i[p * W.N + o]);
            else if (p < W.NI + W.NF) pr->SetFloat(init_f[(p - W.NI) * W.N + o]);
            else pr->SetObject(NFGUID(init_oh[(p - W.NI - W.NF) * W.N + o], init_od[(p - W.NI - W.NF) * W.N + o]));
            int32_t obj = (int32_t)o, pid = p;
            pr->RegisterCallback(PROPERTY_EVENT_FUNCTOR_PTR(new PROPERTY_EVENT_FUNCTOR(
                [obj, pid](const NFGUID&, const std::string&, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                    return OnPropertyEvent(obj, pid, a, b);
                })));
        }
        W.pm[o] = pm;
        std::vector<NF_SHARE_PTR<NFIRecord>> recs;
        for (int r = 0; r < W.NR; r++) {
            NF_SHARE_PTR<NFIDataList> types(new NFCDataList());
            NF_SHARE_PTR<NFIDataList> tags(new NFCDataList());
            for (int c = 0; c < W.rec_cols[r]; c++) {
                if (rctype[r * NFK_MAX_REC_COLS + c] == 0) types->Add((NFINT64)0);
                else types->Add(0.0);
                tags->Add(std::string("c") + std::to_string(c));
            }
            NF_SHARE_PTR<NFIRecord> R(new NFCRecord(id, "rec" + std::to_string(r), types, tags, W.rec_rows[r]));
            for (int row = 0; row < W.rec_rows[r]; row++) {
                if (!((rused[r][o] >> row) & 1)) continue;
                NFCDataList rowv;
                for (int c = 0; c < W.rec_cols[r]; c++) {
                    uint64_t b = rcells[r][((int64_t)o * W.rec_cols[r] + c) * W.rec_rows[r] + row];
                    if (rctype[r * NFK_MAX_REC_COLS + c] == 0) rowv.Add((NFINT64)b);
                    else rowv.Add(bitsd(b));
                }
                R->AddRow(row, rowv);
            }
            int32_t obj = (int32_t)o;
            R->AddRecordHook(RECORD_EVENT_FUNCTOR_PTR(new RECORD_EVENT_FUNCTOR(
                [obj, r](const NFGUID&, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                    return OnRecordEvent(obj, r, ev, a, b);
                })));
            recs.push_back(R);
        }
        W.rec[o] = recs;
        // NFCSceneInfo::AddObjectToGroup (NFISceneAOIModule.h) — the group's player / other maps
        auto& si = W.scenes[W.scene[o]];
        if (!si) si = NF_SHARE_PTR<NFCSceneInfo>(new NFCSceneInfo(W.scene[o]));
        if (!si->GetElement(W.group[o]))
            si->AddElement(W.group[o], NF_SHARE_PTR<NFCSceneGroupInfo>(new NFCSceneGroupInfo(W.scene[o], W.group[o])));
        si->AddObjectToGroup(W.group[o], id, W.isplayer[o] != 0);
    };
    for (int64_t o = 0; o < W.N; o++)
        if (!born || born[o] < 0) create(o);
    nfio_arr* dta = nfio_get(&wf, "d_tick");
    const int64_t ND = dta ? (int64_t)dta->shape[0] : 0;
    int32_t* d_tick = ND ? (int32_t*)dta->data : nullptr;
    int32_t* d_obj = ND ? (int32_t*)GET(wf, "d_obj")->data : nullptr;
    int64_t di = 0;

    SchedProbe sched(nullptr);
    auto hb = OBJECT_SCHEDULE_FUNCTOR_PTR(new OBJECT_SCHEDULE_FUNCTOR(OnHeartBeat));
    int32_t* s_obj = (int32_t*)GET(wf, "s_obj")->data;
    int32_t* s_kind = (int32_t*)GET(wf, "s_kind")->data;
    float* s_interval = (float*)GET(wf, "s_interval")->data;
    int32_t* s_count = (int32_t*)GET(wf, "s_count")->data;
    int64_t* s_time = (int64_t*)GET(wf, "s_time")->data;
    for (int64_t i = 0; i < NS; i++) {
        g_now_ms = s_time[i];
        sched.AddSchedule(W.id[s_obj[i]], W.kname[s_kind[i]], hb, s_interval[i], s_count[i]);
    }
    int64_t* tick_time = (int64_t*)GET(wf, "tick_time")->data;
    nfio_arr* xa = GET(wf, "x_tick");
    int64_t NX = (int64_t)xa->shape[0];
    int32_t* x_tick = (int32_t*)xa->data;
    int32_t* x_obj = (int32_t*)GET(wf, "x_obj")->data;
    int32_t* x_pid = (int32_t*)GET(wf, "x_pid")->data;
    uint64_t* x_bits = (uint64_t*)GET(wf, "x_bits")->data;
    nfio_arr* xma = nfio_get(&wf, "x_mode");  // optional: 1 = SetProperty(p, GetProperty(p) + delta)
    uint8_t* x_mode = xma ? (uint8_t*)xma->data : nullptr;
    uint64_t* x_bits_h = W.NO ? (uint64_t*)GET(wf, "x_bits_h")->data : nullptr;  // SetPropertyObject: head
    nfio_arr* rta = nfio_get(&wf, "r_tick");  // optional: SetRecordInt calls between frames
    const int64_t NRS = rta ? (int64_t)rta->shape[0] : 0;
    int32_t* r_tick = NRS ? (int32_t*)rta->data : nullptr;
    int32_t* r_obj = NRS ? (int32_t*)GET(wf, "r_obj")->data : nullptr;
    int32_t* r_rec = NRS ? (int32_t*)GET(wf, "r_rec")->data : nullptr;
    int32_t* r_row = NRS ? (int32_t*)GET(wf, "r_row")->data : nullptr;
    int32_t* r_col = NRS ? (int32_t*)GET(wf, "r_col")->data : nullptr;
    uint64_t* r_bits = NRS ? (uint64_t*)GET(wf, "r_bits")->data : nullptr;
    // optional record row operations in the same stream: r_op 1 AddRow(r_row, r_vals), 2 Remove(r_row),
    // 3 ClearRecord (KM:492 -> NFCRecord::Clear)
    nfio_arr* roa = NRS ? nfio_get(&wf, "r_op") : nullptr;
    uint8_t* r_op = roa ? (uint8_t*)roa->data : nullptr;
    uint64_t* r_vals = roa ? (uint64_t*)GET(wf, "r_vals")->data : nullptr;
    int64_t ri = 0;
    nfio_arr* ha = GET(wf, "h_tick");
    int64_t NH = (int64_t)ha->shape[0];
    int32_t* h_tick = (int32_t*)ha->data;
    int32_t* h_op = (int32_t*)GET(wf, "h_op")->data;
    int32_t* h_obj = (int32_t*)GET(wf, "h_obj")->data;
    int32_t* h_kind = (int32_t*)GET(wf, "h_kind")->data;
    float* h_interval = (float*)GET(wf, "h_interval")->data;
    int32_t* h_count = (int32_t*)GET(wf, "h_count")->data;
    int64_t* h_time = (int64_t*)GET(wf, "h_time")->data;

    // canonical rank (scene, group, guid) of the live objects; recomputed after SwitchScene,
    // CreateObject and DestroyObject
    std::vector<int32_t> sorted;
    std::vector<int64_t> orank(W.N);
    auto build_order = [&]() {
        sorted.clear();
        for (int64_t i = 0; i < W.N; i++)
            if (W.alive[i]) sorted.push_back((int32_t)i);
        std::sort(sorted.begin(), sorted.end(), [](int32_t a, int32_t b) {
            if (W.scene[a] != W.scene[b]) return W.scene[a] < W.scene[b];
            if (W.group[a] != W.group[b]) return W.group[a] < W.group[b];
            return W.id[a] < W.id[b];
        });
        for (int64_t i = 0; i < W.N; i++) orank[i] = -1;
        for (size_t i = 0; i < sorted.size(); i++) orank[sorted[i]] = (int64_t)i;
    };
    build_order();

    // SwitchScene calls (optional) and the property ids they write
    int32_t pid_scene = -1, pid_group = -1, pid_x = -1, pid_y = -1, pid_z = -1;
    if (nfio_arr* spa = nfio_get(&wf, "scene_props")) {
        int32_t* sp = (int32_t*)spa->data;
        pid_scene = sp[0]; pid_group = sp[1]; pid_x = sp[2]; pid_y = sp[3]; pid_z = sp[4];
    }
    nfio_arr* swa = nfio_get(&wf, "sw_tick");
    const int64_t NSW = swa ? (int64_t)swa->shape[0] : 0;
    int32_t *sw_tick = nullptr, *sw_obj = nullptr, *sw_scene = nullptr, *sw_group = nullptr;
    float *sw_x = nullptr, *sw_y = nullptr, *sw_z = nullptr;
    if (NSW) {
        sw_tick = (int32_t*)swa->data;
        sw_obj = (int32_t*)GET(wf, "sw_obj")->data;
        sw_scene = (int32_t*)GET(wf, "sw_scene")->data;
        sw_group = (int32_t*)GET(wf, "sw_group")->data;
        sw_x = (float*)GET(wf, "sw_x")->data;
        sw_y = (float*)GET(wf, "sw_y")->data;
        sw_z = (float*)GET(wf, "sw_z")->data;
    }
    int64_t swi = 0;

    nfio_writer w;
    if (!bench && nfio_wopen(&w, argv[2]) != 0) { fprintf(stderr, "cannot open output\n"); return 2; }
    int64_t xi = 0, hi = 0;
    double tick_seconds = 0;
    int64_t total_fired = 0;
    for (int t = 0; t < NT; t++) {
        W.slog.clear();
        W.rlog.clear();
        W.fired.clear();
        W.seq = 0;
        // NFCKernelModule::SwitchScene (KM:901-951), restated over the reference's NFCSceneInfo
        // group maps and property manager; made first in the window.  The target group is
        // created on demand (NFCKernelModule::RequestGroupScene).
        bool relayout = false;
        // CreateObject after start (KM:101-271), the window's first calls
        if (born)
            for (int64_t o = 0; o < W.N; o++)
                if (born[o] == t) {
                    create(o);
                    relayout = true;
                }
        while (swi < NSW && sw_tick[swi] == t) {
            const int32_t o = sw_obj[swi];
            const NFGUID self = W.id[o];
            const int ns = sw_scene[swi] < 0 ? W.scene[o] : sw_scene[swi];
            const int ng = sw_scene[swi] < 0 ? W.group[o] : sw_group[swi];
            auto& nsi = W.scenes[ns];
            if (!nsi) nsi = NF_SHARE_PTR<NFCSceneInfo>(new NFCSceneInfo(ns));
            if (!nsi->GetElement(ng)) nsi->AddElement(ng, NF_SHARE_PTR<NFCSceneGroupInfo>(new NFCSceneGroupInfo(ns, ng)));
            W.scenes[W.scene[o]]->RemoveObjectFromGroup(W.group[o], self, true);
            if (ns != W.scene[o]) {
                if (pid_group >= 0) SetInt(self, pid_group, 0);
                if (pid_scene >= 0) SetInt(self, pid_scene, ns);
            }
            if (pid_x >= 0) SetFloat(self, pid_x, (double)sw_x[swi]);
            if (pid_y >= 0) SetFloat(self, pid_y, (double)sw_y[swi]);
            if (pid_z >= 0) SetFloat(self, pid_z, (double)sw_z[swi]);
            if (pid_group >= 0) SetInt(self, pid_group, ng);
            nsi->AddObjectToGroup(ng, self, true);
            relayout |= ns != W.scene[o] || ng != W.group[o];
            W.scene[o] = ns;
            W.group[o] = ng;
            swi++;
        }
        if (relayout) build_order();
        while (hi < NH && h_tick[hi] == t) {
            NFGUID self = W.id[h_obj[hi]];
            if (h_op[hi] == 1) {
                g_now_ms = h_time[hi];
                sched.AddSchedule(self, W.kname[h_kind[hi]], hb, h_interval[hi], h_count[hi]);
            } else if (h_op[hi] == 2) {
                sched.RemoveSchedule(self, W.kname[h_kind[hi]]);
            } else if (h_op[hi] == 3) {
                sched.RemoveSchedule(self);
            }
            hi++;
        }
        auto t0 = std::chrono::steady_clock::now();
        while (xi < NX && x_tick[xi] == t) {
            NFGUID self = W.id[x_obj[xi]];
            const bool rmw = x_mode && x_mode[xi];  // game logic: Set(p, Get(p) + delta) (KM:401 then KM:323)
            if (x_pid[xi] >= W.NI + W.NF)  // NFCKernelModule::SetPropertyObject (KM:362) -> NFCProperty::SetObject
                W.pm[W.obj_of[self]]->SetPropertyObject(W.pname[x_pid[xi]], NFGUID((int64_t)x_bits_h[xi], (int64_t)x_bits[xi]));
            else if (x_pid[xi] < W.NI)
                SetInt(self, x_pid[xi], rmw ? (int64_t)((uint64_t)GetInt(self, x_pid[xi]) + x_bits[xi]) : (int64_t)x_bits[xi]);
            else
                SetFloat(self, x_pid[xi], rmw ? GetFloat(self, x_pid[xi]) + bitsd(x_bits[xi]) : bitsd(x_bits[xi]));
            xi++;
        }
        // SetRecordInt (KM:505 -> NFCObject -> NFCRecord::SetInt, RC:182: valid position, int
        // column, used row, changed value; the record hook fires) made before this Execute
        while (ri < NRS && r_tick[ri] == t) {
            const int32_t o = r_obj[ri], r = r_rec[ri];
            const int op = r_op ? r_op[ri] : 0;
            if (op && W.alive[o]) {
                auto& R = W.rec[o][r];
                if (op == 1) {  // NFCRecord::AddRow(nRow, var) (RC:111)
                    NFCDataList rowv;
                    for (int c = 0; c < W.rec_cols[r]; c++) {
                        const uint64_t b = r_vals[ri * NFK_MAX_REC_COLS + c];
                        if (rctype[r * NFK_MAX_REC_COLS + c] == 0) rowv.Add((NFINT64)b);
                        else rowv.Add(bitsd(b));
                    }
                    R->AddRow(r_row[ri], rowv);
                } else if (op == 2) {
                    R->Remove(r_row[ri]);  // RC:1086
                } else if (op == 3) {
                    R->Clear();  // NFCKernelModule::ClearRecord (KM:492) -> RC:1109
                }
                ri++;
                continue;
            }
            if (!op && W.alive[o]) {
                if (rctype[r * NFK_MAX_REC_COLS + r_col[ri]]) {
                    fprintf(stderr, "nf_ref_harness: SetRecordFloat cannot run on the reference: "
                                    "NFCRecord::SetFloat stores an int64 variant (see --repro-record-float)\n");
                    return 3;
                }
                W.rec[o][r]->SetInt(r_row[ri], r_col[ri], (NFINT64)r_bits[ri]);
            }
            ri++;
        }
        // DestroyObject (KM:273-308), the window's last calls: RemoveObjectFromGroup, then the
        // reference scheduler's RemoveSchedule(self) (SM:240); the object's events go with it
        {
            bool destroyed = false;
            while (di < ND && d_tick[di] == t) {
                const int32_t o = d_obj[di++];
                W.scenes[W.scene[o]]->RemoveObjectFromGroup(W.group[o], W.id[o], W.isplayer[o] != 0);
                sched.RemoveSchedule(W.id[o]);
                W.obj_of.erase(W.id[o]);
                W.alive[o] = 0;
                destroyed = true;
            }
            if (destroyed) {
                W.slog.erase(std::remove_if(W.slog.begin(), W.slog.end(), [](const SetEv& e) { return !W.alive[e.obj]; }),
                             W.slog.end());
                W.rlog.erase(std::remove_if(W.rlog.begin(), W.rlog.end(), [](const RSetEv& e) { return !W.alive[e.obj]; }),
                             W.rlog.end());
                build_order();
            }
        }
        g_now_ms = tick_time[t];
        sched.Execute();
        auto t1 = std::chrono::steady_clock::now();
        tick_seconds += std::chrono::duration<double>(t1 - t0).count();
        if (bench) continue;

        // coalesce per (object, property) and canonicalise
        std::stable_sort(W.slog.begin(), W.slog.end(), [&](const SetEv& a, const SetEv& b) {
            if (orank[a.obj] != orank[b.obj]) return orank[a.obj] < orank[b.obj];
            return a.pid < b.pid;
        });
        std::vector<int32_t> ev_obj, ev_pid;
        std::vector<uint64_t> ev_old, ev_new, ev_oldh, ev_newh;
        for (size_t i = 0; i < W.slog.size();) {
            size_t j = i;
            while (j < W.slog.size() && W.slog[j].obj == W.slog[i].obj && W.slog[j].pid == W.slog[i].pid) j++;
            if (W.slog[i].o != W.slog[j - 1].n || W.slog[i].oh != W.slog[j - 1].nh) {
                ev_obj.push_back(W.slog[i].obj);
                ev_pid.push_back(W.slog[i].pid);
                ev_old.push_back(W.slog[i].o);
                ev_new.push_back(W.slog[j - 1].n);
                ev_oldh.push_back(W.slog[i].oh);
                ev_newh.push_back(W.slog[j - 1].nh);
            }
            i = j;
        }
        // per object, per record: row events in call order, then cell Updates by (row, col)
        std::stable_sort(W.rlog.begin(), W.rlog.end(), [&](const RSetEv& a, const RSetEv& b) {
            if (orank[a.obj] != orank[b.obj]) return orank[a.obj] < orank[b.obj];
            const uint32_t ra = (a.rrc >> 16) & 0xFF, rb = (b.rrc >> 16) & 0xFF;
            if (ra != rb) return ra < rb;
            const bool ua = (a.rrc >> 24) == 0, ub = (b.rrc >> 24) == 0;
            if (ua != ub) return ub;
            return ua ? a.rrc < b.rrc : false;
        });
        std::vector<int32_t> re_obj;
        std::vector<uint32_t> re_rrc;
        std::vector<uint64_t> re_old, re_new;
        for (size_t i = 0; i < W.rlog.size();) {
            size_t j = i + 1;
            const bool upd = (W.rlog[i].rrc >> 24) == 0;  // row events are not coalesced
            if (upd)
                while (j < W.rlog.size() && W.rlog[j].obj == W.rlog[i].obj && W.rlog[j].rrc == W.rlog[i].rrc) j++;
            if (W.rlog[i].o != W.rlog[j - 1].n || !upd) {
                re_obj.push_back(W.rlog[i].obj);
                re_rrc.push_back(W.rlog[i].rrc);
                re_old.push_back(W.rlog[i].o);
                re_new.push_back(W.rlog[j - 1].n);
            }
            i = j;
        }
        std::stable_sort(W.fired.begin(), W.fired.end(), [&](const Fired& a, const Fired& b) {
            if (orank[a.obj] != orank[b.obj]) return orank[a.obj] < orank[b.obj];
            return a.kind < b.kind;
        });
        std::vector<int32_t> fo, fk, fr;
        for (auto& f : W.fired) { fo.push_back(f.obj); fk.push_back(f.kind); fr.push_back(f.rem); }
        // fan-out lists
        std::vector<uint32_t> moff;
        std::vector<int32_t> mr;
        size_t ne = ev_obj.size(), nre = re_obj.size();
        for (size_t e = 0; e < ne + nre; e++) {
            moff.push_back((uint32_t)mr.size());
            int32_t o = e < ne ? ev_obj[e] : re_obj[e - ne];
            uint8_t fl = e < ne ? prop_flags(o, ev_pid[e]) : W.rflags[W.cls[o] * W.NR + ((re_rrc[e - ne] >> 16) & 0xFF)];
            NFCDataList lst;
            broadcast_list(o, fl, lst);
            for (int i = 0; i < lst.GetCount(); i++) mr.push_back(W.obj_of[lst.Object(i)]);
        }
        moff.push_back((uint32_t)mr.size());
        char nm[32];
#define PUT(pfx, s, code, vec, es) snprintf(nm, sizeof nm, "%s_t%d_%s", pfx, t, s); nfio_put1(&w, nm, code, vec.data(), vec.size(), es);
        PUT("ev", "obj", NFIO_I32, ev_obj, 4);
        PUT("ev", "pid", NFIO_I32, ev_pid, 4);
        PUT("ev", "old", NFIO_U64, ev_old, 8);
        PUT("ev", "new", NFIO_U64, ev_new, 8);
        if (W.NO) {
            PUT("ev", "oldh", NFIO_U64, ev_oldh, 8);
            PUT("ev", "newh", NFIO_U64, ev_newh, 8);
        }
        PUT("re", "obj", NFIO_I32, re_obj, 4);
        PUT("re", "rrc", NFIO_U32, re_rrc, 4);
        PUT("re", "old", NFIO_U64, re_old, 8);
        PUT("re", "new", NFIO_U64, re_new, 8);
        PUT("fi", "obj", NFIO_I32, fo, 4);
        PUT("fi", "kind", NFIO_I32, fk, 4);
        PUT("fi", "rem", NFIO_I32, fr, 4);
        PUT("mo", "off", NFIO_U32, moff, 4);
        PUT("mr", "obj", NFIO_I32, mr, 4);
        total_fired += (int64_t)fo.size();
    }
    if (bench) {
        printf("{\"entities\": %lld, \"ticks\": %lld, \"seconds\": %.6f, \"entity_ticks_per_s\": %.3f, \"msgs\": %lld}\n",
               (long long)W.N, (long long)NT, tick_seconds, (double)W.N * NT / tick_seconds, (long long)W.bench_msgs);
        fflush(stdout);
        _exit(0);  // skip static destructors: NFMemoryCounter's static map dies before our objects
    }
    // final state
    std::vector<int64_t> fi(W.NI * W.N);
    std::vector<double> ff(W.NF * W.N);
    for (int64_t o = 0; o < W.N; o++) {
        if (!W.alive[o]) continue;  // objects no longer in the world read 0
        for (int p = 0; p < W.NI; p++) fi[p * W.N + o] = W.pm[o]->GetPropertyInt(W.pname[p]);
        for (int p = 0; p < W.NF; p++) ff[p * W.N + o] = W.pm[o]->GetPropertyFloat(W.pname[W.NI + p]);
    }
    uint64_t sh[2] = {(uint64_t)W.NI, (uint64_t)W.N};
    nfio_put(&w, "final_i", NFIO_I64, 2, sh, fi.data(), fi.size() * 8);
    uint64_t sf[2] = {(uint64_t)W.NF, (uint64_t)W.N};
    nfio_put(&w, "final_f", NFIO_F64, 2, sf, ff.data(), ff.size() * 8);
    if (W.NO) {
        std::vector<int64_t> foh(W.NO * W.N, 0), fod(W.NO * W.N, 0);
        for (int64_t o = 0; o < W.N; o++) {
            if (!W.alive[o]) continue;
            for (int p = 0; p < W.NO; p++) {
                const NFGUID g = W.pm[o]->GetPropertyObject(W.pname[W.NI + W.NF + p]);
                foh[p * W.N + o] = g.nHead64;
                fod[p * W.N + o] = g.nData64;
            }
        }
        uint64_t so[2] = {(uint64_t)W.NO, (uint64_t)W.N};
        nfio_put(&w, "final_oh", NFIO_I64, 2, so, foh.data(), foh.size() * 8);
        nfio_put(&w, "final_od", NFIO_I64, 2, so, fod.data(), fod.size() * 8);
    }
    for (int r = 0; r < W.NR; r++) {
        std::vector<uint64_t> cells((size_t)W.N * W.rec_cols[r] * W.rec_rows[r]);
        for (int64_t o = 0; o < W.N; o++)
            for (int c = 0; c < W.rec_cols[r] && W.alive[o]; c++)
                for (int row = 0; row < W.rec_rows[r]; row++) {
                    auto& R = W.rec[o][r];
                    uint64_t b = rcells[r][((int64_t)o * W.rec_cols[r] + c) * W.rec_rows[r] + row];
                    if (R->IsUsed(row)) {
                        b = rctype[r * NFK_MAX_REC_COLS + c] == 0 ? (uint64_t)R->GetInt(row, c) : dbits(R->GetFloat(row, c));
                    } else if (auto& pv = R->GetRecordVec().at((size_t)row * W.rec_cols[r] + c)) {
                        // a row used once and removed keeps its cells (NFCRecord::Remove, RC:1086)
                        b = rctype[r * NFK_MAX_REC_COLS + c] == 0 ? (uint64_t)pv->GetInt() : dbits(pv->GetFloat());
                    }
                    cells[((size_t)o * W.rec_cols[r] + c) * W.rec_rows[r] + row] = b;
                }
        char nm[32];
        snprintf(nm, sizeof nm, "final_rec%d", r);
        uint64_t sr[3] = {(uint64_t)W.N, (uint64_t)W.rec_cols[r], (uint64_t)W.rec_rows[r]};
        nfio_put(&w, nm, NFIO_U64, 3, sr, cells.data(), cells.size() * 8);
    }
    std::vector<int64_t> sn(W.NK * W.N, 0);
    std::vector<int32_t> srm(W.NK * W.N, 0);
    std::vector<uint8_t> sp(W.NK * W.N, 0);
    for (int k = 0; k < W.NK; k++)
        for (int64_t o = 0; o < W.N; o++) {
            int64_t nx;
            int32_t rm;
            if (sched.Probe(W.id[o], W.kname[k], &nx, &rm)) {
                sp[k * W.N + o] = 1;
                sn[k * W.N + o] = nx;
                srm[k * W.N + o] = rm;
            }
        }
    uint64_t ss[2] = {(uint64_t)W.NK, (uint64_t)W.N};
    nfio_put(&w, "final_s_next", NFIO_I64, 2, ss, sn.data(), sn.size() * 8);
    nfio_put(&w, "final_s_remain", NFIO_I32, 2, ss, srm.data(), srm.size() * 4);
    nfio_put(&w, "final_s_present", NFIO_U8, 2, ss, sp.data(), sp.size());
    nfio_wclose(&w);
    (void)total_fired;
    fflush(stdout);
    _exit(0);  // skip static destructors: NFMemoryCounter's static map dies before our objects
}
