// plugin_shard_replay.cpp — scene shards through the C++ plugin (include/NFGPUKernelModule.hpp +
// include/NFGPUSceneShard.hpp), no Python: R ranks as threads of one process on the one GPU, each an
// NFGPUKernelModule over its own world owning a contiguous range of the workload's scenes
// (shard.py scene_ranges), joined by the host stand-in transport.  Each frame: SwitchScene calls
// (a target scene another rank owns queues a departure), MigrateNow (the exchange), then the
// schedule / SetProperty / SetRecord calls of the objects each rank holds, then Execute.  What the
// callbacks see is written per rank with global object indices, to be compared with the
// single-world oracle split by owner (tests/test_shard_cpp.py).
//
// usage: plugin_shard_replay <workload.nfio> <out_dir> <ranks> [async]
//   async 1: no MigrateNow — the departures move through Execute's own asynchronous exchange (tickets
//   gathered at the end of an Execute, rows moved at the start of the next), so an entity ticks on its
//   source shard for one more frame after its SwitchScene; calls on entities in transit are skipped
//   (the test compares the heartbeat functors: schedules travel with the rows)
//   async 2: as 1, and every window also writes ATK_VALUE (no program writes it) of every entity in
//   transit on its source shard — after its SwitchScene, and after the Execute that started its ticket
//   gather — and writes the last value written per object as "atk_expect" (-1: none): the owner's final
//   ATK_VALUE must equal it (the writes travel with the row)
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "NFGPUKernelModule.hpp"
#include "NFGPUSceneShard.hpp"
#include "../../oracle/nfio.h"

using namespace nfgpu;

static std::string cstr(const uint8_t* p) { return std::string((const char*)p, strnlen((const char*)p, 32)); }

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) return 2;
    const bool async = argc == 5 && atoi(argv[4]) != 0;
    const bool transit_writes = argc == 5 && atoi(argv[4]) == 2;
    nfio_file wf;
    if (nfio_read(argv[1], &wf)) return 2;
    const std::string out_dir = argv[2];
    const int R = atoi(argv[3]);
    auto A = [&](const char* n) {
        nfio_arr* a = nfio_get(&wf, n);
        if (!a) {
            fprintf(stderr, "missing %s\n", n);
            exit(2);
        }
        return a;
    };
    int64_t* cfg = (int64_t*)A("cfg")->data;
    const int64_t N = cfg[0], NI = cfg[1], NF = cfg[2], NC = cfg[3], NK = cfg[4], NR = cfg[5], NS = cfg[6], NT = cfg[7];
    const int64_t NP = NI + NF;
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    uint8_t* pflags = (uint8_t*)A("prop_flags")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    const int OPK = nfio_ops_per_kind(A("ops"));  // ops per kind in the file
    int32_t* nops = (int32_t*)A("n_ops")->data;
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) pname[p] = cstr(pnames + 32 * p);
    for (int k = 0; k < NK; k++) kname[k] = cstr(knames + 32 * k);
    int64_t* gh = (int64_t*)A("guid_head")->data;
    int64_t* gd = (int64_t*)A("guid_data")->data;
    int32_t* sc = (int32_t*)A("scene")->data;
    int32_t* gr = (int32_t*)A("group")->data;
    uint8_t* cl = (uint8_t*)A("cls")->data;
    int64_t* ii = (int64_t*)A("init_i")->data;
    double* ff = (double*)A("init_f")->data;
    std::map<NFGUID, int> glob;
    for (int64_t o = 0; o < N; o++) glob[NFGUID(gh[o], gd[o])] = (int)o;
    // contiguous scene ranges (shard.py scene_ranges)
    std::set<int> scenes(sc, sc + N);
    std::vector<int> sl(scenes.begin(), scenes.end());
    const int per = ((int)sl.size() + R - 1) / R;
    std::map<int, int> owner_of;
    for (size_t i = 0; i < sl.size(); i++) owner_of[sl[i]] = std::min((int)i / per, R - 1);
    auto owner = [owner_of](int s) {
        auto it = owner_of.upper_bound(s);
        return it == owner_of.begin() ? owner_of.begin()->second : std::prev(it)->second;
    };
    int64_t* tick_time = (int64_t*)A("tick_time")->data;
    nfio_arr* xa = A("x_tick");
    const int64_t NX = (int64_t)xa->shape[0];
    int32_t* x_tick = (int32_t*)xa->data;
    int32_t* x_obj = (int32_t*)A("x_obj")->data;
    int32_t* x_pid = (int32_t*)A("x_pid")->data;
    uint64_t* x_bits = (uint64_t*)A("x_bits")->data;
    nfio_arr* ha = A("h_tick");
    const int64_t NH = (int64_t)ha->shape[0];
    int32_t* h_tick = (int32_t*)ha->data;
    int32_t* h_op = (int32_t*)A("h_op")->data;
    int32_t* h_obj = (int32_t*)A("h_obj")->data;
    int32_t* h_kind = (int32_t*)A("h_kind")->data;
    float* h_int = (float*)A("h_interval")->data;
    int32_t* h_cnt = (int32_t*)A("h_count")->data;
    int64_t* h_time = (int64_t*)A("h_time")->data;
    nfio_arr* swa = nfio_get(&wf, "sw_tick");
    const int64_t NW = swa ? (int64_t)swa->shape[0] : 0;
    int32_t* sw_tick = NW ? (int32_t*)swa->data : nullptr;
    int32_t* sw_obj = NW ? (int32_t*)A("sw_obj")->data : nullptr;
    int32_t* sw_scene = NW ? (int32_t*)A("sw_scene")->data : nullptr;
    int32_t* sw_group = NW ? (int32_t*)A("sw_group")->data : nullptr;
    float* sw_x = NW ? (float*)A("sw_x")->data : nullptr;
    float* sw_y = NW ? (float*)A("sw_y")->data : nullptr;
    float* sw_z = NW ? (float*)A("sw_z")->data : nullptr;
    int32_t* s_obj = (int32_t*)A("s_obj")->data;
    int32_t* s_kind = (int32_t*)A("s_kind")->data;
    float* s_int = (float*)A("s_interval")->data;
    int32_t* s_cnt = (int32_t*)A("s_count")->data;
    int64_t* s_time = (int64_t*)A("s_time")->data;

    auto shared = HostTransport::MakeShared(R);
    std::vector<int> rc(R, 0);
    std::vector<int64_t> atk_expect(N, -1);  // (async 2; objects are written by one rank at a time)
    auto rank_main = [&](int r) {
        int64_t now = 0;
        HostTransport t(shared, r, DeviceRowMemory());
        NFGPUKernelModule km((int)N);
        km.SetTimeSource([&now] { return now; });
        for (int p = 0; p < NP; p++) km.AddProperty(pname[p], p < NI ? TDATA_INT : TDATA_FLOAT);
        for (int c = 0; c < NC; c++) {
            km.AddClass(cname[c]);
            for (int p = 0; p < NP; p++) {
                const uint8_t f = pflags[c * NP + p];
                km.SetPropertyFlags(cname[c], pname[p], f & NFK_PUBLIC, f & NFK_PRIVATE, f & NFK_UPLOAD);
            }
        }
        for (int q = 0; q < NR; q++) {
            const int32_t rows = ((int32_t*)A("rec_rows")->data)[q], cols = ((int32_t*)A("rec_cols")->data)[q];
            std::vector<TDATA_TYPE> ty;
            for (int c = 0; c < cols; c++)
                ty.push_back(((uint8_t*)A("rec_ctype")->data)[q * NFK_MAX_REC_COLS + c] ? TDATA_FLOAT : TDATA_INT);
            const std::string rn = "rec" + std::to_string(q);
            km.AddRecord(rn, rows, ty);
            for (int c = 0; c < NC; c++) {
                const uint8_t f = ((uint8_t*)A("rec_flags")->data)[c * NR + q];
                km.SetRecordFlags(cname[c], rn, f & NFK_PUBLIC, f & NFK_PRIVATE, f & NFK_UPLOAD);
            }
        }
        for (int k = 0; k < NK; k++)
            km.AddHeartBeatProgram(kname[k], std::vector<nfk_op>(ops + k * OPK, ops + k * OPK + nops[k]));
        km.Init();
        for (int s : sl)
            if (owner(s) == r) km.CreateScene(s);
        for (int64_t o = 0; o < N; o++) {
            if (owner(sc[o]) != r) continue;
            std::map<std::string, TData> init;
            for (int p = 0; p < NP; p++) {
                TData v;
                v.type = p < NI ? TDATA_INT : TDATA_FLOAT;
                if (p < NI) v.i = ii[p * N + o];
                else v.f = ff[(p - NI) * N + o];
                init[pname[p]] = v;
            }
            km.CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], init);
            for (int q = 0; q < NR; q++) {
                char nm[32];
                const int32_t rows = ((int32_t*)A("rec_rows")->data)[q], cols = ((int32_t*)A("rec_cols")->data)[q];
                snprintf(nm, sizeof nm, "rec%d_cells", q);
                const uint64_t* cells = (const uint64_t*)A(nm)->data + (size_t)o * cols * rows;
                snprintf(nm, sizeof nm, "rec%d_used", q);
                const uint64_t used = ((const uint64_t*)A(nm)->data)[o];
                km.SetCreationRecord(NFGUID(gh[o], gd[o]), "rec" + std::to_string(q), used,
                                     std::vector<uint64_t>(cells, cells + (size_t)cols * rows));
            }
        }
        km.AfterInit();
        int32_t pid_scene = km.PropertyId("SceneID"), pid_group = km.PropertyId("GroupID");
        SceneShard shard(km.World(), &t, owner, pid_scene, pid_group, km.PropertyId("X"), km.PropertyId("Y"),
                         km.PropertyId("Z"));
        km.AttachShard(&shard);
        std::vector<int32_t> ev_obj, ev_pid, re_obj, fi_obj, fi_kind, fi_rem, mr;
        std::vector<uint32_t> re_rrc, moff;
        std::vector<uint64_t> ev_old, ev_new, re_old, re_new;
        km.RegisterCommonPropertyEvent([&](const NFGUID& self, const std::string& name, const TData& a, const TData& b) {
            ev_obj.push_back(glob.at(self));
            ev_pid.push_back((int)(std::find(pname.begin(), pname.end(), name) - pname.begin()));
            uint64_t x, y;
            if (a.GetType() == TDATA_INT) {
                x = (uint64_t)a.GetInt();
                y = (uint64_t)b.GetInt();
            } else {
                const double u = a.GetFloat(), v = b.GetFloat();
                memcpy(&x, &u, 8);
                memcpy(&y, &v, 8);
            }
            ev_old.push_back(x);
            ev_new.push_back(y);
            moff.push_back((uint32_t)mr.size());
            return 0;
        });
        km.AddPropertyEventCallBack([&](const NFGUID&, const std::string&, const TData&, const TData&,
                                        const std::vector<NFGUID>& to) {
            for (auto& g : to) mr.push_back(glob.at(g));
            return 0;
        });
        km.RegisterCommonRecordEvent([&](const NFGUID& self, const RECORD_EVENT_DATA& ev, const TData& a, const TData& b) {
            re_obj.push_back(glob.at(self));
            const uint32_t op = ev.nOpType == RECORD_EVENT_DATA::Add ? 1u : ev.nOpType == RECORD_EVENT_DATA::Del ? 2u
                              : ev.nOpType == RECORD_EVENT_DATA::Cover ? 3u : 0u;
            re_rrc.push_back((op << 24) | ((uint32_t)std::stoi(ev.strRecordName.substr(3)) << 16) |
                             ((uint32_t)ev.nRow << 8) | (uint32_t)ev.nCol);
            uint64_t x = 0, y = 0;
            if (a.GetType() == TDATA_INT) {
                x = (uint64_t)a.GetInt();
                y = (uint64_t)b.GetInt();
            } else if (a.GetType() == TDATA_FLOAT) {
                const double u = a.GetFloat(), v = b.GetFloat();
                memcpy(&x, &u, 8);
                memcpy(&y, &v, 8);
            }
            re_old.push_back(x);
            re_new.push_back(y);
            moff.push_back((uint32_t)mr.size());
            return 0;
        });
        km.AddRecordEventCallBack([&](const NFGUID&, const std::string&, const RECORD_EVENT_DATA&, const TData&,
                                      const TData&, const std::vector<NFGUID>& to) {
            for (auto& g : to) mr.push_back(glob.at(g));
            return 0;
        });
        auto hb = [&](const NFGUID& self, const std::string& name, const float, const int nCount) {
            fi_obj.push_back(glob.at(self));
            fi_kind.push_back((int)(std::find(kname.begin(), kname.end(), name) - kname.begin()));
            fi_rem.push_back(nCount);
            return 0;
        };
        for (int k = 0; k < NK; k++) km.SetKindFunctor(kname[k], hb, 0.0f);
        for (int64_t i = 0; i < NS; i++) {
            if (owner(sc[s_obj[i]]) != r) continue;
            now = s_time[i];
            km.AddSchedule(NFGUID(gh[s_obj[i]], gd[s_obj[i]]), kname[s_kind[i]], hb, s_int[i], s_cnt[i]);
        }
        std::vector<int32_t> cur_sc(sc, sc + N), cur_gr(gr, gr + N);
        nfio_writer w;
        if (nfio_wopen(&w, (out_dir + "/rank" + std::to_string(r) + ".nfio").c_str())) {
            rc[r] = 2;
            return;
        }
        int64_t xi = 0, hi = 0, wi = 0;
        for (int tk = 0; tk < NT; tk++) {
            for (auto* v : {&ev_obj, &ev_pid, &re_obj, &fi_obj, &fi_kind, &fi_rem, &mr}) v->clear();
            for (auto* v : {&re_rrc, &moff}) v->clear();
            for (auto* v : {&ev_old, &ev_new, &re_old, &re_new}) v->clear();
            for (; wi < NW && sw_tick[wi] == tk; wi++) {
                const int o = sw_obj[wi];
                if (sw_scene[wi] >= 0) {
                    cur_sc[o] = sw_scene[wi];
                    cur_gr[o] = sw_group[wi];
                }
                const NFGUID g(gh[o], gd[o]);
                if (km.ObjectIndex(g) < 0 || km.Departing(g)) continue;  // another rank's (or leaving)
                if (owner(cur_sc[o]) == r) km.CreateScene(cur_sc[o]);
                if (!km.SwitchScene(g, cur_sc[o], cur_gr[o], sw_x[wi], sw_y[wi], sw_z[wi])) {
                    rc[r] = 5;
                }
            }
            if (!async) km.MigrateNow();
            if (transit_writes)  // the entities in transit on this rank, after their SwitchScene
                for (int64_t o = 0; o < N; o++) {
                    const NFGUID g(gh[o], gd[o]);
                    if (!km.Departing(g)) continue;
                    const int64_t v = 7000000 + o * 16 + tk;
                    if (!km.SetPropertyInt(g, "ATK_VALUE", v)) rc[r] = 6;
                    atk_expect[o] = v;
                }
            for (; hi < NH && h_tick[hi] == tk; hi++) {
                const NFGUID g(gh[h_obj[hi]], gd[h_obj[hi]]);
                if (km.ObjectIndex(g) < 0 || km.Departing(g)) continue;
                now = h_time[hi];
                if (h_op[hi] == 1) km.AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
                else if (h_op[hi] == 2) km.RemoveSchedule(g, kname[h_kind[hi]]);
                else km.RemoveSchedule(g);
            }
            for (; xi < NX && x_tick[xi] == tk; xi++) {
                const NFGUID g(gh[x_obj[xi]], gd[x_obj[xi]]);
                if (km.ObjectIndex(g) < 0 || km.Departing(g)) continue;
                if (x_pid[xi] < NI) {
                    km.SetPropertyInt(g, pname[x_pid[xi]], (int64_t)x_bits[xi]);
                } else {
                    double v;
                    memcpy(&v, &x_bits[xi], 8);
                    km.SetPropertyFloat(g, pname[x_pid[xi]], v);
                }
            }
            now = tick_time[tk];
            km.Execute();
            if (transit_writes)  // ... and after the Execute that started their tickets' gather
                for (int64_t o = 0; o < N; o++) {
                    const NFGUID g(gh[o], gd[o]);
                    if (!km.Departing(g)) continue;
                    const int64_t v = 8000000 + o * 16 + tk;
                    if (!km.SetPropertyInt(g, "ATK_VALUE", v)) rc[r] = 6;
                    atk_expect[o] = v;
                }
            moff.push_back((uint32_t)mr.size());
            char nm[40];
#define PUT(pfx, s, code, vec, es) snprintf(nm, sizeof nm, "%s_t%d_%s", pfx, tk, s); nfio_put1(&w, nm, code, vec.data(), vec.size(), es);
            PUT("ev", "obj", NFIO_I32, ev_obj, 4);
            PUT("ev", "pid", NFIO_I32, ev_pid, 4);
            PUT("ev", "old", NFIO_U64, ev_old, 8);
            PUT("ev", "new", NFIO_U64, ev_new, 8);
            PUT("re", "obj", NFIO_I32, re_obj, 4);
            PUT("re", "rrc", NFIO_U32, re_rrc, 4);
            PUT("re", "old", NFIO_U64, re_old, 8);
            PUT("re", "new", NFIO_U64, re_new, 8);
            PUT("fi", "obj", NFIO_I32, fi_obj, 4);
            PUT("fi", "kind", NFIO_I32, fi_kind, 4);
            PUT("fi", "rem", NFIO_I32, fi_rem, 4);
            PUT("mo", "off", NFIO_U32, moff, 4);
            PUT("mr", "obj", NFIO_I32, mr, 4);
        }
        // final state of the objects this rank holds: through the plugin API
        std::vector<int64_t> fi((size_t)NI * N, 0);
        std::vector<double> fff((size_t)NF * N, 0.0);
        std::vector<uint8_t> own(N, 0), present((size_t)NK * N, 0);
        for (int64_t o = 0; o < N; o++) {
            const NFGUID g(gh[o], gd[o]);
            if (km.ObjectIndex(g) < 0) continue;
            own[o] = 1;
            for (int p = 0; p < NI; p++) fi[(size_t)p * N + o] = km.GetPropertyInt(g, pname[p]);
            for (int p = 0; p < NF; p++) fff[(size_t)p * N + o] = km.GetPropertyFloat(g, pname[NI + p]);
            for (int k = 0; k < NK; k++) present[(size_t)k * N + o] = km.ExistSchedule(g, kname[k]);
        }
        uint64_t s2[2] = {(uint64_t)NI, (uint64_t)N};
        nfio_put(&w, "final_i", NFIO_I64, 2, s2, fi.data(), fi.size() * 8);
        s2[0] = (uint64_t)NF;
        nfio_put(&w, "final_f", NFIO_F64, 2, s2, fff.data(), fff.size() * 8);
        s2[0] = (uint64_t)NK;
        nfio_put(&w, "final_s_present", NFIO_U8, 2, s2, present.data(), present.size());
        nfio_put1(&w, "final_own", NFIO_U8, own.data(), own.size(), 1);
        const int64_t moved[2] = {km.MigratedOut(), km.MigratedIn()};
        nfio_put1(&w, "migrated", NFIO_I64, moved, 2, 8);
        nfio_wclose(&w);
        km.AttachShard(nullptr);
        km.Shut();
    };
    std::vector<std::thread> th;
    for (int r = 0; r < R; r++) th.emplace_back(rank_main, r);
    for (auto& x : th) x.join();
    for (int r = 0; r < R; r++)
        if (rc[r]) return rc[r];
    if (transit_writes) {
        nfio_writer w;
        if (nfio_wopen(&w, (out_dir + "/atk_expect.nfio").c_str())) return 2;
        nfio_put1(&w, "atk_expect", NFIO_I64, atk_expect.data(), atk_expect.size(), 8);
        nfio_wclose(&w);
    }
    return 0;
}
