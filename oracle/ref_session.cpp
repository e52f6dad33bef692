// ref_session.cpp — a NoahGameFrame game server's frame on the CPU, run by the REFERENCE's own
// modules compiled from /root/reference where they lie (oracle/Makefile `make ref`):
//   NFKernelPlugin   NFCKernelModule, NFCScheduleModule, NFCSceneAOIModule, NFCEventModule
//   NFConfigPlugin   NFCClassModule, NFCElementModule (the class schema from Struct XML)
//   NFCore           NFCDataList, NFCProperty(Manager), NFCRecord(Manager), NFCObject, ...
// with the plugin manager and log module test doubles of oracle/ref_server.hpp.
//
// TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline ("reference" kind: the reference's whole frame
// path — NFCScheduleModule::Execute walking the schedules (SM:49-119), the heartbeat functors'
// SetPropertyInt/Float through NFCKernelModule (KM:323-347: GetElement(self), NFCProperty
// change predicates, the common property event), NFCSceneAOIModule::OnPropertyCommonEvent's
// GetBroadCastObject recipient lists (AOI:227-258, 531-593) handed to the property-event
// callbacks a network layer registers), and a cross-check of the oracle's final state against the
// compiled kernel module (tests/test_oracle.py).
//
// The workload's game logic: each heartbeat name's effect program (nfgpu.h nfk_op) run by its
// functor through NFIKernelModule (GetProperty* / SetProperty*, GetRecord* / SetRecord*), the
// window's SetProperty / AddSchedule / RemoveSchedule calls before each frame.  NFCScheduleModule
// reads wall time through NFGetTime() (NFPlatform.h:367, CLOCK_REALTIME): a virtual clock is
// supplied by defining clock_gettime, as oracle/ref_harness.cpp does.
//
// usage: nf_ref_session <workload.nfio> <ticks> <warmup> [final.nfio]
//   prints {"entity_ticks_per_s", "ms_per_frame", "frames", "entities", "events", "msgs", ...}
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "NFComm/NFConfigPlugin/NFCClassModule.h"
#include "NFComm/NFConfigPlugin/NFCElementModule.h"
#include "NFComm/NFCore/NFCDataList.h"
#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCScheduleModule.h"
#include "NFComm/NFKernelPlugin/NFCSceneAOIModule.h"
#include "ref_server.hpp"

extern "C" int clock_gettime(clockid_t clk, struct timespec* ts) {
    if (clk == CLOCK_REALTIME) {
        ts->tv_sec = g_now / 1000;
        ts->tv_nsec = (g_now % 1000) * 1000000;
        return 0;
    }
    return (int)syscall(SYS_clock_gettime, clk, ts);
}

static uint64_t dbits(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}
static double bitsd(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}
static std::string cstr(const uint8_t* p) { return std::string((const char*)p, strnlen((const char*)p, 32)); }

// what a network layer's AOI callbacks receive per frame (counted, as a packer would walk them)
struct Consumer {
    int64_t events = 0, msgs = 0, rec_events = 0;
    int OnAOIProp(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&,
                  const NFIDataList& to) {
        events++;
        msgs += to.GetCount();
        return 0;
    }
    int OnAOIRecord(const NFGUID&, const std::string&, const RECORD_EVENT_DATA&, const NFIDataList::TData&,
                    const NFIDataList::TData&, const NFIDataList& to) {
        rec_events++;
        msgs += to.GetCount();
        return 0;
    }
};

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) {
        fprintf(stderr, "usage: nf_ref_session <workload.nfio> <ticks> <warmup> [final.nfio]\n");
        return 2;
    }
    nfio_file wf;
    if (nfio_read(argv[1], &wf)) return 2;
    auto A = [&](const char* n) {
        nfio_arr* a = nfio_get(&wf, n);
        if (!a) {
            fprintf(stderr, "missing %s\n", n);
            exit(2);
        }
        return a;
    };
    int64_t* cfg = (int64_t*)A("cfg")->data;
    const int64_t N = cfg[0], NI = cfg[1], NF = cfg[2], NC = cfg[3], NK = cfg[4], NR = cfg[5], NS = cfg[6];
    const int64_t NT = std::min<int64_t>(cfg[7], atoll(argv[2])), W = std::min<int64_t>(NT, atoll(argv[3]));
    nfio_arr* noa = nfio_get(&wf, "n_oprops");
    const int64_t NO = noa ? ((int64_t*)noa->data)[0] : 0;
    const int64_t NP = NI + NF + NO;
    auto has_rows = [&](const char* n) {
        nfio_arr* a = nfio_get(&wf, n);
        return a && a->shape[0] > 0;
    };
    if (has_rows("sw_tick") || has_rows("d_tick") || nfio_get(&wf, "born") || has_rows("r_tick")) {
        fprintf(stderr, "nf_ref_session: membership changes and record calls are not replayed here\n");
        return 5;
    }
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    int32_t* nops = (int32_t*)A("n_ops")->data;
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) pname[p] = cstr(pnames + 32 * p);
    for (int k = 0; k < NK; k++) kname[k] = cstr(knames + 32 * k);
    for (int k = 0; k < NK; k++)
        for (int i = 0; i < nops[k]; i++)
            if (ops[k * NFK_MAX_OPS + i].code == NFK_OP_RFAFFINE) {
                fprintf(stderr, "nf_ref_session: record f64 ops cannot run on the reference (NFCRecord::SetFloat, "
                                "see nf_ref_harness --repro-record-float)\n");
                return 3;
            }

    TestPluginManager pm;
    write_class_schema(pm, wf, pname, cname, NI, NF, NC, NR);
    TestLogModule log;
    NFCClassModule classes(&pm);
    NFCElementModule elements(&pm);
    NFCKernelModule kernel(&pm);
    NFCSceneAOIModule aoi(&pm);
    NFCEventModule events(&pm);
    NFCScheduleModule sched(&pm);
    pm.AddModule(typeid(NFILogModule).name(), &log);
    pm.AddModule(typeid(NFIClassModule).name(), &classes);
    pm.AddModule(typeid(NFIElementModule).name(), &elements);
    pm.AddModule(typeid(NFIKernelModule).name(), &kernel);
    pm.AddModule(typeid(NFISceneAOIModule).name(), &aoi);
    pm.AddModule(typeid(NFIEventModule).name(), &events);
    pm.AddModule(typeid(NFIScheduleModule).name(), &sched);
    std::vector<NFIModule*> all = {&log, &classes, &elements, &kernel, &aoi, &events, &sched};
    for (auto* m : all) m->Awake();
    for (auto* m : all) m->Init();
    NFIKernelModule* km = &kernel;
    NFIScheduleModule* sm = &sched;

    int64_t* gh = (int64_t*)A("guid_head")->data;
    int64_t* gd = (int64_t*)A("guid_data")->data;
    int32_t* sc = (int32_t*)A("scene")->data;
    int32_t* gr = (int32_t*)A("group")->data;
    uint8_t* cl = (uint8_t*)A("cls")->data;
    int64_t* ii = (int64_t*)A("init_i")->data;
    double* ff = (double*)A("init_f")->data;
    int64_t* ioh = NO ? (int64_t*)A("init_oh")->data : nullptr;
    int64_t* iod = NO ? (int64_t*)A("init_od")->data : nullptr;
    {  // scenes and their groups 1..G (CreateScene / RequestGroupScene, KM:981, 1104)
        std::map<int, int> groups;
        for (int64_t o = 0; o < N; o++) groups[sc[o]] = std::max(groups[sc[o]], gr[o]);
        for (auto& kv : groups) {
            km->CreateScene(kv.first);
            for (int g = 1; g <= kv.second; g++)
                if (km->RequestGroupScene(kv.first) != g) return 3;
        }
    }
    for (int64_t o = 0; o < N; o++) {  // NFCKernelModule::CreateObject (KM:101) with the workload's values
        NFCDataList arg;
        for (int p = 0; p < NP; p++) {
            if (pname[p] == "SceneID" || pname[p] == "GroupID") continue;
            arg.Add(pname[p]);
            if (p < NI) arg.Add((NFINT64)ii[p * N + o]);
            else if (p < NI + NF) arg.Add(ff[(p - NI) * N + o]);
            else arg.Add(NFGUID(ioh[(p - NI - NF) * N + o], iod[(p - NI - NF) * N + o]));
        }
        if (!km->CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], "", arg)) return 3;
    }
    for (int r = 0; r < NR; r++) {  // creation-time record rows
        char nm[32];
        snprintf(nm, sizeof nm, "rec%d_cells", r);
        uint64_t* cells = (uint64_t*)A(nm)->data;
        snprintf(nm, sizeof nm, "rec%d_used", r);
        uint64_t* used = (uint64_t*)A(nm)->data;
        const int32_t rows = ((int32_t*)A("rec_rows")->data)[r], cols = ((int32_t*)A("rec_cols")->data)[r];
        uint8_t* ct = (uint8_t*)A("rec_ctype")->data;
        for (int64_t o = 0; o < N; o++) {
            NF_SHARE_PTR<NFIRecord> R = km->FindRecord(NFGUID(gh[o], gd[o]), "rec" + std::to_string(r));
            for (int row = 0; row < rows; row++) {
                if (!((used[o] >> row) & 1)) continue;
                NFCDataList v;
                for (int c = 0; c < cols; c++) {
                    const uint64_t b = cells[((size_t)o * cols + c) * rows + row];
                    if (ct[r * NFK_MAX_REC_COLS + c]) v.Add(bitsd(b));
                    else v.Add((NFINT64)b);
                }
                R->AddRow(row, v);
            }
        }
    }
    for (auto* m : all) m->AfterInit();
    Consumer net;
    NFISceneAOIModule* am = &aoi;  // (the interface's member templates)
    am->AddPropertyEventCallBack(&net, &Consumer::OnAOIProp);
    am->AddRecordEventCallBack(&net, &Consumer::OnAOIRecord);
    for (auto* m : all) m->ReadyExecute();

    // the heartbeat functor: the name's effect program through NFIKernelModule, as game logic
    // written against the reference would run it (the oracle's arithmetic, same operation order)
    std::map<std::string, int> kid;
    for (int k = 0; k < NK; k++) kid[kname[k]] = k;
    std::vector<std::string> rname;
    for (int r = 0; r < NR; r++) rname.push_back("rec" + std::to_string(r));
    int64_t fired = 0;
    auto heartbeat = [&](const NFGUID& self, const std::string& name, const float, const int) -> int {
        fired++;
        const int k = kid.at(name);
        for (int i = 0; i < nops[k]; i++) {
            const nfk_op& op = ops[k * NFK_MAX_OPS + i];
            switch (op.code) {
            case NFK_OP_IADD_CLAMP: {
                const std::string& d = pname[op.dst];
                const int64_t cur = km->GetPropertyInt(self, d);
                const int64_t a = (op.flags & NFK_A_PROP) ? km->GetPropertyInt(self, pname[op.a]) : op.a;
                const int64_t lo = (op.flags & NFK_LO_PROP) ? km->GetPropertyInt(self, pname[op.b]) : op.b;
                const int64_t hi = (op.flags & NFK_HI_PROP) ? km->GetPropertyInt(self, pname[op.c]) : op.c;
                int64_t v = (int64_t)((uint64_t)cur + (uint64_t)a);
                if (v < lo) v = lo;
                if (v > hi) v = hi;
                km->SetPropertyInt(self, d, v);
                break;
            }
            case NFK_OP_FLERP: {
                const std::string& d = pname[op.dst];
                const double x = km->GetPropertyFloat(self, d);
                const double t = km->GetPropertyFloat(self, pname[op.a]);
                const double dd = t - x;
                const double m = dd * bitsd((uint64_t)op.b);
                km->SetPropertyFloat(self, d, x + m);
                break;
            }
            case NFK_OP_FAFFINE: {
                const std::string& d = pname[op.dst];
                const double x = km->GetPropertyFloat(self, d);
                const double m = x * bitsd((uint64_t)op.a);
                km->SetPropertyFloat(self, d, m + bitsd((uint64_t)op.b));
                break;
            }
            case NFK_OP_RIADD_CLAMP: {  // every used row of the column (NFCRecord::SetInt, RC:182)
                const std::string& rn = rname[op.dst >> 8];
                const int col = op.dst & 255;
                NF_SHARE_PTR<NFIRecord> R = km->FindRecord(self, rn);
                for (int row = 0; R && row < R->GetRows(); row++) {
                    if (!R->IsUsed(row)) continue;
                    int64_t v = (int64_t)((uint64_t)km->GetRecordInt(self, rn, row, col) + (uint64_t)op.a);
                    if (v < op.b) v = op.b;
                    if (v > op.c) v = op.c;
                    km->SetRecordInt(self, rn, row, col, v);
                }
                break;
            }
            default:
                break;
            }
        }
        return 0;
    };
    OBJECT_SCHEDULE_FUNCTOR_PTR hb(new OBJECT_SCHEDULE_FUNCTOR(heartbeat));
    int32_t* s_obj = (int32_t*)A("s_obj")->data;
    int32_t* s_kind = (int32_t*)A("s_kind")->data;
    float* s_int = (float*)A("s_interval")->data;
    int32_t* s_cnt = (int32_t*)A("s_count")->data;
    int64_t* s_time = (int64_t*)A("s_time")->data;
    for (int64_t i = 0; i < NS; i++) {  // NFIScheduleModule::AddSchedule (SM:218)
        g_now = s_time[i];
        sm->AddSchedule(NFGUID(gh[s_obj[i]], gd[s_obj[i]]), kname[s_kind[i]], hb, s_int[i], s_cnt[i]);
    }

    int64_t* tick_time = (int64_t*)A("tick_time")->data;
    nfio_arr* xa = A("x_tick");
    const int64_t NX = (int64_t)xa->shape[0];
    int32_t* x_tick = (int32_t*)xa->data;
    int32_t* x_obj = (int32_t*)A("x_obj")->data;
    int32_t* x_pid = (int32_t*)A("x_pid")->data;
    uint64_t* x_bits = (uint64_t*)A("x_bits")->data;
    uint64_t* x_bits_h = NO ? (uint64_t*)A("x_bits_h")->data : nullptr;
    nfio_arr* xma = nfio_get(&wf, "x_mode");
    uint8_t* x_mode = xma ? (uint8_t*)xma->data : nullptr;
    nfio_arr* ha = A("h_tick");
    const int64_t NH = (int64_t)ha->shape[0];
    int32_t* h_tick = (int32_t*)ha->data;
    int32_t* h_op = (int32_t*)A("h_op")->data;
    int32_t* h_obj = (int32_t*)A("h_obj")->data;
    int32_t* h_kind = (int32_t*)A("h_kind")->data;
    float* h_int = (float*)A("h_interval")->data;
    int32_t* h_cnt = (int32_t*)A("h_count")->data;
    int64_t* h_time = (int64_t*)A("h_time")->data;

    using clk = std::chrono::steady_clock;
    clk::time_point t0 = clk::now();
    int64_t ev0 = 0, msg0 = 0, re0 = 0, fi0 = 0;
    int64_t xi = 0, hi = 0;
    for (int64_t t = 0; t < NT; t++) {
        if (t == W) {  // the timed frames start here
            t0 = clk::now();
            ev0 = net.events;
            msg0 = net.msgs;
            re0 = net.rec_events;
            fi0 = fired;
        }
        for (; hi < NH && h_tick[hi] == t; hi++) {
            const NFGUID g(gh[h_obj[hi]], gd[h_obj[hi]]);
            g_now = h_time[hi];
            if (h_op[hi] == 1) sm->AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
            else if (h_op[hi] == 2) sm->RemoveSchedule(g, kname[h_kind[hi]]);
            else sm->RemoveSchedule(g);
        }
        for (; xi < NX && x_tick[xi] == t; xi++) {
            const NFGUID g(gh[x_obj[xi]], gd[x_obj[xi]]);
            const std::string& pn = pname[x_pid[xi]];
            const bool rmw = x_mode && x_mode[xi];  // KM:401 after KM:323
            if (x_pid[xi] < NI)
                km->SetPropertyInt(g, pn, rmw ? (int64_t)((uint64_t)km->GetPropertyInt(g, pn) + x_bits[xi]) : (int64_t)x_bits[xi]);
            else if (x_pid[xi] < NI + NF)
                km->SetPropertyFloat(g, pn, rmw ? km->GetPropertyFloat(g, pn) + bitsd(x_bits[xi]) : bitsd(x_bits[xi]));
            else
                km->SetPropertyObject(g, pn, NFGUID((int64_t)x_bits_h[xi], (int64_t)x_bits[xi]));
        }
        g_now = tick_time[t];
        for (auto* m : all) m->Execute();  // NFCScheduleModule::Execute walks the schedules (SM:49)
    }
    const double sec = std::chrono::duration<double>(clk::now() - t0).count();
    const int64_t frames = NT - W;
    printf("{\"entity_ticks_per_s\": %.6g, \"ms_per_frame\": %.4f, \"frames\": %lld, \"warmup\": %lld, "
           "\"entities\": %lld, \"fired\": %lld, \"events\": %lld, \"rec_events\": %lld, \"msgs\": %lld, "
           "\"seconds\": %.3f, \"log_errors\": %d}\n",
           frames > 0 ? (double)N * frames / sec : 0.0, frames > 0 ? 1000.0 * sec / frames : 0.0, (long long)frames,
           (long long)W, (long long)N, (long long)(fired - fi0), (long long)(net.events - ev0),
           (long long)(net.rec_events - re0), (long long)(net.msgs - msg0), sec, log.errors);
    fflush(stdout);
    if (argc == 5) {  // the final state through NFIKernelModule::GetProperty* (the oracle cross-check)
        std::vector<int64_t> fi((size_t)NI * N, 0);
        std::vector<double> fff((size_t)NF * N, 0.0);
        for (int64_t o = 0; o < N; o++) {
            const NFGUID g(gh[o], gd[o]);
            for (int p = 0; p < NI; p++) fi[(size_t)p * N + o] = km->GetPropertyInt(g, pname[p]);
            for (int p = 0; p < NF; p++) fff[(size_t)p * N + o] = km->GetPropertyFloat(g, pname[NI + p]);
        }
        nfio_writer w;
        if (nfio_wopen(&w, argv[4])) return 2;
        uint64_t s2[2] = {(uint64_t)NI, (uint64_t)N};
        nfio_put(&w, "final_i", NFIO_I64, 2, s2, fi.data(), fi.size() * 8);
        s2[0] = (uint64_t)NF;
        nfio_put(&w, "final_f", NFIO_F64, 2, s2, fff.data(), fff.size() * 8);
        int64_t counts[4] = {fired, net.events, net.rec_events, net.msgs};
        nfio_put1(&w, "counts", NFIO_I64, counts, 4, 8);
        nfio_wclose(&w);
    }
    _exit(0);  // (static destructors: NFMemoryCounter's static map dies before the modules' objects)
}
