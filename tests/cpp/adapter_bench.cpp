// adapter_bench.cpp — the DROP-IN path timed: a NoahGameFrame game server that loads the reference-side
// plugin (integration/NFGPUKernelPlugin.cpp: NFGPUKernelAdapter, NFGPUSceneAOIAdapter,
// NFGPUScheduleAdapter) in NFKernelPlugin's place, with the reference's own NFCKernelModule (under the
// adapter), NFCSceneAOIModule (under the AOI adapter), NFCEventModule, NFCScheduleModule, NFCClassModule
// and NFCElementModule compiled from /root/reference where they lie (tests/cpp/Makefile.adapter).  A
// workload world (bench.py writes BASELINE config[1] or config[0]) is created through
// NFIKernelModule::CreateObject with the class schema read from Struct XML, and the game logic a
// server registers is in place:
//   * a heartbeat functor on every schedule (NFIScheduleModule::AddSchedule, SM:257; the kind's effect
//     program runs on the device, the functor after the device frame);
//   * a common property and a common record callback (NFIKernelModule::RegisterCommonPropertyEvent,
//     NFIKernelModule.h:71-84) and the AOI module's recipient-list callbacks
//     (NFISceneAOIModule::AddPropertyEventCallBack / AddRecordEventCallBack: the client sync, AOI:703-727);
//   * mode 1 (Tutorial3, HelloWorld3Module.cpp:40-110): a per-object callback on every object's World
//     property and the OnEvent handler's SetPropertyInt(self, "World", v) on 1 % of the objects per
//     frame (the workload's x calls) between frames.
// Frames run back to back (every module's Execute, the window's calls before each); prints one JSON line:
// host ms per frame (median of the timed frames), the plugin's phases, what the callbacks received and
// how many device events reached NFCSceneAOIModule's own handlers (GetBroadCastObject) — 0.
//
//   * mode 2 (config[1] with NFCNPCRefreshModule's callback, NFCNPCRefreshModule.cpp:98-105): every NPC
//     registers AddPropertyCallBack(self, "HP", OnObjectHPEvent) at its creation (its newVar <= 0 test
//     counted): every NPC is eager and HP is logged per Set (k_chain), so each frame also fires one callback
//     per accepted HP Set of its heartbeat programs, in the walk's order.
//
// usage: adapter_bench <workload.nfio> <warmup> <frames> [mode] [calls] [wait]
//   mode 0: the config[1] logic above;  1: Tutorial3's (per-object World callbacks, OnEvent Sets)
//   calls 1: the workload's SetProperty / schedule calls between frames (mode 1 always makes its Sets)
//   wait 1: after the host objects are built (nothing has touched the GPU yet) print {"ready": ...} and
//           wait for a line on stdin before AfterInit: bench.py overlaps the reference's CreateObject of
//           1M objects (minutes of host work) with its GPU legs and times the frames after them
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../integration/NFGPUKernelPlugin.cpp"
#include "NFComm/NFConfigPlugin/NFCClassModule.h"
#include "NFComm/NFConfigPlugin/NFCElementModule.h"
#include "../../oracle/nfio.h"
#include "../../oracle/ref_server.hpp"

#ifdef ADAPTER_BENCH_PG
extern "C" void _mcleanup(void);  // (glibc's gmon writer)
#endif
static std::string cstr(const uint8_t* p) { return std::string((const char*)p, strnlen((const char*)p, 32)); }
static double bitsd(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}

struct Counters {
    int64_t hb = 0, prop = 0, rec = 0, aoi_prop = 0, aoi_rec = 0, rcpt = 0, obj_cb = 0;
    int OnHeartBeat(const NFGUID&, const std::string&, const float, const int) {
        hb++;
        return 0;
    }
    int OnProp(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&) {
        prop++;
        return 0;
    }
    int OnRecord(const NFGUID&, const RECORD_EVENT_DATA&, const NFIDataList::TData&, const NFIDataList::TData&) {
        rec++;
        return 0;
    }
    int OnAOIProp(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&, const NFIDataList& to) {
        aoi_prop++;
        rcpt += to.GetCount();
        return 0;
    }
    int OnAOIRecord(const NFGUID&, const std::string&, const RECORD_EVENT_DATA&, const NFIDataList::TData&,
                    const NFIDataList::TData&, const NFIDataList& to) {
        aoi_rec++;
        rcpt += to.GetCount();
        return 0;
    }
    int OnWorld(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&) {  // HelloWorld3Module.cpp:52
        obj_cb++;
        return 0;
    }
    int64_t kills = 0;
    int OnObjectHPEvent(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData& b) {
        obj_cb++;  // NFCNPCRefreshModule.cpp:113: newVar <= 0 kills
        kills += b.GetInt() <= 0;
        return 0;
    }
};

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    nfio_file wf;
    if (nfio_read(argv[1], &wf)) return 2;
    const int W = atoi(argv[2]), K = atoi(argv[3]);
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    const bool calls = mode == 1 || (argc > 5 && atoi(argv[5]) != 0);
    const bool wait = argc > 6 && atoi(argv[6]) != 0;

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
    if (W + K > NT) {
        fprintf(stderr, "workload has %lld frames, %d requested\n", (long long)NT, W + K);
        return 2;
    }
    const int64_t NP = NI + NF;
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    const int OPK = nfio_ops_per_kind(A("ops"));
    int32_t* nops = (int32_t*)A("n_ops")->data;
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) pname[p] = cstr(pnames + 32 * p);
    for (int k = 0; k < NK; k++) kname[k] = cstr(knames + 32 * k);

    const auto tb = std::chrono::steady_clock::now();
    TestPluginManager pm;
    write_class_schema(pm, wf, pname, cname, NI, NF, NC, NR);
    TestLogModule log;
    NFCClassModule classes(&pm);
    NFCElementModule elements(&pm);
    NFGPUKernelAdapter kernel(&pm);
    NFGPUSceneAOIAdapter aoi(&pm);
    NFCEventModule events(&pm);
    NFGPUScheduleAdapter sched(&pm);
    pm.AddModule(typeid(NFILogModule).name(), &log);
    pm.AddModule(typeid(NFIClassModule).name(), &classes);
    pm.AddModule(typeid(NFIElementModule).name(), &elements);
    pm.AddModule(typeid(NFIKernelModule).name(), &kernel);
    pm.AddModule(typeid(NFISceneAOIModule).name(), &aoi);
    pm.AddModule(typeid(NFIEventModule).name(), &events);
    pm.AddModule(typeid(NFIScheduleModule).name(), &sched);
    std::vector<NFIModule*> all = {&log, &classes, &elements, &kernel, &aoi, &events, &sched};
    kernel.gpu_.SetTimeSource([] { return g_now; });
    std::vector<std::string> rname;
    for (int r = 0; r < NR; r++) rname.push_back("rec" + std::to_string(r));
    // each schedule name's device program (a logic module's Init; an empty one for a functor-only
    // heartbeat such as Tutorial3's OnHeartBeat: the device scans its timers)
    for (int k = 0; k < NK; k++)
        kernel.gpu_.AddHeartBeatProgram(kname[k], std::vector<nfk_op>(ops + k * OPK, ops + k * OPK + nops[k]), pname, rname);
    for (auto* m : all) m->Awake();
    for (auto* m : all) m->Init();
    NFIKernelModule* km = &kernel;
    NFIScheduleModule* sm = &sched;
    NFISceneAOIModule* am = &aoi;

    int64_t* gh = (int64_t*)A("guid_head")->data;
    int64_t* gd = (int64_t*)A("guid_data")->data;
    int32_t* sc = (int32_t*)A("scene")->data;
    int32_t* gr = (int32_t*)A("group")->data;
    uint8_t* cl = (uint8_t*)A("cls")->data;
    int64_t* ii = (int64_t*)A("init_i")->data;
    double* ff = (double*)A("init_f")->data;
    {
        std::map<int, int> groups;
        for (int64_t o = 0; o < N; o++) groups[sc[o]] = std::max(groups[sc[o]], gr[o]);
        for (auto& kv : groups) {
            km->CreateScene(kv.first);
            for (int g = 1; g <= kv.second; g++)
                if (km->RequestGroupScene(kv.first) != g) return 3;
        }
    }
    Counters C;
    // objects are created group by group (a server spawning a scene's groups one after the other): the
    // reference's AOI module reads every member's ClassName for each object entering a group
    // (OnGroupEvent, AOI:357-440), so a group's members are re-read while they are in cache
    std::vector<int64_t> order((size_t)N);
    for (int64_t o = 0; o < N; o++) order[(size_t)o] = o;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return sc[a] != sc[b] ? sc[a] < sc[b] : gr[a] < gr[b];
    });
    for (int64_t o : order) {  // NFCKernelModule::CreateObject (KM:101) with the values as arguments
        NFCDataList arg;
        for (int p = 0; p < NP; p++) {
            if (pname[p] == "SceneID" || pname[p] == "GroupID") continue;
            arg.Add(pname[p]);
            if (p < NI) arg.Add((NFINT64)ii[p * N + o]);
            else arg.Add(ff[(p - NI) * N + o]);
        }
        NF_SHARE_PTR<NFIObject> ob = km->CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], "", arg);
        if (!ob) return 3;
        if (mode == 1) ob->AddPropertyCallBack("World", &C, &Counters::OnWorld);  // HelloWorld3Module.cpp:95
        if (mode == 2 && cl[o] == 0)  // NFCNPCRefreshModule.cpp:104, at the NPC's creation
            km->AddPropertyCallBack(NFGUID(gh[o], gd[o]), "HP", &C, &Counters::OnObjectHPEvent);
    }
    const double host_build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();
    if (wait) {
        printf("{\"ready\": %.1f}\n", host_build_s);
        fflush(stdout);
        char line[64];
        if (!fgets(line, sizeof line, stdin)) return 4;
    }
    const auto ta = std::chrono::steady_clock::now();
    for (auto* m : all) m->AfterInit();
    km->RegisterCommonPropertyEvent(&C, &Counters::OnProp);
    km->RegisterCommonRecordEvent(&C, &Counters::OnRecord);
    am->AddPropertyEventCallBack(&C, &Counters::OnAOIProp);
    am->AddRecordEventCallBack(&C, &Counters::OnAOIRecord);
    for (auto* m : all) m->ReadyExecute();
    OBJECT_SCHEDULE_FUNCTOR_PTR hb(new OBJECT_SCHEDULE_FUNCTOR(
        std::bind(&Counters::OnHeartBeat, &C, std::placeholders::_1, std::placeholders::_2, std::placeholders::_3,
                  std::placeholders::_4)));
    int32_t* s_obj = (int32_t*)A("s_obj")->data;
    int32_t* s_kind = (int32_t*)A("s_kind")->data;
    float* s_int = (float*)A("s_interval")->data;
    int32_t* s_cnt = (int32_t*)A("s_count")->data;
    int64_t* s_time = (int64_t*)A("s_time")->data;
    for (int64_t i = 0; i < NS; i++) {
        g_now = s_time[i];
        sm->AddSchedule(NFGUID(gh[s_obj[i]], gd[s_obj[i]]), kname[s_kind[i]], hb, s_int[i], s_cnt[i]);
    }
    const double build_s = host_build_s + std::chrono::duration<double>(std::chrono::steady_clock::now() - ta).count();

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

    int64_t xi = 0, hi = 0;
    // frames [t0, t0 + W + K): the window's calls before each, every module's Execute; the timed K frames
    // as one JSON object
    auto run = [&](int t0, int W, int K) -> std::string {
        std::vector<nfgpu::NFGPUKernelModule::FrameStats> st;
        std::vector<double> call_ms, frame_ms;
        int64_t ncalls = 0;
        int64_t syncs0 = kernel.MirrorSyncs(), chain0 = kernel.ChainCallbacks();
        Counters c0;
        if (kernel.gpu_.World()) nfk_set_profiling(kernel.gpu_.World(), 1);  // (HIP events around each kernel)
        for (int t = t0; t < t0 + W + K; t++) {
            if (t == t0 + W) {  // (the timed frames' counts)
                if (kernel.gpu_.World()) nfk_reset_kernel_times(kernel.gpu_.World());
                c0 = C;
                syncs0 = kernel.MirrorSyncs();
                chain0 = kernel.ChainCallbacks();
            }
            const auto ts0 = std::chrono::steady_clock::now();
            for (; hi < NH && h_tick[hi] == t; hi++) {
                if (!calls) continue;
                const NFGUID g(gh[h_obj[hi]], gd[h_obj[hi]]);
                g_now = h_time[hi];
                if (h_op[hi] == 1) sm->AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
                else if (h_op[hi] == 2) sm->RemoveSchedule(g, kname[h_kind[hi]]);
                else sm->RemoveSchedule(g);
                ncalls += t >= t0 + W;
            }
            for (; xi < NX && x_tick[xi] == t; xi++) {
                if (!calls) continue;
                const NFGUID g(gh[x_obj[xi]], gd[x_obj[xi]]);
                if (x_pid[xi] < NI) km->SetPropertyInt(g, pname[x_pid[xi]], (int64_t)x_bits[xi]);
                else km->SetPropertyFloat(g, pname[x_pid[xi]], bitsd(x_bits[xi]));
                ncalls += t >= t0 + W;
            }
            const auto ts1 = std::chrono::steady_clock::now();
            g_now = tick_time[t];
            for (auto* m : all) m->Execute();
            const auto ts2 = std::chrono::steady_clock::now();
            if (t >= t0 + W) {
                st.push_back(kernel.gpu_.LastFrameStats());
                call_ms.push_back(std::chrono::duration<double, std::milli>(ts1 - ts0).count());
                frame_ms.push_back(std::chrono::duration<double, std::milli>(ts2 - ts0).count());
            }
        }
        auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v.empty() ? 0.0 : v[v.size() / 2];
        };
        auto medf = [&](double nfgpu::NFGPUKernelModule::FrameStats::*m) {
            std::vector<double> v;
            for (auto& s : st) v.push_back(s.*m);
            return med(v);
        };
        // the device kernels' HIP-event time per frame (timer names: nfgpu.h nfk_kernel_times)
        double kms[NFK_N_KERNEL_TIMERS] = {0};
        int64_t kl[NFK_N_KERNEL_TIMERS] = {0}, kb[NFK_N_KERNEL_TIMERS] = {0};
        if (kernel.gpu_.World()) nfk_kernel_times(kernel.gpu_.World(), kms, kl, kb);
        const nfk_summary& s = kernel.gpu_.LastSummary();
        const double kf = K ? (double)K : 1.0;
        char buf[4096];
        snprintf(buf, sizeof buf,
                 "{\"adapter_frame_ms\": %.3f, \"entities\": %lld, \"entity_ticks_per_s\": %.4g, \"calls_per_frame\": %lld, "
                 "\"phases_ms\": {\"calls\": %.3f, \"device\": %.3f, \"functors\": %.3f, \"events_read\": %.3f, "
                 "\"deliver\": %.3f, \"functor_calls\": %.3f, \"plugin_execute\": %.3f, \"gather\": %.3f, \"mirror\": %.3f}, "
                 "\"per_frame\": {\"fired\": %lld, \"prop_events\": %lld, \"rec_events\": %lld, \"messages\": %lld}, "
                 "\"received_per_frame\": {\"heartbeats\": %.0f, \"common_prop\": %.0f, \"common_rec\": %.0f, \"aoi_prop\": %.0f, "
                 "\"aoi_rec\": %.0f, \"recipients\": %.0f, \"per_object_callbacks\": %.0f, \"hp_kills\": %.0f}, "
                 "\"aoi\": {\"device_list_calls\": %lld, \"host_getbroadcastobject_calls_for_device_events\": %lld}, "
                 "\"mirror\": {\"lazy_syncs_per_frame\": %.1f, \"chain_callbacks_per_frame\": %.0f}, "
                 "\"device_kernels_ms_per_frame\": {\"k_tick\": %.4f, \"k_records\": %.4f, \"k_fanout\": %.4f, \"aux\": %.4f, "
                 "\"k_scan_tiles\": %.4f, \"membership\": %.4f, \"k_chain\": %.4f}, \"k_chain_launches\": %lld, "
                 "\"frames\": %d, \"warmup\": %d",
                 med(frame_ms), (long long)N, (double)N / (med(frame_ms) * 1e-3), (long long)(K ? ncalls / K : 0),
                 med(call_ms), medf(&nfgpu::NFGPUKernelModule::FrameStats::device),
                 medf(&nfgpu::NFGPUKernelModule::FrameStats::functors), medf(&nfgpu::NFGPUKernelModule::FrameStats::events_read),
                 medf(&nfgpu::NFGPUKernelModule::FrameStats::deliver), medf(&nfgpu::NFGPUKernelModule::FrameStats::calls),
                 medf(&nfgpu::NFGPUKernelModule::FrameStats::total), medf(&nfgpu::NFGPUKernelModule::FrameStats::gather),
                 medf(&nfgpu::NFGPUKernelModule::FrameStats::mirror),
                 (long long)s.n_fired, (long long)s.n_prop_events, (long long)s.n_rec_events, (long long)s.n_msgs,
                 (C.hb - c0.hb) / kf, (C.prop - c0.prop) / kf, (C.rec - c0.rec) / kf, (C.aoi_prop - c0.aoi_prop) / kf,
                 (C.aoi_rec - c0.aoi_rec) / kf, (C.rcpt - c0.rcpt) / kf, (C.obj_cb - c0.obj_cb) / kf, (C.kills - c0.kills) / kf,
                 (long long)kernel.AOIDeviceCalls(), (long long)kernel.AOIHostDeviceCalls(),
                 (kernel.MirrorSyncs() - syncs0) / kf, (kernel.ChainCallbacks() - chain0) / kf, kms[0] / kf, kms[1] / kf,
                 kms[2] / kf, kms[3] / kf, kms[4] / kf, kms[5] / kf, kms[6] / kf, (long long)kl[6], K, W);
        return buf;
    };
    std::string line = run(0, W, K);
    char tail[200];
    snprintf(tail, sizeof tail, ", \"build_s\": %.1f, \"host_objects_s\": %.1f, \"mode\": \"%s\"", build_s, host_build_s,
             mode == 1 ? "tutorial3" : mode == 2 ? "config1-npc-hp-callbacks" : calls ? "config1-with-calls" : "config1");
    line += tail;
    printf("%s}\n", line.c_str());
    fflush(stdout);
#ifdef ADAPTER_BENCH_PG
    _mcleanup();  // (the -pg build: gmon.out, which exit() would write)
#endif
    _exit(0);  // (static destructors: NFMemoryCounter's static map dies before the modules' objects)
}
