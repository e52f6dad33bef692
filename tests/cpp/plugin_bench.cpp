// plugin_bench.cpp — the C++ plugin frame (NFGPUKernelModule::Execute) timed from a C++ game-server
// client, no Python anywhere: a workload world (normally BASELINE config[1], written by
// bench.py / workload.bench_world) is built through the plugin API, a functor is registered on
// every schedule (AddSchedule, SM:257), a common property / record callback and an AOI recipient
// callback are registered (they count what they receive), and frames run back to back.  Prints one
// JSON line: host ms per frame (median of the timed frames) and its phases (FrameStats).
//
// usage: plugin_bench <workload.nfio> <warmup> <frames> [calls] [consumer]
//   calls = 1: the workload's SetProperty / schedule calls are made between frames (game logic)
//   consumer = 0: the reference's per-call API (a functor per schedule, common property / record and
//                 AOI recipient callbacks per event)
//              1: one frame batch callback (AddFrameCallBack: fired list + events + recipient CSR as
//                 arrays), schedules without host functors
//              2: no host consumer (schedules without functors, no callbacks: the frame's outputs stay
//                 on the device for a device-side consumer)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "NFGPUKernelModule.hpp"
#include "../../oracle/nfio.h"

using namespace nfgpu;

static int64_t g_now = 0;
static std::string cstr(const uint8_t* p) { return std::string((const char*)p, strnlen((const char*)p, 32)); }

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    nfio_file wf;
    if (nfio_read(argv[1], &wf)) return 2;
    const int W = atoi(argv[2]), K = atoi(argv[3]);
    const bool calls = argc > 4 && atoi(argv[4]) != 0;
    const int consumer = argc > 5 ? atoi(argv[5]) : 0;
    auto A = [&](const char* n) {
        nfio_arr* a = nfio_get(&wf, n);
        if (!a) {
            fprintf(stderr, "missing %s\n", n);
            exit(2);
        }
        return a;
    };
    int64_t* cfg = (int64_t*)A("cfg")->data;
    const int64_t N = cfg[0], NI = cfg[1], NF = cfg[2], NC = cfg[3], NK = cfg[4], NS = cfg[6], NT = cfg[7];
    if (W + K > NT) {
        fprintf(stderr, "workload has %lld frames, %d requested\n", (long long)NT, W + K);
        return 2;
    }
    const int64_t NP = NI + NF;
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    uint8_t* pflags = (uint8_t*)A("prop_flags")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    const int OPK = nfio_ops_per_kind(A("ops"));  // ops per kind in the file
    int32_t* nops = (int32_t*)A("n_ops")->data;

    const auto tb = std::chrono::steady_clock::now();
    NFGPUKernelModule km((int)N);
    km.SetTimeSource([] { return g_now; });
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) {
        pname[p] = cstr(pnames + 32 * p);
        km.AddProperty(pname[p], p < NI ? TDATA_INT : TDATA_FLOAT);
    }
    for (int c = 0; c < NC; c++) {
        km.AddClass(cname[c]);
        for (int p = 0; p < NP; p++) {
            const uint8_t f = pflags[c * NP + p];
            km.SetPropertyFlags(cname[c], pname[p], f & NFK_PUBLIC, f & NFK_PRIVATE, f & NFK_UPLOAD);
        }
    }
    for (int k = 0; k < NK; k++) {
        kname[k] = cstr(knames + 32 * k);
        km.AddHeartBeatProgram(kname[k], std::vector<nfk_op>(ops + k * OPK, ops + k * OPK + nops[k]));
    }
    km.Init();
    int64_t* gh = (int64_t*)A("guid_head")->data;
    int64_t* gd = (int64_t*)A("guid_data")->data;
    int32_t* sc = (int32_t*)A("scene")->data;
    int32_t* gr = (int32_t*)A("group")->data;
    uint8_t* cl = (uint8_t*)A("cls")->data;
    int64_t* ii = (int64_t*)A("init_i")->data;
    double* ff = (double*)A("init_f")->data;
    for (int64_t o = 0; o < N; o++) {
        km.CreateScene(sc[o]);
        std::map<std::string, TData> init;
        for (int p = 0; p < NP; p++) {
            TData t;
            t.type = p < NI ? TDATA_INT : TDATA_FLOAT;
            if (p < NI) t.i = ii[p * N + o];
            else t.f = ff[(p - NI) * N + o];
            init[pname[p]] = t;
        }
        if (!km.CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], init)) return 3;
    }
    km.AfterInit();
    // the game logic's callbacks: they count what they receive
    int64_t n_prop = 0, n_rec = 0, n_rcpt = 0, n_hb = 0;
    if (consumer == 1)
        km.AddFrameCallBack(
            [&](const nfk_frame_host& f, const NFGUID*) {
                n_hb += f.n_fi;
                n_prop += f.n_ev;
                n_rec += f.n_re;
                n_rcpt += f.n_msgs;
            },
            NFK_READ_FIRED | NFK_READ_FIRED_GUID_ORDER | NFK_READ_EVENTS | NFK_READ_FANOUT);
    if (consumer == 0) {
    km.RegisterCommonPropertyEvent([&](const NFGUID&, const std::string&, const TData&, const TData&) {
        n_prop++;
        return 0;
    });
    km.RegisterCommonRecordEvent([&](const NFGUID&, const RECORD_EVENT_DATA&, const TData&, const TData&) {
        n_rec++;
        return 0;
    });
    km.AddPropertyEventCallBack([&](const NFGUID&, const std::string&, const TData&, const TData&,
                                    const std::vector<NFGUID>& to) {
        n_rcpt += (int64_t)to.size();
        return 0;
    });
    }
    OBJECT_SCHEDULE_FUNCTOR hb;
    if (consumer == 0)
        hb = [&](const NFGUID&, const std::string&, const float, const int) {
            n_hb++;
            return 0;
        };
    int32_t* s_obj = (int32_t*)A("s_obj")->data;
    int32_t* s_kind = (int32_t*)A("s_kind")->data;
    float* s_int = (float*)A("s_interval")->data;
    int32_t* s_cnt = (int32_t*)A("s_count")->data;
    int64_t* s_time = (int64_t*)A("s_time")->data;
    for (int64_t i = 0; i < NS; i++) {
        g_now = s_time[i];
        km.AddSchedule(NFGUID(gh[s_obj[i]], gd[s_obj[i]]), kname[s_kind[i]], hb, s_int[i], s_cnt[i]);
    }
    const double build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();

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

    std::vector<NFGPUKernelModule::FrameStats> st;
    std::vector<double> call_ms, frame_ms;
    int64_t xi = 0, hi = 0, ncalls = 0;
    std::vector<NFGUID> hg, xg;
    for (int t = 0; t < W + K; t++) {
        // the frame's calls as game logic makes them, NFGUIDs in hand (gathered from the workload's
        // object arrays before the timed region, as bench.py's host_calls leg does)
        hg.clear();
        xg.clear();
        for (int64_t j = hi; j < NH && h_tick[j] == t; j++) hg.emplace_back(gh[h_obj[j]], gd[h_obj[j]]);
        for (int64_t j = xi; j < NX && x_tick[j] == t; j++) xg.emplace_back(gh[x_obj[j]], gd[x_obj[j]]);
        const int64_t hi0 = hi, xi0 = xi;
        const auto t0 = std::chrono::steady_clock::now();
        for (; hi < NH && h_tick[hi] == t; hi++) {
            if (!calls) continue;
            const NFGUID& g = hg[(size_t)(hi - hi0)];
            g_now = h_time[hi];
            if (h_op[hi] == 1) km.AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
            else if (h_op[hi] == 2) km.RemoveSchedule(g, kname[h_kind[hi]]);
            else km.RemoveSchedule(g);
            ncalls += t >= W;
        }
        for (; xi < NX && x_tick[xi] == t; xi++) {
            if (!calls) continue;
            const NFGUID& g = xg[(size_t)(xi - xi0)];
            if (x_pid[xi] < NI) {
                km.SetPropertyInt(g, pname[x_pid[xi]], (int64_t)x_bits[xi]);
            } else {
                double v;
                memcpy(&v, &x_bits[xi], 8);
                km.SetPropertyFloat(g, pname[x_pid[xi]], v);
            }
            ncalls += t >= W;
        }
        const auto t1 = std::chrono::steady_clock::now();
        g_now = tick_time[t];
        km.Execute();
        const auto t2 = std::chrono::steady_clock::now();
        if (t >= W) {
            st.push_back(km.LastFrameStats());
            call_ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            frame_ms.push_back(std::chrono::duration<double, std::milli>(t2 - t0).count());
        }
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v.empty() ? 0.0 : v[v.size() / 2];
    };
    auto medf = [&](double NFGPUKernelModule::FrameStats::*m) {
        std::vector<double> v;
        for (auto& s : st) v.push_back(s.*m);
        return med(v);
    };
    const nfk_summary& s = km.LastSummary();
    printf("{\"plugin_frame_ms\": %.3f, \"entities\": %lld, \"entity_ticks_per_s\": %.4g, \"calls_per_frame\": %lld, "
           "\"phases_ms\": {\"calls\": %.3f, \"device\": %.3f, \"functors\": %.3f, \"events_read\": %.3f, "
           "\"deliver\": %.3f, \"functor_calls\": %.3f, \"execute\": %.3f, \"gather\": %.3f}, "
           "\"per_frame\": {\"fired\": %lld, \"prop_events\": %lld, \"rec_events\": %lld, \"messages\": %lld}, "
           "\"received\": {\"heartbeats\": %lld, \"prop_events\": %lld, \"recipients\": %lld}, \"build_s\": %.1f, "
           "\"frames\": %d, \"warmup\": %d, \"consumer\": \"%s\", \"threads\": \"%s\"}\n",
           med(frame_ms), (long long)N, (double)N / (med(frame_ms) * 1e-3), (long long)(K ? ncalls / K : 0),
           med(call_ms), medf(&NFGPUKernelModule::FrameStats::device), medf(&NFGPUKernelModule::FrameStats::functors),
           medf(&NFGPUKernelModule::FrameStats::events_read), medf(&NFGPUKernelModule::FrameStats::deliver),
           medf(&NFGPUKernelModule::FrameStats::calls), medf(&NFGPUKernelModule::FrameStats::total),
           medf(&NFGPUKernelModule::FrameStats::gather),
           (long long)s.n_fired, (long long)s.n_prop_events, (long long)s.n_rec_events, (long long)s.n_msgs,
           (long long)n_hb, (long long)n_prop, (long long)n_rcpt, build_s, K, W,
           consumer == 0 ? "per-call" : consumer == 1 ? "frame-batch" : "none",
           getenv("NFGPU_PLUGIN_THREADS") ? getenv("NFGPU_PLUGIN_THREADS") : "default");
    fflush(stdout);
    km.Shut();
    return 0;
}
