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
// Per-frame mode (a frames.nfio path): the window's calls also include CreateObject after start,
// SwitchScene (KM:901-951), DestroyObject (KM:273-308), SetRecordInt and the record row operations
// (NFCRecord::AddRow / Remove, KM:492 ClearRecord), and every frame writes what the reference's
// modules raised: the common property / record events in call order (the creation-time events of an
// object being created excluded), the heartbeat functors in walk order, and, at the frame's end, the
// compiled NFCSceneAOIModule::GetBroadCastObject list (AOI:531-593) of every (object, property /
// record) with an event.  The AOI module's own common callbacks are unregistered in this mode: its
// OnGroupEvent releases a group a player leaves (AOI:389-393), a side effect outside the frame path.
//
// usage: nf_ref_session <workload.nfio> <ticks> <warmup> [final.nfio [frames.nfio]]
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

// the reference's kernel module, able to drop the common callbacks registered so far (protected
// lists of NFCKernelModule.h:174-178)
struct FrameKernel : NFCKernelModule {
    using NFCKernelModule::NFCKernelModule;
    void DropCommonCallbacks() {
        mtCommonClassCallBackList.clear();
        mtCommonPropertyCallBackList.clear();
        mtCommonRecordCallBackList.clear();
    }
};
// the compiled GetBroadCastObject (a protected member of NFCSceneAOIModule)
struct AOIProbe : NFCSceneAOIModule {
    using NFCSceneAOIModule::NFCSceneAOIModule;
    using NFCSceneAOIModule::GetBroadCastObject;
};

// what the reference raised in one frame (per-frame mode)
struct FrameLog {
    std::map<NFGUID, int> obj;
    std::map<std::string, int> pid, rid;
    int ni = 0, nf = 0;
    bool creating = false;
    std::vector<int32_t> pe_obj, pe_pid, rr_obj, fi_obj, fi_kind, fi_rem;
    std::vector<uint32_t> rr_rrc;
    std::vector<uint64_t> pe_old, pe_new, pe_oldh, pe_newh, rr_old, rr_new;
    void clear() {
        for (auto* v : {&pe_obj, &pe_pid, &rr_obj, &fi_obj, &fi_kind, &fi_rem}) v->clear();
        rr_rrc.clear();
        for (auto* v : {&pe_old, &pe_new, &pe_oldh, &pe_newh, &rr_old, &rr_new}) v->clear();
    }
    int OnProp(const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {
        auto o = obj.find(self);
        auto p = pid.find(name);
        if (creating || o == obj.end() || p == pid.end()) return 0;
        pe_obj.push_back(o->second);
        pe_pid.push_back(p->second);
        if (p->second < ni) {
            pe_old.push_back((uint64_t)a.GetInt());
            pe_new.push_back((uint64_t)b.GetInt());
            pe_oldh.push_back(0);
            pe_newh.push_back(0);
        } else if (p->second < ni + nf) {
            pe_old.push_back(dbits(a.GetFloat()));
            pe_new.push_back(dbits(b.GetFloat()));
            pe_oldh.push_back(0);
            pe_newh.push_back(0);
        } else {
            pe_old.push_back((uint64_t)a.GetObject().nData64);
            pe_new.push_back((uint64_t)b.GetObject().nData64);
            pe_oldh.push_back((uint64_t)a.GetObject().nHead64);
            pe_newh.push_back((uint64_t)b.GetObject().nHead64);
        }
        return 0;
    }
    int OnRecord(const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
        auto o = obj.find(self);
        auto r = rid.find(ev.strRecordName);
        if (creating || o == obj.end() || r == rid.end()) return 0;
        const uint32_t op = ev.nOpType == RECORD_EVENT_DATA::Add ? 1u : ev.nOpType == RECORD_EVENT_DATA::Del ? 2u
                          : ev.nOpType == RECORD_EVENT_DATA::Cover ? 3u : 0u;
        rr_obj.push_back(o->second);
        rr_rrc.push_back((op << 24) | ((uint32_t)r->second << 16) | ((uint32_t)ev.nRow << 8) | (uint32_t)ev.nCol);
        rr_old.push_back(op ? 0 : a.GetType() == TDATA_INT ? (uint64_t)a.GetInt() : dbits(a.GetFloat()));
        rr_new.push_back(op ? 0 : b.GetType() == TDATA_INT ? (uint64_t)b.GetInt() : dbits(b.GetFloat()));
        return 0;
    }
};

int main(int argc, char** argv) {
    if (argc < 4 || argc > 6) {
        fprintf(stderr, "usage: nf_ref_session <workload.nfio> <ticks> <warmup> [final.nfio [frames.nfio]]\n");
        return 2;
    }
    const bool per_frame = argc == 6;
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
    if (!per_frame && (has_rows("sw_tick") || has_rows("d_tick") || nfio_get(&wf, "born") || has_rows("r_tick"))) {
        fprintf(stderr, "nf_ref_session: membership changes and record calls are replayed in per-frame mode only\n");
        return 5;
    }
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    const int OPK = nfio_ops_per_kind(A("ops"));  // ops per kind in the file
    int32_t* nops = (int32_t*)A("n_ops")->data;
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) pname[p] = cstr(pnames + 32 * p);
    for (int k = 0; k < NK; k++) kname[k] = cstr(knames + 32 * k);
    for (int k = 0; k < NK; k++)
        for (int i = 0; i < nops[k]; i++)
            if (ops[k * OPK + i].code == NFK_OP_RFAFFINE) {
                fprintf(stderr, "nf_ref_session: record f64 ops cannot run on the reference (NFCRecord::SetFloat, "
                                "see nf_ref_harness --repro-record-float)\n");
                return 3;
            }

    TestPluginManager pm;
    write_class_schema(pm, wf, pname, cname, NI, NF, NC, NR);
    TestLogModule log;
    NFCClassModule classes(&pm);
    NFCElementModule elements(&pm);
    FrameKernel kernel(&pm);
    AOIProbe aoi(&pm);
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
    for (auto* m : all) {
        m->Init();
        if (per_frame && m == &aoi) kernel.DropCommonCallbacks();  // (only the AOI module's so far)
    }
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
    nfio_arr* ba = nfio_get(&wf, "born");
    int32_t* born = ba ? (int32_t*)ba->data : nullptr;
    nfio_arr* swa = nfio_get(&wf, "sw_tick");
    const int64_t NSW = swa ? (int64_t)swa->shape[0] : 0;
    int32_t* sw_tick = NSW ? (int32_t*)swa->data : nullptr;
    int32_t* sw_obj = NSW ? (int32_t*)A("sw_obj")->data : nullptr;
    int32_t* sw_scene = NSW ? (int32_t*)A("sw_scene")->data : nullptr;
    int32_t* sw_group = NSW ? (int32_t*)A("sw_group")->data : nullptr;
    float* sw_x = NSW ? (float*)A("sw_x")->data : nullptr;
    float* sw_y = NSW ? (float*)A("sw_y")->data : nullptr;
    float* sw_z = NSW ? (float*)A("sw_z")->data : nullptr;
    {  // scenes and their groups 1..G (CreateScene / RequestGroupScene, KM:981, 1104), the SwitchScene
       // targets' included
        std::map<int, int> groups;
        for (int64_t o = 0; o < N; o++) groups[sc[o]] = std::max(groups[sc[o]], gr[o]);
        for (int64_t i = 0; i < NSW; i++)
            if (sw_scene[i] >= 0) groups[sw_scene[i]] = std::max(groups[sw_scene[i]], sw_group[i]);
        for (auto& kv : groups) {
            km->CreateScene(kv.first);
            for (int g = 1; g <= kv.second; g++)
                if (km->RequestGroupScene(kv.first) != g) return 3;
        }
    }
    FrameLog fl;
    fl.ni = (int)NI;
    fl.nf = (int)NF;
    for (int p = 0; p < NP; p++) fl.pid[pname[p]] = p;
    for (int r = 0; r < NR; r++) fl.rid["rec" + std::to_string(r)] = r;
    for (int64_t o = 0; o < N; o++) fl.obj[NFGUID(gh[o], gd[o])] = (int)o;
    auto create = [&](int64_t o) {  // NFCKernelModule::CreateObject (KM:101) with the workload's values
        NFCDataList arg;
        for (int p = 0; p < NP; p++) {
            if (pname[p] == "SceneID" || pname[p] == "GroupID") continue;
            arg.Add(pname[p]);
            if (p < NI) arg.Add((NFINT64)ii[p * N + o]);
            else if (p < NI + NF) arg.Add(ff[(p - NI) * N + o]);
            else arg.Add(NFGUID(ioh[(p - NI - NF) * N + o], iod[(p - NI - NF) * N + o]));
        }
        fl.creating = true;
        const bool ok = km->CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], "", arg) != nullptr;
        fl.creating = false;
        return ok;
    };
    for (int64_t o = 0; o < N; o++)
        if ((!born || born[o] < 0) && !create(o)) return 3;
    for (int r = 0; r < NR; r++) {  // creation-time record rows
        char nm[32];
        snprintf(nm, sizeof nm, "rec%d_cells", r);
        uint64_t* cells = (uint64_t*)A(nm)->data;
        snprintf(nm, sizeof nm, "rec%d_used", r);
        uint64_t* used = (uint64_t*)A(nm)->data;
        const int32_t rows = ((int32_t*)A("rec_rows")->data)[r], cols = ((int32_t*)A("rec_cols")->data)[r];
        uint8_t* ct = (uint8_t*)A("rec_ctype")->data;
        for (int64_t o = 0; o < N; o++) {
            if (born && born[o] >= 0) continue;
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
    if (per_frame) {
        km->RegisterCommonPropertyEvent(&fl, &FrameLog::OnProp);
        km->RegisterCommonRecordEvent(&fl, &FrameLog::OnRecord);
    }
    for (auto* m : all) m->ReadyExecute();

    // the heartbeat functor: the name's effect program through NFIKernelModule, as game logic
    // written against the reference would run it (the oracle's arithmetic, same operation order)
    std::map<std::string, int> kid;
    for (int k = 0; k < NK; k++) kid[kname[k]] = k;
    std::vector<std::string> rname;
    for (int r = 0; r < NR; r++) rname.push_back("rec" + std::to_string(r));
    int64_t fired = 0;
    auto heartbeat = [&](const NFGUID& self, const std::string& name, const float, const int nCount) -> int {
        fired++;
        const int k = kid.at(name);
        if (per_frame) {
            fl.fi_obj.push_back(fl.obj.at(self));
            fl.fi_kind.push_back(k);
            fl.fi_rem.push_back(nCount);
        }
        for (int i = 0; i < nops[k]; i++) {
            const nfk_op& op = ops[k * OPK + i];
            if (op.flags & NFK_GUARD) {
                const int64_t g = km->GetPropertyInt(self, pname[op.guard & 0xFFFF]);
                const int64_t h = (op.guard & NFK_GUARD_PROP) ? km->GetPropertyInt(self, pname[op.guard >> 19]) : NFK_GUARD_KVAL(op.guard);
                const int c = (op.guard >> 16) & 3;
                if (!(c == NFK_GUARD_GT0 ? g > h : c == NFK_GUARD_LE0 ? g <= h : c == NFK_GUARD_NE0 ? g != h : g == h))
                    continue;
            }
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
            case NFK_OP_ISET:
                km->SetPropertyInt(self, pname[op.dst],
                                   (op.flags & NFK_A_PROP) ? km->GetPropertyInt(self, pname[op.a]) : op.a);
                break;
            case NFK_OP_FSET:
                km->SetPropertyFloat(self, pname[op.dst], (op.flags & NFK_A_PROP) ? km->GetPropertyFloat(self, pname[op.a])
                                                                                  : bitsd((uint64_t)op.a));
                break;
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

    nfio_arr* rsa = nfio_get(&wf, "r_tick");
    const int64_t NRS = rsa ? (int64_t)rsa->shape[0] : 0;
    int32_t* r_tick = NRS ? (int32_t*)rsa->data : nullptr;
    int32_t* r_obj = NRS ? (int32_t*)A("r_obj")->data : nullptr;
    int32_t* r_rec = NRS ? (int32_t*)A("r_rec")->data : nullptr;
    int32_t* r_row = NRS ? (int32_t*)A("r_row")->data : nullptr;
    int32_t* r_col = NRS ? (int32_t*)A("r_col")->data : nullptr;
    uint64_t* r_bits = NRS ? (uint64_t*)A("r_bits")->data : nullptr;
    nfio_arr* roa = NRS ? nfio_get(&wf, "r_op") : nullptr;
    uint8_t* r_op = roa ? (uint8_t*)roa->data : nullptr;
    uint64_t* r_vals = roa ? (uint64_t*)A("r_vals")->data : nullptr;
    uint8_t* r_ct = NR ? (uint8_t*)A("rec_ctype")->data : nullptr;
    nfio_arr* dta = nfio_get(&wf, "d_tick");
    const int64_t ND = dta ? (int64_t)dta->shape[0] : 0;
    int32_t* d_tick = ND ? (int32_t*)dta->data : nullptr;
    int32_t* d_obj = ND ? (int32_t*)A("d_obj")->data : nullptr;
    std::vector<uint8_t> alive(N, 1);
    if (born)
        for (int64_t o = 0; o < N; o++) alive[o] = born[o] < 0;
    std::vector<int32_t> cur_scene(sc, sc + N), cur_group(gr, gr + N);
    nfio_writer fw;
    if (per_frame && nfio_wopen(&fw, argv[5])) return 2;

    using clk = std::chrono::steady_clock;
    clk::time_point t0 = clk::now();
    int64_t ev0 = 0, msg0 = 0, re0 = 0, fi0 = 0;
    int64_t xi = 0, hi = 0, swi = 0, ri = 0, di = 0;
    for (int64_t t = 0; t < NT; t++) {
        fl.clear();
        // the window's calls in the workload's order (oracle/nf_oracle.c): CreateObject, SwitchScene,
        // schedule calls, SetProperty*, record calls, DestroyObject
        if (born)
            for (int64_t o = 0; o < N; o++)
                if (born[o] == t) {
                    if (!create(o)) return 8;
                    alive[o] = 1;
                }
        for (; swi < NSW && sw_tick[swi] == t; swi++) {
            const int o = sw_obj[swi];
            const int ns = sw_scene[swi] < 0 ? cur_scene[o] : sw_scene[swi];
            const int ng = sw_scene[swi] < 0 ? cur_group[o] : sw_group[swi];
            if (!km->SwitchScene(NFGUID(gh[o], gd[o]), ns, ng, sw_x[swi], sw_y[swi], sw_z[swi], 0.0f, NFCDataList()))
                return 11;
            cur_scene[o] = ns;
            cur_group[o] = ng;
        }
        if (t == W) {  // the timed frames start here
            t0 = clk::now();
            ev0 = net.events;
            msg0 = net.msgs;
            re0 = net.rec_events;
            fi0 = fired;
        }
        for (; hi < NH && h_tick[hi] == t; hi++) {
            // (a call on an object that is not in the world — destroyed, or not yet created — is
            // not made: the reference's NFCScheduleModule would keep a schedule for a GUID that no
            // longer names an object, SM:257)
            if (!alive[h_obj[hi]]) continue;
            const NFGUID g(gh[h_obj[hi]], gd[h_obj[hi]]);
            g_now = h_time[hi];
            if (h_op[hi] == 1) sm->AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
            else if (h_op[hi] == 2) sm->RemoveSchedule(g, kname[h_kind[hi]]);
            else sm->RemoveSchedule(g);
        }
        for (; xi < NX && x_tick[xi] == t; xi++) {
            if (!alive[x_obj[xi]]) continue;  // "There is no object" (KM:331)
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
        for (; ri < NRS && r_tick[ri] == t; ri++) {
            const int o = r_obj[ri];
            if (!alive[o]) continue;
            const NFGUID g(gh[o], gd[o]);
            const std::string rn = "rec" + std::to_string(r_rec[ri]);
            NF_SHARE_PTR<NFIRecord> R = km->FindRecord(g, rn);
            const int op = r_op ? r_op[ri] : 0;
            if (op == 1) {  // NFCRecord::AddRow (RC:111)
                NFCDataList v;
                for (int c = 0; R && c < R->GetCols(); c++) {
                    const uint64_t b = r_vals[ri * NFK_MAX_REC_COLS + c];
                    if (r_ct[r_rec[ri] * NFK_MAX_REC_COLS + c]) v.Add(bitsd(b));
                    else v.Add((NFINT64)b);
                }
                if (R) R->AddRow(r_row[ri], v);
            } else if (op == 2) {
                if (R) R->Remove(r_row[ri]);  // RC:1086
            } else if (op == 3) {
                km->ClearRecord(g, rn);  // KM:492
            } else if (r_ct[r_rec[ri] * NFK_MAX_REC_COLS + r_col[ri]]) {
                fprintf(stderr, "nf_ref_session: SetRecordFloat cannot run on the reference (NFCRecord::SetFloat)\n");
                return 3;
            } else {
                km->SetRecordInt(g, rn, r_row[ri], r_col[ri], (int64_t)r_bits[ri]);  // KM:505
            }
        }
        for (; di < ND && d_tick[di] == t; di++) {  // DestroyObject (KM:273)
            if (!km->DestroyObject(NFGUID(gh[d_obj[di]], gd[d_obj[di]]))) return 9;
            alive[d_obj[di]] = 0;
        }
        g_now = tick_time[t];
        for (auto* m : all) m->Execute();  // NFCScheduleModule::Execute walks the schedules (SM:49)
        if (per_frame) {
            // recipients at the frame's end: the compiled GetBroadCastObject of every (object, key)
            // with an event (key = property id, or 0x10000 | record id)
            std::map<std::pair<int, int>, std::string> keys;
            for (size_t i = 0; i < fl.pe_obj.size(); i++)
                if (alive[fl.pe_obj[i]]) keys[{fl.pe_obj[i], fl.pe_pid[i]}] = pname[fl.pe_pid[i]];
            for (size_t i = 0; i < fl.rr_obj.size(); i++)
                if (alive[fl.rr_obj[i]]) {
                    const int r = (fl.rr_rrc[i] >> 16) & 0xFF;
                    keys[{fl.rr_obj[i], 0x10000 | r}] = "rec" + std::to_string(r);
                }
            std::vector<int32_t> bo, bk, rc;
            std::vector<uint32_t> boff;
            for (auto& kv : keys) {
                NFCDataList to;
                aoi.GetBroadCastObject(NFGUID(gh[kv.first.first], gd[kv.first.first]), kv.second,
                                       (kv.first.second & 0x10000) != 0, to);
                bo.push_back(kv.first.first);
                bk.push_back(kv.first.second);
                boff.push_back((uint32_t)rc.size());
                for (int i = 0; i < to.GetCount(); i++) rc.push_back(fl.obj.at(to.Object(i)));
            }
            boff.push_back((uint32_t)rc.size());
            char nm[40];
#define FPUT(pfx, s, code, vec, es) snprintf(nm, sizeof nm, "%s_t%d_%s", pfx, (int)t, s); nfio_put1(&fw, nm, code, vec.data(), vec.size(), es);
            FPUT("pe", "obj", NFIO_I32, fl.pe_obj, 4);
            FPUT("pe", "pid", NFIO_I32, fl.pe_pid, 4);
            FPUT("pe", "old", NFIO_U64, fl.pe_old, 8);
            FPUT("pe", "new", NFIO_U64, fl.pe_new, 8);
            FPUT("pe", "oldh", NFIO_U64, fl.pe_oldh, 8);
            FPUT("pe", "newh", NFIO_U64, fl.pe_newh, 8);
            FPUT("rr", "obj", NFIO_I32, fl.rr_obj, 4);
            FPUT("rr", "rrc", NFIO_U32, fl.rr_rrc, 4);
            FPUT("rr", "old", NFIO_U64, fl.rr_old, 8);
            FPUT("rr", "new", NFIO_U64, fl.rr_new, 8);
            FPUT("fi", "obj", NFIO_I32, fl.fi_obj, 4);
            FPUT("fi", "kind", NFIO_I32, fl.fi_kind, 4);
            FPUT("fi", "rem", NFIO_I32, fl.fi_rem, 4);
            FPUT("bc", "obj", NFIO_I32, bo, 4);
            FPUT("bc", "key", NFIO_I32, bk, 4);
            FPUT("bc", "off", NFIO_U32, boff, 4);
            FPUT("bc", "rcpt", NFIO_I32, rc, 4);
            std::vector<uint8_t> al(alive);
            FPUT("al", "ive", NFIO_U8, al, 1);
        }
    }
    if (per_frame) nfio_wclose(&fw);
    const double sec = std::chrono::duration<double>(clk::now() - t0).count();
    const int64_t frames = NT - W;
    printf("{\"entity_ticks_per_s\": %.6g, \"ms_per_frame\": %.4f, \"frames\": %lld, \"warmup\": %lld, "
           "\"entities\": %lld, \"fired\": %lld, \"events\": %lld, \"rec_events\": %lld, \"msgs\": %lld, "
           "\"seconds\": %.3f, \"log_errors\": %d}\n",
           frames > 0 ? (double)N * frames / sec : 0.0, frames > 0 ? 1000.0 * sec / frames : 0.0, (long long)frames,
           (long long)W, (long long)N, (long long)(fired - fi0), (long long)(net.events - ev0),
           (long long)(net.rec_events - re0), (long long)(net.msgs - msg0), sec, log.errors);
    fflush(stdout);
    if (argc >= 5) {  // the final state through NFIKernelModule::GetProperty* (the oracle cross-check)
        std::vector<int64_t> fi((size_t)NI * N, 0);
        std::vector<double> fff((size_t)NF * N, 0.0);
        for (int64_t o = 0; o < N; o++) {
            if (!alive[o]) continue;  // (objects no longer in the world read 0, as the oracle's)
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
