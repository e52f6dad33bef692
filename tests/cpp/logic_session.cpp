// logic_session.cpp — game logic written against the reference's plugin interfaces, run on two
// servers and logged the same way, so tests/test_logic_session.py can compare them frame by frame:
//
//   LOGIC_REF   the reference's own NFCKernelModule + NFCScheduleModule (with NFCSceneAOIModule,
//               NFCEventModule, NFCClassModule, NFCElementModule), compiled from /root/reference
//               where they lie — the heartbeat effect programs run as functors through
//               NFIKernelModule (as oracle/ref_session.cpp does);
//   (default)   the reference-side GPU plugin (integration/NFGPUKernelPlugin.cpp: NFGPUKernelAdapter +
//               NFGPUScheduleAdapter + NFGPUSceneAOIAdapter) in the same modules' place — the programs
//               run on the device.
//
// The logic uses what the reference's game modules use beyond the frame path:
//   * Tutorial3's own sequence (Tutorial/Tutorial3/HelloWorld3Module.cpp:40-110, restated): a class
//     callback on Player that, at COE_CREATE_HASDATA, registers an object event callback and a
//     functor-only heartbeat AddSchedule(self, "OnHeartBeat", 5.0f, 10); the object NFGUID(0, 10)
//     with the dynamic properties Hello (string) and World (int), per-object callbacks on both,
//     pObject->SetPropertyString / SetPropertyInt, and DoEvent(self, 1, [int, string]) whose
//     handler calls SetPropertyInt / SetPropertyString through NFIKernelModule — once at start and
//     once per frame;
//   * per-object callbacks (NFIKernelModule::AddPropertyCallBack / AddRecordCallBack,
//     NFIKernelModule.h:28-45) on every workload object's HP, MP, X, TargetX, Gold, Level and rec0;
//     the HP one also does what NFCNPCRefreshModule::OnObjectHPEvent does (NFCNPCRefreshModule.cpp:
//     113-124, restated): at newVar <= 0 the object is killed and a functor-only heartbeat
//     AddSchedule(self, "OnDeadDestroyHeart", 5.0f, 1) is added — so an HP that crosses 0 and recovers
//     within one frame kills only when the callbacks fire per accepted Set;
//   * the workload's window calls split between NFIKernelModule (SetProperty*, SetRecordInt,
//     ClearRecord) and the objects themselves (GetObject(self)->SetProperty*,
//     FindRecord(self, r)->SetInt / AddRow / Remove), read-modify-write Sets included; schedule
//     calls; DestroyObject and CreateObject after start.
//
// A workload's `logic_mode` bits (0 when absent) add:
//   1  cross-object reads in the heartbeat functors: after its effect each functor reads another object's
//      HP / X (NFIKernelModule::GetPropertyInt / Float) and MP through that object (GetObject(peer)->
//      GetPropertyInt), and its own HP, which a later schedule name of the same object may write —
//      NFCScheduleModule::Execute runs the functors object by object in NFGUID order (SM:52-80), so the
//      reference's read sees the Sets of the functors before it in the walk and none after;
//   2  (GPU plugin) NFGPUKernelModule::SetWalkOrderReads(true): those reads answered in walk order;
//   4  components (NFIComponent, run by NFCObject::Execute in NFCKernelModule::Execute's walk, KM:88-95,
//      NFCObject.cpp:42-47) that destroy their own object (deferred to the next Execute through
//      mtDeleteSelfList, KM:275-279 / KM:1434) or another object (at once);
//   8  NFCNPCRefreshModule's callbacks only (NFCNPCRefreshModule.cpp:98-105): every NPC gets
//      AddPropertyCallBack(self, "HP", ...) at creation and nothing else is watched — every NPC's HP
//      Sets fire callbacks, no record callbacks, no managers handed out;
//  16  only EXP watched (every object): with the set_ops programs, EXP's Sets in Poison depend on what the
//      earlier schedule names Patrol (SP, Camp) and HPRegen (HP) left in the same walk, kinds that write
//      no watched property themselves (the per-Set log must re-run them too).
//
// Logged per frame t: per-object property and record callbacks with the phase they fired in (0 =
// the window's calls, 1 = Execute), the heartbeat functors, Tutorial3's callback lines, the kills and
// OnDeadDestroyHeart calls, and every
// object's device properties and rec0 int cells read through the HOST objects
// (GetObject(self)->GetProperty*, FindRecord(self, r)->GetInt) and through NFIKernelModule.
//
// TEST INFRASTRUCTURE ONLY.  usage: logic_session <workload.nfio> <out.nfio>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#ifdef LOGIC_REF
#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCScheduleModule.h"
#include "NFComm/NFKernelPlugin/NFCSceneAOIModule.h"
#else
#include "../../integration/NFGPUKernelPlugin.cpp"
#endif
#include "NFComm/NFConfigPlugin/NFCClassModule.h"
#include "NFComm/NFConfigPlugin/NFCElementModule.h"
#include "NFComm/NFMessageDefine/NFProtocolDefine.hpp"
#include "../../oracle/nfio.h"
#include "../../oracle/ref_server.hpp"

// NFGetTime() (NFPlatform.h:367) reads CLOCK_REALTIME: the session's virtual clock, so both servers'
// schedules (NFCScheduleModule's and the device's) see the workload's call and frame times
extern "C" int clock_gettime(clockid_t clk, struct timespec* ts) {
    if (clk == CLOCK_REALTIME) {
        ts->tv_sec = g_now / 1000;
        ts->tv_nsec = (g_now % 1000) * 1000000;
        return 0;
    }
    return (int)syscall(SYS_clock_gettime, clk, ts);
}

static std::string cstr(const uint8_t* p) { return std::string((const char*)p, strnlen((const char*)p, 32)); }
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

struct Logic {
    NFIKernelModule* km = nullptr;
    NFIScheduleModule* sm = nullptr;
    NFIEventModule* em = nullptr;
    std::map<std::string, int> pid, kid;
    std::map<NFGUID, int> obj;
    int ni = 0, phase = 0, frame = -1;
    // per-object callbacks: (phase, obj, pid, old, new) / (phase, obj, rrc, old, new)
    std::vector<int32_t> pc_phase, pc_obj, pc_pid, rc_phase, rc_obj;
    std::vector<uint32_t> rc_rrc;
    std::vector<uint64_t> pc_old, pc_new, rc_old, rc_new;
    std::vector<int32_t> fi_obj, fi_kind, fi_rem;
    std::string t3;  // Tutorial3's callback lines
    std::string kills, dead;  // OnObjectHPEvent's kills, OnDeadDestroyHeart's calls
    std::string comp;         // the components' DestroyObject calls and the objects gone after Execute
    // (logic_mode 1) the functors' reads: reader, kind, peer, peer's HP / X / MP (through the object), own HP
    std::vector<int32_t> xr_obj, xr_kind, xr_peer;
    std::vector<uint64_t> xr_hp, xr_x, xr_mp, xr_self;
    int64_t mode = 0;
    void clear() {
        for (auto* v : {&pc_phase, &pc_obj, &pc_pid, &rc_phase, &rc_obj, &fi_obj, &fi_kind, &fi_rem, &xr_obj, &xr_kind, &xr_peer}) v->clear();
        rc_rrc.clear();
        for (auto* v : {&pc_old, &pc_new, &rc_old, &rc_new, &xr_hp, &xr_x, &xr_mp, &xr_self}) v->clear();
        t3.clear();
        kills.clear();
        dead.clear();
        comp.clear();
    }
    int ObjOf(const NFGUID& g) const {
        auto it = obj.find(g);
        return it == obj.end() ? -1 : it->second;
    }

    // ---- per-object callbacks on the workload objects ----
    int OnObjProp(const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {
        const int p = pid.at(name);
        pc_phase.push_back(phase);
        pc_obj.push_back(ObjOf(self));
        pc_pid.push_back(p);
        pc_old.push_back(p < ni ? (uint64_t)a.GetInt() : dbits(a.GetFloat()));
        pc_new.push_back(p < ni ? (uint64_t)b.GetInt() : dbits(b.GetFloat()));
        return 0;
    }
    int OnObjRecord(const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
        const uint32_t op = ev.nOpType == RECORD_EVENT_DATA::Add ? 1u : ev.nOpType == RECORD_EVENT_DATA::Del ? 2u
                          : ev.nOpType == RECORD_EVENT_DATA::Cover ? 3u : 0u;
        rc_phase.push_back(phase);
        rc_obj.push_back(ObjOf(self));
        rc_rrc.push_back((op << 24) | ((uint32_t)std::stoi(ev.strRecordName.substr(3)) << 16) | ((uint32_t)ev.nRow << 8) |
                         (uint32_t)ev.nCol);
        rc_old.push_back(op ? 0 : (uint64_t)a.GetInt());
        rc_new.push_back(op ? 0 : (uint64_t)b.GetInt());
        return 0;
    }
    // NFCNPCRefreshModule::OnObjectHPEvent (NFCNPCRefreshModule.cpp:113-124, restated without the
    // LastAttacker test: this schema has no object properties)
    int OnObjectHPEvent(const NFGUID& self, const std::string&, const NFIDataList::TData& a, const NFIDataList::TData& b) {
        if (b.GetInt() <= 0) {
            kills += std::to_string(ObjOf(self)) + " " + std::to_string(a.GetInt()) + " " + std::to_string(b.GetInt()) + "\n";
            sm->AddSchedule(self, "OnDeadDestroyHeart", this, &Logic::OnDeadDestroyHeart, 5.0f, 1);
        }
        return 0;
    }
    int OnDeadDestroyHeart(const NFGUID& self, const std::string&, const float, const int nCount) {  // :127
        dead += std::to_string(ObjOf(self)) + " " + std::to_string(nCount) + "\n";
        return 0;
    }
    void Watch(const NFGUID& g, bool npc) {
        if (mode & 16) {
            km->AddPropertyCallBack(g, "EXP", this, &Logic::OnObjProp);
            return;
        }
        if (mode & 8) {  // NFCNPCRefreshModule.cpp:104: the NPCs' HP, nothing else
            if (npc) {
                km->AddPropertyCallBack(g, "HP", this, &Logic::OnObjProp);
                km->AddPropertyCallBack(g, "HP", this, &Logic::OnObjectHPEvent);
            }
            return;
        }
        for (const char* n : {"HP", "MP", "X", "TargetX", "Gold", "Level"}) km->AddPropertyCallBack(g, n, this, &Logic::OnObjProp);
        km->AddPropertyCallBack(g, "HP", this, &Logic::OnObjectHPEvent);
        km->AddRecordCallBack(g, "rec0", this, &Logic::OnObjRecord);
    }
    // the heartbeat functor's log (both servers); the effect runs in Effect (reference) or on the device
    void Fired(const NFGUID& self, const std::string& name, int nCount) {
        fi_obj.push_back(ObjOf(self));
        fi_kind.push_back(kid.at(name));
        fi_rem.push_back(nCount);
    }

    // ---- Tutorial3 (HelloWorld3Module.cpp, restated) ----
    void Line(const std::string& s) { t3 += std::to_string(frame) + " " + s + "\n"; }
    int OnEvent(const NFGUID& self, const NFEventDefine event, const NFIDataList& arg) {  // :13-22
        Line("OnEvent " + std::to_string((int)event) + " " + std::to_string(self.nData64) + " " +
             std::to_string(arg.Int(0)) + " " + arg.String(1));
        const bool a = km->SetPropertyInt(self, "Hello", arg.Int(0));  // (a string property: refused)
        const bool b = km->SetPropertyString(self, "Hello", arg.String(1));
        Line(std::string("OnEvent sets ") + (a ? "1" : "0") + (b ? "1" : "0"));
        return 0;
    }
    int OnHeartBeat(const NFGUID& self, const std::string& name, const float fTime, const int nCount) {  // :24-34
        Line("OnHeartBeat " + std::to_string(self.nHead64) + "-" + std::to_string(self.nData64) + " " + name + " " +
             std::to_string(fTime) + " " + std::to_string(nCount));
        return 0;
    }
    int OnClassEvent(const NFGUID& self, const std::string& cls, const CLASS_OBJECT_EVENT event, const NFIDataList&) {  // :36-50
        Line("OnClassCallBackEvent " + cls + " " + std::to_string(self.nData64) + " " + std::to_string((int)event));
        if (event == COE_CREATE_HASDATA) {
            em->AddEventCallBack(self, NFEventDefine(1), this, &Logic::OnEvent);
            sm->AddSchedule(self, "OnHeartBeat", this, &Logic::OnHeartBeat, 5.0f, 10);
        }
        return 0;
    }
    int OnWorld(const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {  // :52-58
        Line("OnPropertyCallBackEvent " + std::to_string(self.nData64) + " " + name + " " + std::to_string(a.GetInt()) +
             " " + std::to_string(b.GetInt()));
        return 0;
    }
    int OnHello(const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {  // :60-66
        Line("OnPropertyStrCallBackEvent " + std::to_string(self.nData64) + " " + name + " " + a.GetString() + " " +
             b.GetString());
        return 0;
    }
    NFGUID t3_self;
    // (logic_mode 1) a functor's reads of another object and of itself, after its own effect
    void CrossReads(const NFGUID& self, const std::string& name, const NFGUID& peer) {
        xr_obj.push_back(ObjOf(self));
        xr_kind.push_back(kid.at(name));
        xr_peer.push_back(ObjOf(peer));
        xr_hp.push_back((uint64_t)km->GetPropertyInt(peer, "HP"));
        xr_x.push_back(dbits(km->GetPropertyFloat(peer, "X")));
        NF_SHARE_PTR<NFIObject> po = km->GetObject(peer);
        xr_mp.push_back(po ? (uint64_t)po->GetPropertyInt("MP") : 0);
        xr_self.push_back((uint64_t)km->GetPropertyInt(self, "HP"));
    }
    bool Tutorial3(int scene) {  // HelloWorld3Module::AfterInit (:68-100)
        km->AddClassCallBack(NFrame::Player::ThisName(), this, &Logic::OnClassEvent);
        NF_SHARE_PTR<NFIObject> o = km->CreateObject(NFGUID(0, 10), scene, 0, NFrame::Player::ThisName(), "", NFCDataList());
        if (!o) return false;
        t3_self = o->Self();
        o->GetPropertyManager()->AddProperty(o->Self(), "Hello", TDATA_STRING);
        o->GetPropertyManager()->AddProperty(o->Self(), "World", TDATA_INT);
        o->AddPropertyCallBack("Hello", this, &Logic::OnHello);
        o->AddPropertyCallBack("World", this, &Logic::OnWorld);
        o->SetPropertyString("Hello", "hello,World");
        o->SetPropertyInt("World", 1111);
        em->DoEvent(o->Self(), NFEventDefine(1), NFCDataList() << int(100) << "200");
        return true;
    }
};

// (logic_mode 4) NFCComponentManager::Execute runs it in NFCKernelModule::Execute's object walk
struct DestroyComponent : public NFIComponent {
    DestroyComponent(Logic* l, const NFGUID& self, const NFGUID& victim, int at)
        : NFIComponent(self, "DestroyComponent"), L(l), me(self), victim(victim), at(at) {}
    bool Execute() override {
        if (L->frame != at || done) return true;
        done = true;
        const bool ok = L->km->DestroyObject(victim);  // the reference defers its own object (KM:275)
        L->comp += "destroy " + std::to_string(L->ObjOf(me)) + " " + std::to_string(L->ObjOf(victim)) + " " +
                   std::to_string(ok ? 1 : 0) + "\n";
        return true;
    }
    Logic* L;
    NFGUID me, victim;
    int at;
    bool done = false;
};

int main(int argc, char** argv) {
    if (argc != 3) return 2;
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
    const int64_t N = cfg[0], NI = cfg[1], NF = cfg[2], NC = cfg[3], NK = cfg[4], NR = cfg[5], NS = cfg[6], NT = cfg[7];
    nfio_arr* lma = nfio_get(&wf, "logic_mode");
    const int64_t mode = lma ? ((int64_t*)lma->data)[0] : 0;
    nfio_arr* noa = nfio_get(&wf, "n_oprops");
    if ((noa && ((int64_t*)noa->data)[0]) || (nfio_get(&wf, "sw_tick") && A("sw_tick")->shape[0] > 0) || NR != 1) {
        fprintf(stderr, "logic_session: int/float properties, one record, no SwitchScene\n");
        return 5;
    }
    const int64_t NP = NI + NF;
    uint8_t* pnames = (uint8_t*)A("prop_names")->data;
    uint8_t* knames = (uint8_t*)A("kind_names")->data;
    nfk_op* ops = (nfk_op*)A("ops")->data;
    const int OPK = nfio_ops_per_kind(A("ops"));  // ops per kind in the file
    int32_t* nops = (int32_t*)A("n_ops")->data;
    std::vector<std::string> pname(NP), kname(NK), cname = {"NPC", "Player"};
    for (int p = 0; p < NP; p++) pname[p] = cstr(pnames + 32 * p);
    for (int k = 0; k < NK; k++) kname[k] = cstr(knames + 32 * k);
    uint8_t* rct = (uint8_t*)A("rec_ctype")->data;
    const int32_t rows = ((int32_t*)A("rec_rows")->data)[0], cols = ((int32_t*)A("rec_cols")->data)[0];
    for (int c = 0; c < cols; c++)
        if (rct[c]) {
            fprintf(stderr, "logic_session: int record columns only (NFCRecord::SetFloat, see test_oracle.py)\n");
            return 5;
        }

    TestPluginManager pm;
    write_class_schema(pm, wf, pname, cname, NI, NF, NC, NR);
    TestLogModule log;
    NFCClassModule classes(&pm);
    NFCElementModule elements(&pm);
#ifdef LOGIC_REF
    NFCKernelModule kernel(&pm);
    NFCScheduleModule sched(&pm);
    NFCSceneAOIModule aoi(&pm);
#else
    NFGPUKernelAdapter kernel(&pm);
    NFGPUScheduleAdapter sched(&pm);
    NFGPUSceneAOIAdapter aoi(&pm);
#endif
    NFCEventModule events(&pm);
    pm.AddModule(typeid(NFILogModule).name(), &log);
    pm.AddModule(typeid(NFIClassModule).name(), &classes);
    pm.AddModule(typeid(NFIElementModule).name(), &elements);
    pm.AddModule(typeid(NFIKernelModule).name(), &kernel);
    pm.AddModule(typeid(NFISceneAOIModule).name(), &aoi);
    pm.AddModule(typeid(NFIEventModule).name(), &events);
    pm.AddModule(typeid(NFIScheduleModule).name(), &sched);
    std::vector<NFIModule*> all = {&log, &classes, &elements, &kernel, &aoi, &events, &sched};
    std::vector<std::string> rname = {"rec0"};
#ifndef LOGIC_REF
    // each heartbeat name's device effect program (a logic module's Init); OnHeartBeat has none
    for (int k = 0; k < NK; k++)
        kernel.gpu_.AddHeartBeatProgram(kname[k], std::vector<nfk_op>(ops + k * OPK, ops + k * OPK + nops[k]),
                                        pname, rname);
#endif
#ifndef LOGIC_REF
    if (mode & 2) kernel.gpu_.SetWalkOrderReads(true);
#endif
    for (auto* m : all) m->Awake();
    for (auto* m : all) m->Init();
    Logic L;
    L.mode = mode;
    L.km = &kernel;
    L.sm = &sched;
    L.em = &events;
    L.ni = (int)NI;
    for (int p = 0; p < NP; p++) L.pid[pname[p]] = p;
    for (int k = 0; k < NK; k++) L.kid[kname[k]] = k;
    NFIKernelModule* km = &kernel;
    NFIScheduleModule* sm = &sched;

    int64_t* gh = (int64_t*)A("guid_head")->data;
    int64_t* gd = (int64_t*)A("guid_data")->data;
    int32_t* sc = (int32_t*)A("scene")->data;
    int32_t* gr = (int32_t*)A("group")->data;
    uint8_t* cl = (uint8_t*)A("cls")->data;
    int64_t* ii = (int64_t*)A("init_i")->data;
    double* ff = (double*)A("init_f")->data;
    nfio_arr* ba = nfio_get(&wf, "born");
    int32_t* born = ba ? (int32_t*)ba->data : nullptr;
    for (int64_t o = 0; o < N; o++) L.obj[NFGUID(gh[o], gd[o])] = (int)o;
    L.obj[NFGUID(0, 10)] = (int)N;  // Tutorial3's object
    {
        std::map<int, int> groups;
        for (int64_t o = 0; o < N; o++) groups[sc[o]] = std::max(groups[sc[o]], gr[o]);
        for (auto& kv : groups) {
            km->CreateScene(kv.first);
            for (int g = 1; g <= kv.second; g++)
                if (km->RequestGroupScene(kv.first) != g) return 3;
        }
    }
    auto create = [&](int64_t o) {
        NFCDataList arg;
        for (int p = 0; p < NP; p++) {
            if (pname[p] == "SceneID" || pname[p] == "GroupID") continue;
            arg.Add(pname[p]);
            if (p < NI) arg.Add((NFINT64)ii[p * N + o]);
            else arg.Add(ff[(p - NI) * N + o]);
        }
        return km->CreateObject(NFGUID(gh[o], gd[o]), sc[o], gr[o], cname[cl[o]], "", arg) != nullptr;
    };
    for (int64_t o = 0; o < N; o++)
        if ((!born || born[o] < 0) && !create(o)) return 3;
    uint64_t* cells0 = (uint64_t*)A("rec0_cells")->data;
    uint64_t* used0 = (uint64_t*)A("rec0_used")->data;
    auto fill_rows = [&](int64_t o) {  // creation-time rows (NFCRecord::AddRow)
        NF_SHARE_PTR<NFIRecord> R = km->GetObject(NFGUID(gh[o], gd[o]))->GetRecordManager()->GetElement("rec0");
        for (int row = 0; row < rows; row++) {
            if (!((used0[o] >> row) & 1)) continue;
            NFCDataList v;
            for (int c = 0; c < cols; c++) v.Add((NFINT64)cells0[((size_t)o * cols + c) * rows + row]);
            R->AddRow(row, v);
        }
    };
    for (int64_t o = 0; o < N; o++)
        if (!born || born[o] < 0) fill_rows(o);
    for (auto* m : all) m->AfterInit();
    for (auto* m : all) m->ReadyExecute();
    std::vector<uint8_t> alive(N, 1);
    if (born)
        for (int64_t o = 0; o < N; o++) alive[o] = born[o] < 0;
    for (int64_t o = 0; o < N; o++)
        if (alive[o]) L.Watch(NFGUID(gh[o], gd[o]), cl[o] == 0);
    nfio_arr* dta0 = nfio_get(&wf, "d_tick");
    if (mode & 4) {  // components on objects that live from the start and that the workload never destroys
        std::vector<uint8_t> keep(N, 1);
        if (dta0)
            for (int64_t i = 0; i < (int64_t)dta0->shape[0]; i++) keep[((int32_t*)A("d_obj")->data)[i]] = 0;
        for (int64_t o = 0; o < N; o++)
            if (!alive[o]) keep[o] = 0;
        for (int64_t o = 0; o + 20 < N; o++) {
            const NFGUID g(gh[o], gd[o]);
            NFGUID victim;
            int at = -1;
            if (o % 61 == 3 && keep[o]) {
                victim = g;  // itself
                at = 1 + (int)((o / 61) % std::max<int64_t>(NT - 2, 1));
            } else if (o % 61 == 10 && keep[o] && keep[o + 20]) {
                victim = NFGUID(gh[o + 20], gd[o + 20]);
                at = 2 + (int)((o / 61) % std::max<int64_t>(NT - 3, 1));
            }
            if (at < 0) continue;
            NF_SHARE_PTR<NFIObject> ob = km->GetObject(g);
            ob->GetComponentManager()->AddComponent("DestroyComponent", NF_SHARE_PTR<NFIComponent>(new DestroyComponent(&L, g, victim, at)));
        }
    }

    // the heartbeat functor: the effect program through NFIKernelModule on the reference; on the
    // device the program ran before the functor, which only logs
    std::function<int(const NFGUID&, const std::string&, const float, const int)> heartbeat =
        [&](const NFGUID& self, const std::string& name, const float, const int nCount) -> int {
        L.Fired(self, name, nCount);
        struct XR {  // (logic_mode 1) the reads after the functor's effect, either way it is made
            Logic& L;
            const NFGUID& self;
            const std::string& name;
            int64_t N;
            const int64_t *gh, *gd;
            ~XR() {
                if (!(L.mode & 1)) return;
                const int o = L.ObjOf(self);
                const int64_t q = (o * 7 + 3) % N;  // (random NFGUIDs: the peer is before or after it in the walk)
                L.CrossReads(self, name, NFGUID(gh[q], gd[q]));
            }
        } xr{L, self, name, N, gh, gd};
#ifdef LOGIC_REF
        const int k = L.kid.at(name);
        for (int i = 0; i < nops[k]; i++) {
            const nfk_op& op = ops[k * OPK + i];
            if (op.flags & NFK_GUARD) {  // the functor's `if (GetPropertyInt(self, g) ...)`
                const int64_t g = km->GetPropertyInt(self, pname[op.guard & 0xFFFF]);
                const int64_t h = (op.guard & NFK_GUARD_PROP) ? km->GetPropertyInt(self, pname[op.guard >> 19]) : NFK_GUARD_KVAL(op.guard);
                const int c = (op.guard >> 16) & 3;
                if (!(c == NFK_GUARD_GT0 ? g > h : c == NFK_GUARD_LE0 ? g <= h : c == NFK_GUARD_NE0 ? g != h : g == h))
                    continue;
            }
            if (op.code == NFK_OP_ISET) {
                km->SetPropertyInt(self, pname[op.dst], (op.flags & NFK_A_PROP) ? km->GetPropertyInt(self, pname[op.a]) : op.a);
            } else if (op.code == NFK_OP_FSET) {
                km->SetPropertyFloat(self, pname[op.dst], (op.flags & NFK_A_PROP) ? km->GetPropertyFloat(self, pname[op.a])
                                                                                  : bitsd((uint64_t)op.a));
            } else if (op.code == NFK_OP_IADD_CLAMP) {
                const std::string& d = pname[op.dst];
                const int64_t cur = km->GetPropertyInt(self, d);
                const int64_t a = (op.flags & NFK_A_PROP) ? km->GetPropertyInt(self, pname[op.a]) : op.a;
                const int64_t lo = (op.flags & NFK_LO_PROP) ? km->GetPropertyInt(self, pname[op.b]) : op.b;
                const int64_t hi = (op.flags & NFK_HI_PROP) ? km->GetPropertyInt(self, pname[op.c]) : op.c;
                int64_t v = (int64_t)((uint64_t)cur + (uint64_t)a);
                if (v < lo) v = lo;
                if (v > hi) v = hi;
                km->SetPropertyInt(self, d, v);
            } else if (op.code == NFK_OP_FLERP) {
                const std::string& d = pname[op.dst];
                const double x = km->GetPropertyFloat(self, d);
                const double t = km->GetPropertyFloat(self, pname[op.a]);
                const double dd = t - x;
                const double m = dd * bitsd((uint64_t)op.b);
                km->SetPropertyFloat(self, d, x + m);
            } else if (op.code == NFK_OP_FAFFINE) {
                const std::string& d = pname[op.dst];
                const double x = km->GetPropertyFloat(self, d);
                const double m = x * bitsd((uint64_t)op.a);
                km->SetPropertyFloat(self, d, m + bitsd((uint64_t)op.b));
            } else if (op.code == NFK_OP_RIADD_CLAMP) {
                NF_SHARE_PTR<NFIRecord> R = km->FindRecord(self, rname[op.dst >> 8]);
                const int col = op.dst & 255;
                for (int row = 0; R && row < R->GetRows(); row++) {
                    if (!R->IsUsed(row)) continue;
                    int64_t v = (int64_t)((uint64_t)km->GetRecordInt(self, "rec0", row, col) + (uint64_t)op.a);
                    if (v < op.b) v = op.b;
                    if (v > op.c) v = op.c;
                    km->SetRecordInt(self, "rec0", row, col, v);
                }
            }
        }
#endif
        return 0;
    };
    OBJECT_SCHEDULE_FUNCTOR_PTR hb(new OBJECT_SCHEDULE_FUNCTOR(heartbeat));
    int32_t* s_obj = (int32_t*)A("s_obj")->data;
    int32_t* s_kind = (int32_t*)A("s_kind")->data;
    float* s_int = (float*)A("s_interval")->data;
    int32_t* s_cnt = (int32_t*)A("s_count")->data;
    int64_t* s_time = (int64_t*)A("s_time")->data;
    for (int64_t i = 0; i < NS; i++) {
        g_now = s_time[i];
        sm->AddSchedule(NFGUID(gh[s_obj[i]], gd[s_obj[i]]), kname[s_kind[i]], hb, s_int[i], s_cnt[i]);
    }
    int64_t* tick_time = (int64_t*)A("tick_time")->data;
    g_now = tick_time[0] - 1000;
    L.frame = -1;
    if (!L.Tutorial3(sc[0])) return 4;
    const std::string t3_setup = L.t3;

    nfio_arr* xa = A("x_tick");
    const int64_t NX = (int64_t)xa->shape[0];
    int32_t* x_tick = (int32_t*)xa->data;
    int32_t* x_obj = (int32_t*)A("x_obj")->data;
    int32_t* x_pid = (int32_t*)A("x_pid")->data;
    uint64_t* x_bits = (uint64_t*)A("x_bits")->data;
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
    int32_t* r_row = NRS ? (int32_t*)A("r_row")->data : nullptr;
    int32_t* r_col = NRS ? (int32_t*)A("r_col")->data : nullptr;
    uint64_t* r_bits = NRS ? (uint64_t*)A("r_bits")->data : nullptr;
    nfio_arr* roa = NRS ? nfio_get(&wf, "r_op") : nullptr;
    uint8_t* r_op = roa ? (uint8_t*)roa->data : nullptr;
    uint64_t* r_vals = roa ? (uint64_t*)A("r_vals")->data : nullptr;
    nfio_arr* dta = nfio_get(&wf, "d_tick");
    const int64_t ND = dta ? (int64_t)dta->shape[0] : 0;
    int32_t* d_tick = ND ? (int32_t*)dta->data : nullptr;
    int32_t* d_obj = ND ? (int32_t*)A("d_obj")->data : nullptr;

    // (LOGIC_TIMING=1: seconds per phase on stderr)
    const bool timing = getenv("LOGIC_TIMING") != nullptr;
    double tm[4] = {0, 0, 0, 0};
    auto clk = [] { return std::chrono::steady_clock::now(); };
    auto since = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    nfio_writer w;
    if (nfio_wopen(&w, argv[2])) return 2;
    {
        std::vector<uint8_t> s(t3_setup.begin(), t3_setup.end());
        nfio_put1(&w, "t3_setup", NFIO_U8, s.data(), s.size(), 1);
    }
    int64_t xi = 0, hi = 0, di = 0, ri = 0;
    for (int t = 0; t < NT; t++) {
        auto tp = clk();
        L.clear();
        L.frame = t;
        L.phase = 0;
        g_now = tick_time[t] - 50;  // the window's calls, between the frames
        if (born)  // CreateObject after start
            for (int64_t o = 0; o < N; o++)
                if (born[o] == t) {
                    if (!create(o)) return 8;
                    alive[o] = 1;
                    L.Watch(NFGUID(gh[o], gd[o]), cl[o] == 0);
                }
        events.DoEvent(L.t3_self, NFEventDefine(1), NFCDataList() << (NFINT64)(1000 + t) << ("s" + std::to_string(t)));
        for (; hi < NH && h_tick[hi] == t; hi++) {
            const NFGUID g(gh[h_obj[hi]], gd[h_obj[hi]]);
            // (not on an object a component destroyed: NFCScheduleModule::AddSchedule has no object check,
            // SM:257, and would keep a schedule firing for an object that is gone; the plugin drops it)
            if (!alive[h_obj[hi]]) continue;
            g_now = h_time[hi];
            if (h_op[hi] == 1) sm->AddSchedule(g, kname[h_kind[hi]], hb, h_int[hi], h_cnt[hi]);
            else if (h_op[hi] == 2) sm->RemoveSchedule(g, kname[h_kind[hi]]);
            else sm->RemoveSchedule(g);
        }
        for (; xi < NX && x_tick[xi] == t; xi++) {
            const NFGUID g(gh[x_obj[xi]], gd[x_obj[xi]]);
            if (!alive[x_obj[xi]]) continue;
            const std::string& pn = pname[x_pid[xi]];
            const bool rmw = x_mode && x_mode[xi];
            const bool direct = xi % 3 == 1;  // GetObject(self)->SetProperty* (NFIObject.h)
            NF_SHARE_PTR<NFIObject> ob = km->GetObject(g);
            if (x_pid[xi] < NI) {
                const int64_t cur = direct ? ob->GetPropertyInt(pn) : km->GetPropertyInt(g, pn);
                const int64_t v = rmw ? (int64_t)((uint64_t)cur + x_bits[xi]) : (int64_t)x_bits[xi];
                if (direct) ob->SetPropertyInt(pn, v);
                else km->SetPropertyInt(g, pn, v);
            } else {
                const double cur = direct ? ob->GetPropertyFloat(pn) : km->GetPropertyFloat(g, pn);
                const double v = rmw ? cur + bitsd(x_bits[xi]) : bitsd(x_bits[xi]);
                if (direct) ob->SetPropertyFloat(pn, v);
                else km->SetPropertyFloat(g, pn, v);
            }
        }
        for (; ri < NRS && r_tick[ri] == t; ri++) {
            const NFGUID g(gh[r_obj[ri]], gd[r_obj[ri]]);
            if (!alive[r_obj[ri]]) continue;
            NF_SHARE_PTR<NFIRecord> R = km->FindRecord(g, "rec0");
            const int op = r_op ? r_op[ri] : 0;
            if (op == 1) {  // NFCRecord::AddRow on the object's record
                NFCDataList v;
                for (int c = 0; c < cols; c++) v.Add((NFINT64)r_vals[ri * NFK_MAX_REC_COLS + c]);
                R->AddRow(r_row[ri], v);
            } else if (op == 2) {
                R->Remove(r_row[ri]);
            } else if (op == 3) {
                km->ClearRecord(g, "rec0");  // KM:492
            } else if (ri % 2) {
                R->SetInt(r_row[ri], r_col[ri], (int64_t)r_bits[ri]);  // FindRecord(self, r)->SetInt
            } else {
                km->SetRecordInt(g, "rec0", r_row[ri], r_col[ri], (int64_t)r_bits[ri]);  // KM:505
            }
        }
        for (; di < ND && d_tick[di] == t; di++) {  // DestroyObject (KM:273)
            if (!km->DestroyObject(NFGUID(gh[d_obj[di]], gd[d_obj[di]]))) return 9;
            alive[d_obj[di]] = 0;
        }
        g_now = tick_time[t];
        L.phase = 1;
        tm[0] += since(tp);
        tp = clk();
        for (auto* m : all) m->Execute();
        tm[1] += since(tp);
        tp = clk();
        if (mode & 4)  // the objects the components destroyed (their own: at the next Execute)
            for (int64_t o = 0; o < N; o++)
                if (alive[o] && !km->GetObject(NFGUID(gh[o], gd[o]))) {
                    alive[o] = 0;
                    L.comp += "gone " + std::to_string(o) + "\n";
                }
        char nm[48];
#define PUT(pfx, s, code, vec, es) snprintf(nm, sizeof nm, "%s_t%d_%s", pfx, t, s); nfio_put1(&w, nm, code, vec.data(), vec.size(), es);
        PUT("pc", "phase", NFIO_I32, L.pc_phase, 4);
        PUT("pc", "obj", NFIO_I32, L.pc_obj, 4);
        PUT("pc", "pid", NFIO_I32, L.pc_pid, 4);
        PUT("pc", "old", NFIO_U64, L.pc_old, 8);
        PUT("pc", "new", NFIO_U64, L.pc_new, 8);
        PUT("rc", "phase", NFIO_I32, L.rc_phase, 4);
        PUT("rc", "obj", NFIO_I32, L.rc_obj, 4);
        PUT("rc", "rrc", NFIO_U32, L.rc_rrc, 4);
        PUT("rc", "old", NFIO_U64, L.rc_old, 8);
        PUT("rc", "new", NFIO_U64, L.rc_new, 8);
        PUT("fi", "obj", NFIO_I32, L.fi_obj, 4);
        PUT("fi", "kind", NFIO_I32, L.fi_kind, 4);
        PUT("fi", "rem", NFIO_I32, L.fi_rem, 4);
        std::vector<uint8_t> t3(L.t3.begin(), L.t3.end());
        PUT("t3", "log", NFIO_U8, t3, 1);
        std::vector<uint8_t> kl(L.kills.begin(), L.kills.end()), dl(L.dead.begin(), L.dead.end());
        PUT("k", "kills", NFIO_U8, kl, 1);
        PUT("k", "dead", NFIO_U8, dl, 1);
        std::vector<uint8_t> cp(L.comp.begin(), L.comp.end());
        PUT("k", "comp", NFIO_U8, cp, 1);
        PUT("xr", "obj", NFIO_I32, L.xr_obj, 4);
        PUT("xr", "kind", NFIO_I32, L.xr_kind, 4);
        PUT("xr", "peer", NFIO_I32, L.xr_peer, 4);
        PUT("xr", "hp", NFIO_U64, L.xr_hp, 8);
        PUT("xr", "x", NFIO_U64, L.xr_x, 8);
        PUT("xr", "mp", NFIO_U64, L.xr_mp, 8);
        PUT("xr", "self", NFIO_U64, L.xr_self, 8);
        // every object's properties through the host object and through NFIKernelModule, and its
        // rec0 used rows' int cells through the host record
        std::vector<uint64_t> vh((size_t)NP * N, 0), vk((size_t)NP * N, 0), rv((size_t)N * cols * rows, 0), ru(N, 0);
        std::vector<uint64_t> rk((size_t)N * cols * rows, 0);  // (the same cells through NFIKernelModule::GetRecordInt)
        for (int64_t o = 0; o < N; o++) {
            if (!alive[o]) continue;
            const NFGUID g(gh[o], gd[o]);
            NF_SHARE_PTR<NFIObject> ob = km->GetObject(g);
            for (int p = 0; p < NP; p++) {
                vh[(size_t)p * N + o] = p < NI ? (uint64_t)ob->GetPropertyInt(pname[p]) : dbits(ob->GetPropertyFloat(pname[p]));
                vk[(size_t)p * N + o] = p < NI ? (uint64_t)km->GetPropertyInt(g, pname[p]) : dbits(km->GetPropertyFloat(g, pname[p]));
            }
            NF_SHARE_PTR<NFIRecord> R = ob->GetRecordManager()->GetElement("rec0");
            for (int row = 0; row < rows; row++) {
                if (!R->IsUsed(row)) continue;
                ru[o] |= 1ull << row;
                for (int c = 0; c < cols; c++) {
                    rv[((size_t)o * cols + c) * rows + row] = (uint64_t)R->GetInt(row, c);
                    rk[((size_t)o * cols + c) * rows + row] = (uint64_t)km->GetRecordInt(g, "rec0", row, c);
                }
            }
        }
        PUT("v", "host", NFIO_U64, vh, 8);
        PUT("v", "kernel", NFIO_U64, vk, 8);
        PUT("r", "cells", NFIO_U64, rv, 8);
        PUT("r", "used", NFIO_U64, ru, 8);
        PUT("r", "kcells", NFIO_U64, rk, 8);
        tm[2] += since(tp);
    }
    if (timing) fprintf(stderr, "logic_session: window calls %.2f s, Execute %.2f s, logging %.2f s\n", tm[0], tm[1], tm[2]);
    nfio_wclose(&w);
    fflush(stdout);
    _exit(0);  // (static destructors: NFMemoryCounter's static map dies before the modules' objects)
}
