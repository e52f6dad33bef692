// NFGPUKernelPlugin.cpp — the REFERENCE-SIDE plugin a NoahGameFrame maintainer adds to swap the
// MI355X frame path in for NFKernelPlugin.  It compiles against the reference's
// own headers and links against libnfgpu_plugin.so / libnfgpu.so plus the reference's NFCore and
// NFKernelPlugin objects; tests/cpp/adapter_session.cpp runs it that way (tests/test_adapter.py).
//
//   NFGPUKernelAdapter    NFIKernelModule (NFIKernelModule.h:103-148) as a subclass of the reference's
//                         NFCKernelModule: the int / float / object properties and the int / float
//                         records of the class schema live on the device (nfgpu::NFGPUKernelModule);
//                         strings, vectors, object lists, scenes and class events stay in the host
//                         NFCKernelModule.  The schema is read from NFIClassModule in AfterInit.
//   NFGPUSceneAOIAdapter  NFISceneAOIModule as a subclass of the reference's NFCSceneAOIModule: a device
//                         property / record event reaches its OnPropertyEvent / OnRecordEvent
//                         (AOI:703-727, the recipient-list callbacks) with the DEVICE's recipient list
//                         (k_tick / k_records fan-out) — the host's GetBroadCastObject (AOI:531-593) is
//                         never run for a device event; GroupID / SceneID events still run its
//                         OnGroupEvent / OnSceneEvent (AOI:233-239); host-only properties (strings,
//                         vectors) take the reference's own path.
//   NFGPUScheduleAdapter  NFIScheduleModule (NFIScheduleModule.h:23-39): object schedules whose name
//                         has a device program on the device; every other schedule (functor-only
//                         heartbeats, module schedules) on the reference's own NFCScheduleModule.
//   NFGPUKernelPlugin     the NFIPlugin that registers them (NFKernelPlugin.cpp:40-46 pattern).
//
// The host NFCObjects are a MIRROR of the device objects, kept up to date lazily:
//   * every write to a device property or int record cell goes to the HOST object first — through
//     NFIKernelModule or straight through the object (GetObject(self)->SetPropertyInt,
//     FindRecord(self, r)->SetInt / AddRow / Remove) — so the reference's change predicates and
//     per-object callbacks run at call time as in the reference; the host common event of that write
//     is forwarded to the device queue instead of the common callbacks;
//   * the common callbacks and the AOI module receive the device's coalesced frame events (the
//     dirty-sync list) with the device's recipient lists;
//   * objects with per-object callbacks (NFIKernelModule::AddPropertyCallBack / AddRecordCallBack,
//     NFIKernelModule.h:28-45, or NFIObject's, seen through the object handle GetObject returns) are
//     EAGER: after the device frame, before the heartbeat functors run, their callbacks fire once per
//     accepted Set of the frame's heartbeat programs — the device's per-Set log (nfk_watch_props /
//     k_chain) — in the order NFCScheduleModule::Execute makes the Sets: objects in NFGUID order, each
//     object's schedules in name order, each program's ops (and a record op's rows) in order
//     (SM:52-80); their other evented properties and cells take the frame's values;
//   * every other object is marked STALE by its events (one byte per event) and brought up to date
//     from the device the next time the host touches it: GetObject, FindRecord, any write through
//     NFIKernelModule, SwitchScene.  A frame therefore costs the host nothing per event beyond the
//     callbacks a server registered, instead of a read-back of every evented (object, property).
//     SetEagerMirror(true) keeps every object eager (the round-4 behaviour) for a server that holds
//     NFIObject pointers across frames without going back through GetObject.
//   f64 record cells are the exception: NFCRecord::SetFloat stores a double into the int64 alternative
//   of the cell (RC:243-297; tests/test_oracle.py::test_reference_record_setfloat_bug), so they are
//   device-only (SetRecordFloat / GetRecordFloat through NFIKernelModule read and write the device).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <tuple>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCScheduleModule.h"
#include "NFComm/NFKernelPlugin/NFCSceneAOIModule.h"
#include "NFComm/NFCore/NFCDataList.h"
#include "NFComm/NFMessageDefine/NFProtocolDefine.hpp"
#include "NFComm/NFPluginModule/NFIClassModule.h"
#include "NFComm/NFPluginModule/NFIPlugin.h"
#include "NFComm/NFPluginModule/NFIPluginManager.h"
#include "NFComm/NFPluginModule/NFIScheduleModule.h"
#include "NFComm/NFPluginModule/NFPlatform.h"
#include "NFGPUKernelModule.hpp"

namespace {
nfgpu::NFGUID to_gpu(const NFGUID& g) { return nfgpu::NFGUID(g.nHead64, g.nData64); }
NFGUID to_ref(const nfgpu::NFGUID& g) { return NFGUID(g.nHead64, g.nData64); }
nfgpu::TDATA_TYPE to_gpu(TDATA_TYPE t) {
    return t == TDATA_INT ? nfgpu::TDATA_INT : t == TDATA_FLOAT ? nfgpu::TDATA_FLOAT
         : t == TDATA_OBJECT ? nfgpu::TDATA_OBJECT : nfgpu::TDATA_UNKNOWN;
}
NFIDataList::TData to_ref(const nfgpu::TData& v) {
    NFIDataList::TData r;
    if (v.type == nfgpu::TDATA_INT) r.SetInt(v.i);
    else if (v.type == nfgpu::TDATA_FLOAT) r.SetFloat(v.f);
    else if (v.type == nfgpu::TDATA_OBJECT) r.SetObject(to_ref(v.o));
    return r;
}
double dbl(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}
struct GuidHash {
    size_t operator()(const NFGUID& g) const { return (size_t)(g.nData64 * 0x9E3779B97F4A7C15ull ^ (uint64_t)g.nHead64); }
};
}  // namespace

// What a device event hands the AOI module (NFGPUSceneAOIAdapter): the event and the device's
// recipient list for it.
class NFGPUDeviceAOI {
public:
    virtual ~NFGPUDeviceAOI() {}
    virtual void DevicePropertyEvent(const NFGUID& self, const std::string& name, const NFIDataList::TData& oldVar,
                                     const NFIDataList::TData& newVar, const NFIDataList& to) = 0;
    virtual void DeviceRecordEvent(const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& oldVar,
                                   const NFIDataList::TData& newVar, const NFIDataList& to) = 0;
};

class NFGPUObject;

class NFGPUKernelAdapter : public NFCKernelModule {
public:
    explicit NFGPUKernelAdapter(NFIPluginManager* p) : NFCKernelModule(p), gpu_(/*capacity=*/1 << 20) {
        gpu_.SetTimeSource([] { return NFGetTime(); });  // NFPlatform.h:367, as NFCScheduleModule reads it
    }

    bool Init() override {
        NFCKernelModule::Init();
        m_pClassModule = pPluginManager->FindModule<NFIClassModule>();
        return true;
    }

    // The device schema from the class definitions (Struct/Class/*.xml through NFIClassModule):
    // every int / float / object property, every record whose columns are all int or float (at
    // most NFK_MAX_REC_ROWS x NFK_MAX_REC_COLS), each class's Public / Private / Upload flags.  The
    // objects created so far enter with their current values, then the layout is committed.
    bool AfterInit() override {
        NFCKernelModule::AfterInit();
        for (NF_SHARE_PTR<NFIClass> c = m_pClassModule->First(); c; c = m_pClassModule->Next()) {
            const std::string cls = c->GetClassName();
            gpu_.AddClass(cls);
            NF_SHARE_PTR<NFIPropertyManager> pm = c->GetPropertyManager();
            for (NF_SHARE_PTR<NFIProperty> p = pm->First(); p; p = pm->Next()) {
                const nfgpu::TDATA_TYPE t = to_gpu(p->GetType());
                if (t == nfgpu::TDATA_UNKNOWN) continue;  // strings / vectors stay on the host
                gpu_.AddProperty(p->GetKey(), t);
                if (dev_props_.insert(p->GetKey()).second) dev_prop_ix_.insert(p->GetKey(), 1);
                gpu_.SetPropertyFlags(cls, p->GetKey(), p->GetPublic(), p->GetPrivate(), p->GetUpload());
            }
            NF_SHARE_PTR<NFIRecordManager> rm = c->GetRecordManager();
            for (NF_SHARE_PTR<NFIRecord> r = rm->First(); r; r = rm->Next()) {
                std::vector<nfgpu::TDATA_TYPE> cols;
                bool ok = r->GetRows() > 0 && r->GetRows() <= NFK_MAX_REC_ROWS && r->GetCols() <= NFK_MAX_REC_COLS;
                for (int i = 0; ok && i < r->GetCols(); i++) {
                    const nfgpu::TDATA_TYPE t = to_gpu(r->GetColType(i));
                    ok = t == nfgpu::TDATA_INT || t == nfgpu::TDATA_FLOAT;
                    cols.push_back(t);
                }
                if (!ok) continue;  // a record with string / object columns stays on the host
                if (!dev_records_.count(r->GetName())) {
                    gpu_.AddRecord(r->GetName(), r->GetRows(), cols);
                    dev_records_.insert(r->GetName());
                    dev_rec_ix_.insert(r->GetName(), 1);
                    for (int i = 0; i < r->GetCols(); i++) col_tags_[r->GetName()][r->GetColTag(i)] = i;
                }
                gpu_.SetRecordFlags(cls, r->GetName(), r->GetPublic(), r->GetPrivate(), r->GetUpload());
            }
        }
        for (int s : scenes_) gpu_.CreateScene(s);
        for (NF_SHARE_PTR<NFIObject> o = First(); o; o = Next()) {
            MirrorObject(o);
            MirrorRecords(o);
        }
        // host writes of device state -> the device (first in the host common lists: the modules
        // register their common callbacks in their own Init / AfterInit)
        NFCKernelModule::RegisterCommonPropertyEvent(PROPERTY_EVENT_FUNCTOR_PTR(new PROPERTY_EVENT_FUNCTOR(
            [this](const NFGUID& self, const std::string& name, const NFIDataList::TData&, const NFIDataList::TData& v) {
                return ForwardProperty(self, name, v);
            })));
        NFCKernelModule::RegisterCommonRecordEvent(RECORD_EVENT_FUNCTOR_PTR(new RECORD_EVENT_FUNCTOR(
            [this](const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData&, const NFIDataList::TData&) {
                return ForwardRecord(self, ev);
            })));
        // the device's frame events -> the common callbacks and the AOI module, in registration order
        gpu_.AddPropertySyncCallBack([this](const nfgpu::NFGUID& g, int pid, const nfgpu::TData& a, const nfgpu::TData& b,
                                            const nfgpu::NFGPUKernelModule::SyncArgs& sa) { DeliverProperty(g, pid, a, b, sa); });
        gpu_.AddRecordSyncCallBack([this](const nfgpu::NFGUID& g, const nfgpu::RECORD_EVENT_DATA& e, const nfgpu::TData& a,
                                          const nfgpu::TData& b, const nfgpu::NFGPUKernelModule::SyncArgs& sa) {
            DeliverRecord(g, e, a, b, sa);
        });
        // the host mirror after the device frame, before the heartbeat functors run
        gpu_.SetFrameHook([this](const nfk_frame_host& f) { OnFrame(f); });
        const bool ok = gpu_.AfterInit();
        // the record op of each (record, column): its kind and op index, the order key of its
        // per-object callbacks (at most one op per record column, nfgpu.h NFK_MAX_REC_OPS)
        for (int k = 0; k < gpu_.HeartBeatCount(); k++) {
            const std::vector<nfk_op>& ops = gpu_.HeartBeatOps(k);
            for (int i = 0; i < (int)ops.size(); i++)
                if (ops[i].code == NFK_OP_RIADD_CLAMP || ops[i].code == NFK_OP_RFAFFINE)
                    rec_op_[ops[i].dst] = std::make_pair(k, i);
        }
        for (const std::string& nm : watch_pending_)
            if (dev_props_.count(nm) && watched_.insert(nm).second) gpu_.WatchProperty(nm);
        watch_pending_.clear();
        // the device schedule calls made while their objects were being created (class callbacks at
        // COE_CREATE_HASDATA, e.g. HelloWorld3Module.cpp:47), now that the layout exists
        FlushCreationSchedules();
        return ok;
    }

    // NFCKernelModule::Execute (KM:70-99) + NFCScheduleModule::Execute (SM:49) + the AOI fan-out.  KM's
    // walk of every object is kept only for the objects that can have components: NFCObject::Execute
    // runs the object's components and nothing else (NFCObject.cpp:42-47, NFCComponentManager.cpp:73-85),
    // and a component is added through the object's component manager (NFIObject::AddComponent), so the
    // objects whose manager was handed out are walked, in NFGUID order as KM's map walk; the others'
    // Execute is empty (a walk of 1M host objects costs ~0.7 s per frame).
    bool Execute() override {
        ProcessMemFree();
        if (!mtDeleteSelfList.empty()) {  // KM:76-84
            for (const NFGUID& g : mtDeleteSelfList) DestroyObject(g);
            mtDeleteSelfList.clear();
        }
        if (NFISceneAOIModule* a = pPluginManager->FindModule<NFISceneAOIModule>()) a->Execute();  // KM:86
        // (a copy: a component may destroy or create objects; its own object's DestroyObject is
        // deferred to the next Execute through mtDeleteSelfList, KM:275-279 / KM:1434)
        walk_.assign(has_components_.begin(), has_components_.end());
        for (const NFGUID& g : walk_) {
            NF_SHARE_PTR<NFIObject> o = GetElement(g);
            if (!o) continue;
            cur_exe_ = g;  // KM:92-94 (mnCurExeObject is private to NFCKernelModule)
            o->Execute();
            cur_exe_ = NFGUID();
        }
        return gpu_.Execute();
    }

    bool CreateScene(const int nSceneID) override {  // KM:981
        const bool ok = NFCKernelModule::CreateScene(nSceneID);
        if (ok) {
            scenes_.insert(nSceneID);
            gpu_.CreateScene(nSceneID);
        }
        return ok;
    }

    // NFCKernelModule::CreateObject (KM:101-271) builds the host object (class events, config and
    // argument values, SceneID / GroupID; the property / record events of that build go to the
    // common callbacks from the host object, as in the reference); its device properties then enter
    // the device world with those values (before AfterInit: with the layout; after it: at the start
    // of the next frame).  Rows that creation-time handlers add to a device record after AfterInit
    // are not carried over: the device record starts empty (use AddRow once the object exists).
    // Returns the object's handle (NFGPUObject).
    NF_SHARE_PTR<NFIObject> CreateObject(const NFGUID& self, const int nSceneID, const int nGroupID,
                                         const std::string& strClassName, const std::string& strConfigIndex,
                                         const NFIDataList& arg) override {
        creating_.push_back(self);
        NF_SHARE_PTR<NFIObject> o = NFCKernelModule::CreateObject(self, nSceneID, nGroupID, strClassName, strConfigIndex, arg);
        creating_.pop_back();
        if (!o) {
            DropCreationSchedules(self);
            return o;
        }
        if (!dev_props_.empty()) MirrorObject(o);
        CacheClassName(self, o);
        if (gpu_.World()) FlushCreationSchedules();
        return Handle(self, o);
    }

    // The reference's AOI module asks for a group's players with a ClassName test of every member
    // (KM:1270-1294 reads each member's ClassName string through an NFGUID map) once per creation-time
    // Set of an object entering a group (AOI:260 -> 531-593) and once per member in OnGroupEvent
    // (AOI:357-440): O(group) string lookups per call.  The same answers, faster: the class name of each
    // object kept beside it (CacheClassName), and a Player list taken from the group's player map — the
    // objects CreateObject adds as players (KM:146) and every SwitchScene arrival (KM:945), whose
    // ClassName is still tested — since no object of class Player is ever in the other map.
    const std::string& GetPropertyString(const NFGUID& self, const std::string& name) override {  // KM:425
        if (name == NFrame::IObject::ClassName()) {
            auto it = class_of_.find(self);
            if (it != class_of_.end()) return *it->second;
        }
        return NFCKernelModule::GetPropertyString(self, name);
    }
    bool SetPropertyString(const NFGUID& self, const std::string& name, const std::string& v) override {  // KM:349
        const bool ok = NFCKernelModule::SetPropertyString(self, name, v);
        if (name == NFrame::IObject::ClassName()) RefreshClassName(self);
        return ok;
    }
    bool GetGroupObjectList(const int scene, const int group, const std::string& cls, const NFGUID& noSelf,
                            NFIDataList& list) override {  // KM:1270
        if (cls != NFrame::Player::ThisName()) return NFCKernelModule::GetGroupObjectList(scene, group, cls, noSelf, list);
        NFCDataList& pl = gl_scratch_;
        pl.Clear();
        if (!NFCKernelModule::GetGroupObjectList(scene, group, pl, true)) return false;
        for (int i = 0; i < pl.GetCount(); i++) {
            const NFGUID id = pl.Object(i);
            if (!id.IsNull() && id != noSelf && GetPropertyString(id, NFrame::IObject::ClassName()) == cls) list.AddObject(id);
        }
        return true;
    }
    bool GetGroupObjectList(const int scene, const int group, const std::string& cls, NFIDataList& list) override {  // KM:1245
        return GetGroupObjectList(scene, group, cls, NFGUID(), list);
    }
    // the object's handle: its device state is brought up to date first
    NF_SHARE_PTR<NFIObject> GetObject(const NFGUID& ident) override {
        NF_SHARE_PTR<NFIObject> o = NFCKernelModule::GetObject(ident);
        if (!o) return o;
        SyncObject(ident);
        return Handle(ident, o);
    }
    // a record handed out may get hooks and be read later: its object is kept up to date every frame
    NF_SHARE_PTR<NFIRecord> FindRecord(const NFGUID& self, const std::string& rec) override {  // KM:479
        if (DevRecord(self, rec)) MarkEager(self, true);
        return NFCKernelModule::FindRecord(self, rec);
    }

    // the reference's DestroyObject reads SceneID / GroupID through GetPropertyInt (KM:283-284),
    // which this adapter answers from the device: it runs while the object is still there
    bool DestroyObject(const NFGUID& self) override {  // KM:273
        if (self == cur_exe_ && !self.IsNull()) {  // KM:275-279: DestroySelf, applied by the next Execute
            mtDeleteSelfList.push_back(self);
            return true;
        }
        ForgetHostObject(self);
        DropCreationSchedules(self);
        const bool ok = NFCKernelModule::DestroyObject(self);
        gpu_.DestroyObject(to_gpu(self));
        handles_.erase(self);
        pre_eager_.erase(self);
        class_of_.erase(self);
        has_components_.erase(self);
        return ok;
    }

    // Writes through NFIKernelModule: the reference's own NFCKernelModule on the host object (KM:323-372,
    // 492-544), its state brought up to date first; ForwardProperty / ForwardRecord queue the accepted
    // writes on the device.
    // (a device object's host NFCObject from the adapter's index-keyed cache: KM:325-328's GetElement(self)
    // without its walk of the object tree; any other object takes the reference's own path)
    bool SetPropertyInt(const NFGUID& self, const std::string& name, const NFINT64 v) override {  // KM:323
        if (NFIObject* ob = SyncedHostObject(self)) return ob->SetPropertyInt(name, v);
        return NFCKernelModule::SetPropertyInt(self, name, v);
    }
    bool SetPropertyFloat(const NFGUID& self, const std::string& name, const double v) override {  // KM:336
        if (NFIObject* ob = SyncedHostObject(self)) return ob->SetPropertyFloat(name, v);
        return NFCKernelModule::SetPropertyFloat(self, name, v);
    }
    bool SetPropertyObject(const NFGUID& self, const std::string& name, const NFGUID& v) override {  // KM:362
        if (NFIObject* ob = SyncedHostObject(self)) return ob->SetPropertyObject(name, v);
        return NFCKernelModule::SetPropertyObject(self, name, v);
    }
    bool SetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const int nCol, const NFINT64 v) override {
        SyncObject(self);  // KM:505
        return NFCKernelModule::SetRecordInt(self, rec, nRow, nCol, v);
    }
    bool SetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag,
                      const NFINT64 v) override {  // KM:525
        SyncObject(self);
        return NFCKernelModule::SetRecordInt(self, rec, nRow, tag, v);
    }
    bool ClearRecord(const NFGUID& self, const std::string& rec) override {  // KM:492 (without marking the record handed out)
        SyncObject(self);
        NF_SHARE_PTR<NFIObject> o = GetElement(self);
        NF_SHARE_PTR<NFIRecord> r = o ? o->GetRecordManager()->GetElement(rec) : nullptr;
        return r ? r->Clear() : false;
    }
    NFINT64 GetPropertyInt(const NFGUID& self, const std::string& name) override {  // KM:401, read-your-writes
        return DevProp(self, name) ? gpu_.GetPropertyInt(to_gpu(self), name) : NFCKernelModule::GetPropertyInt(self, name);
    }
    double GetPropertyFloat(const NFGUID& self, const std::string& name) override {  // KM:413
        return DevProp(self, name) ? gpu_.GetPropertyFloat(to_gpu(self), name) : NFCKernelModule::GetPropertyFloat(self, name);
    }
    const NFGUID& GetPropertyObject(const NFGUID& self, const std::string& name) override {  // KM:440
        if (!DevProp(self, name)) return NFCKernelModule::GetPropertyObject(self, name);
        obj_scratch_ = to_ref(gpu_.GetPropertyObject(to_gpu(self), name));
        return obj_scratch_;
    }
    // f64 record cells: device only (see the header)
    bool SetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const int nCol,
                        const double v) override {  // KM:545
        return DevRecord(self, rec) ? gpu_.SetRecordFloat(to_gpu(self), rec, nRow, nCol, v)
                                       : NFCKernelModule::SetRecordFloat(self, rec, nRow, nCol, v);
    }
    bool SetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag,
                        const double v) override {  // NFIKernelModule.h:128
        if (!DevRecord(self, rec)) return NFCKernelModule::SetRecordFloat(self, rec, nRow, tag, v);
        const int c = ColOf(rec, tag);
        return c >= 0 && gpu_.SetRecordFloat(to_gpu(self), rec, nRow, c, v);
    }
    NFINT64 GetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const int nCol) override {
        return DevRecord(self, rec) ? gpu_.GetRecordInt(to_gpu(self), rec, nRow, nCol)  // NFIKernelModule.h:134
                                       : NFCKernelModule::GetRecordInt(self, rec, nRow, nCol);
    }
    double GetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const int nCol) override {
        return DevRecord(self, rec) ? gpu_.GetRecordFloat(to_gpu(self), rec, nRow, nCol)  // NFIKernelModule.h:135
                                       : NFCKernelModule::GetRecordFloat(self, rec, nRow, nCol);
    }
    NFINT64 GetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag) override {
        if (!DevRecord(self, rec)) return NFCKernelModule::GetRecordInt(self, rec, nRow, tag);
        const int c = ColOf(rec, tag);
        return c >= 0 ? gpu_.GetRecordInt(to_gpu(self), rec, nRow, c) : 0;
    }
    double GetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag) override {
        if (!DevRecord(self, rec)) return NFCKernelModule::GetRecordFloat(self, rec, nRow, tag);
        const int c = ColOf(rec, tag);
        return c >= 0 ? gpu_.GetRecordFloat(to_gpu(self), rec, nRow, c) : 0.0;
    }

    bool SwitchScene(const NFGUID& self, const int scene, const int group, const float fX, const float fY,
                     const float fZ, const float fOrient, const NFIDataList& arg) override {  // NFIKernelModule.h:148
        // the host-side scene lists and the host object's SceneID / GroupID / X / Y / Z writes
        // (KM:930-942: its per-object callbacks fire here); the device queues the same writes with
        // the membership change itself, so they are not forwarded
        SyncObject(self);
        ++quiet_;
        NFCKernelModule::SwitchScene(self, scene, group, fX, fY, fZ, fOrient, arg);
        --quiet_;
        return gpu_.SwitchScene(to_gpu(self), scene, group, fX, fY, fZ, fOrient);
    }

    // every object eager (the host mirror written every frame): for a server that keeps NFIObject
    // pointers across frames without going back through GetObject
    void SetEagerMirror(bool on) {
        eager_all_ = on;
        if (on)
            for (auto& m : mstate_) m |= kEager | kMirrorAll;
    }
    // (measurement) device events that reached NFCSceneAOIModule's common handlers — and so its
    // GetBroadCastObject — must stay 0; device events handed to the AOI module with the device's list
    int64_t AOIHostDeviceCalls() const { return aoi_host_device_calls_; }
    int64_t AOIDeviceCalls() const { return aoi_device_calls_; }
    int64_t MirrorSyncs() const { return n_syncs_; }  // objects brought up to date lazily
    int64_t ChainCallbacks() const { return n_chain_fired_; }

    // NFGPUSceneAOIAdapter::Init wraps NFCSceneAOIModule::Init in these: the common callbacks the AOI
    // module registers meanwhile (AOI.cpp:20-22) get the device's events through `aoi`
    void BeginAOIRegistration(NFGPUDeviceAOI* aoi) {
        aoi_ = aoi;
        aoi_registering_ = true;
    }
    void EndAOIRegistration() { aoi_registering_ = false; }

    // (NFGPUScheduleAdapter) a device schedule call on an object that is not on the device yet — being
    // created (its class callbacks run inside CreateObject, KM:146-267, before the adapter hands it to the
    // device) or created before AfterInit: kept in call order with the clock of the call and made once the
    // object is there (NFCScheduleModule applies AddSchedule at its next Execute anyway, SM:257, 95-117)
    bool DeferSchedule(const NFGUID& self) const {
        return !DevObject(self) && (!gpu_.World() || std::find(creating_.begin(), creating_.end(), self) != creating_.end());
    }
    struct DeferredSchedule {
        int op;  // 1 AddSchedule, 2 RemoveSchedule(self, name), 3 RemoveSchedule(self)
        NFGUID self;
        std::string name;
        nfgpu::OBJECT_SCHEDULE_FUNCTOR cb;
        float t;
        int count;
        int64_t now;
    };
    void QueueCreationSchedule(DeferredSchedule d) { creation_sched_.push_back(std::move(d)); }
    // (NFGPUObject) the host object is about to be read or written through its handle
    void Touch(const NFGUID& self) { SyncObject(self); }
    // (NFGPUObject) a read of a device property inside the heartbeat functor walk with walk-order reads
    // on (NFGPUKernelModule::SetWalkOrderReads) goes to the device log, not the host object
    bool WalkRead(const NFGUID& self, const std::string& name) const {
        return gpu_.WalkOrderReads() && gpu_.InFunctorWalk() && DevProp(self, name);
    }
    // (NFGPUObject) its ClassName was written; its component manager was handed out
    void ClassNameChanged(const NFGUID& self) { RefreshClassName(self); }
    void HasComponents(const NFGUID& self) { has_components_.insert(self); }
    // (NFGPUObject) a per-object callback registered on a device property / record, or the object's
    // managers handed out: the object is eager from now on, a device property's Sets are logged
    void Watched(const NFGUID& self, const std::string& prop) {
        MarkEager(self, prop.empty());
        if (prop.empty() || watched_.count(prop)) return;
        if (!gpu_.World()) {  // before AfterInit the device properties are not known yet (a callback
            watch_pending_.push_back(prop);  // registered at creation, e.g. NFCNPCRefreshModule.cpp:104)
            return;
        }
        if (!dev_props_.count(prop)) return;
        watched_.insert(prop);
        gpu_.WatchProperty(prop);
    }

    nfgpu::NFGPUKernelModule gpu_;

protected:
    // Common property / record callbacks (NFIKernelModule.h:181-182): the device's coalesced events
    // for its properties and records (delivered by Execute), the host's for the rest (strings,
    // vectors, host-only records).  The AOI module's own (registered while BeginAOIRegistration is
    // on) receive no device event: NFGPUSceneAOIAdapter gets those with the device's recipients.
    bool RegisterCommonPropertyEvent(const PROPERTY_EVENT_FUNCTOR_PTR& cb) override {
        const bool aoi = aoi_registering_;
        PROPERTY_EVENT_FUNCTOR_PTR host(new PROPERTY_EVENT_FUNCTOR(
            [this, cb, aoi](const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                if (MirrorTarget(self, name) || DevProp(self, name)) return 0;
                if (aoi) ++aoi_host_calls_;
                return (*cb)(self, name, a, b);
            }));
        NFCKernelModule::RegisterCommonPropertyEvent(host);
        prop_cb_.push_back({cb, aoi});
        return true;
    }
    bool RegisterCommonRecordEvent(const RECORD_EVENT_FUNCTOR_PTR& cb) override {
        const bool aoi = aoi_registering_;
        RECORD_EVENT_FUNCTOR_PTR host(new RECORD_EVENT_FUNCTOR(
            [this, cb, aoi](const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                if (DevRecord(self, ev.strRecordName)) return 0;
                if (aoi) ++aoi_host_calls_;
                return (*cb)(self, ev, a, b);
            }));
        NFCKernelModule::RegisterCommonRecordEvent(host);
        rec_cb_.push_back({cb, aoi});
        return true;
    }

private:
    template <class F>
    struct Common {
        F cb;
        bool aoi;  // the AOI module's: device events go to NFGPUSceneAOIAdapter instead
    };
    // kWritten: a host write of one of the object's device properties / record cells that a heartbeat
    // program also writes was forwarded since the last frame (OnFrame marks it stale: the program may have
    // put the value back where the frame started, which raises no event, while the host mirror holds the
    // written value; a property no program writes has its event whenever the write changed it)
    // kEager: the object's per-object callbacks fire from the device's per-Set log (OnFrame); kMirrorAll:
    // its host object is also written with every frame event (its managers or records were handed out,
    // or SetEagerMirror) — an eager object without it is marked stale by its other events instead,
    // like any other object (NFCNPCRefreshModule's HP callback on every NPC, NFCNPCRefreshModule.cpp:104,
    // then costs the host the HP Sets' callbacks and a byte per other event)
    enum : uint8_t { kStale = 1, kEager = 2, kWritten = 4, kMirrorAll = 8 };
    // a Set whose per-object callbacks OnFrame fires, keyed (NFGUID of o, kind, op, row)
    struct Fire {
        int32_t o, kind, op, row;
        int64_t i;  // LastChain() index (row < 0) or record event index
    };

    NF_SHARE_PTR<NFIObject> Handle(const NFGUID& self, const NF_SHARE_PTR<NFIObject>& o);
    // the object's class name, one shared string per class (see GetPropertyString)
    void CacheClassName(const NFGUID& self, const NF_SHARE_PTR<NFIObject>& o) {
        const std::string& c = o->GetPropertyString(NFrame::IObject::ClassName());
        auto it = class_names_.insert(c).first;
        class_of_[self] = &*it;
    }
    void RefreshClassName(const NFGUID& self) {
        NF_SHARE_PTR<NFIObject> o = GetElement(self);
        if (o) CacheClassName(self, o);
        else class_of_.erase(self);
    }

    // an accepted host write of a device property (NFCProperty::SetInt / SetFloat / SetObject raised
    // the common event): queued on the device in call order
    int ForwardProperty(const NFGUID& self, const std::string& name, const NFIDataList::TData& v) {
        if (quiet_ || OwnWrite(self, name, -1, -1) || !DevProp(self, name)) return 0;
        const nfgpu::NFGUID g = to_gpu(self);
        if (gpu_.ProgramWrites(gpu_.PropertyId(name))) Written(g);  // (only a program can undo it unseen)
        if (v.GetType() == TDATA_INT) gpu_.SetPropertyInt(g, name, v.GetInt());
        else if (v.GetType() == TDATA_FLOAT) gpu_.SetPropertyFloat(g, name, v.GetFloat());
        else if (v.GetType() == TDATA_OBJECT) gpu_.SetPropertyObject(g, name, to_gpu(v.GetObject()));
        return 0;
    }
    // an accepted host write of a device record (NFCRecord's Update / Add / Cover / Del events,
    // RC:170-177, 225-231, 1092-1098): the same call queued on the device
    int ForwardRecord(const NFGUID& self, const RECORD_EVENT_DATA& ev) {
        if (quiet_ || (ev.nOpType == RECORD_EVENT_DATA::Update && OwnWrite(self, ev.strRecordName, ev.nRow, ev.nCol)) ||
            !DevRecord(self, ev.strRecordName))
            return 0;
        NF_SHARE_PTR<NFIObject> o = GetElement(self);
        NF_SHARE_PTR<NFIRecord> r = o ? o->GetRecordManager()->GetElement(ev.strRecordName) : nullptr;
        if (!r) return 0;
        const nfgpu::NFGUID g = to_gpu(self);
        {
            const int rid = gpu_.RecordId(ev.strRecordName);
            if (ev.nOpType == RECORD_EVENT_DATA::Update ? gpu_.ProgramWritesRecord(rid, ev.nCol) : gpu_.ProgramWritesRecord(rid))
                Written(g);
        }
        switch (ev.nOpType) {
            case RECORD_EVENT_DATA::Update:
                // (an f64 cell written on the host holds the double in the int64 alternative and
                // cannot be read back: f64 record cells are device-only)
                if (r->GetColType(ev.nCol) == TDATA_INT)
                    gpu_.SetRecordInt(g, ev.strRecordName, ev.nRow, ev.nCol, r->GetInt(ev.nRow, ev.nCol));
                break;
            case RECORD_EVENT_DATA::Add:
            case RECORD_EVENT_DATA::Cover: {  // the row as AddRow left it (values already stored)
                std::vector<nfgpu::TData> vals((size_t)r->GetCols());
                for (int c = 0; c < r->GetCols(); c++) {
                    vals[c].type = to_gpu(r->GetColType(c));
                    if (vals[c].type == nfgpu::TDATA_INT) vals[c].i = r->GetInt(ev.nRow, c);
                    else vals[c].f = r->GetFloat(ev.nRow, c);
                }
                gpu_.AddRow(g, ev.strRecordName, ev.nRow, vals);
                break;
            }
            case RECORD_EVENT_DATA::Del:  // raised while the row is still used (RC:1092)
                gpu_.RemoveRow(g, ev.strRecordName, ev.nRow);
                break;
            default:  // Swap / Sort / Create / Cleared: no device counterpart
                break;
        }
        return 0;
    }

    // the device's recipient run as the NFIDataList the AOI callbacks take (rebuilt only when the run
    // differs from the last one: consecutive events of a scene group mostly share it)
    const NFIDataList& Recipients(const nfgpu::NFGPUKernelModule::SyncArgs& sa) {
        if (sa.rcpt->empty()) return none_;
        if (!sa.same || !rl_valid_) {
            rl_.Clear();
            for (const nfgpu::NFGUID& g : *sa.rcpt) rl_.Add(to_ref(g));
            rl_valid_ = true;
        }
        return rl_;
    }
    // one device property event: the common callbacks in registration order, the AOI module's slot
    // with the device's recipient list
    void DeliverProperty(const nfgpu::NFGUID& g, int pid, const nfgpu::TData& a, const nfgpu::TData& b,
                         const nfgpu::NFGPUKernelModule::SyncArgs& sa) {
        if (prop_cb_.empty()) return;
        const NFGUID s = to_ref(g);
        const std::string& name = gpu_.PropertyName(pid);
        const NFIDataList::TData ra = to_ref(a), rb = to_ref(b);
        for (auto& c : prop_cb_) {
            if (!c.aoi) {
                (*c.cb)(s, name, ra, rb);
            } else if (aoi_) {
                ++aoi_device_calls_;
                aoi_->DevicePropertyEvent(s, name, ra, rb, Recipients(sa));
            }
        }
    }
    void DeliverRecord(const nfgpu::NFGUID& g, const nfgpu::RECORD_EVENT_DATA& e, const nfgpu::TData& a,
                       const nfgpu::TData& b, const nfgpu::NFGPUKernelModule::SyncArgs& sa) {
        if (rec_cb_.empty()) return;
        const NFGUID s = to_ref(g);
        rev_.nOpType = (RECORD_EVENT_DATA::RecordOptype)e.nOpType;
        rev_.nRow = e.nRow;
        rev_.nCol = e.nCol;
        if (rev_.strRecordName != e.strRecordName) rev_.strRecordName = e.strRecordName;
        const NFIDataList::TData ra = to_ref(a), rb = to_ref(b);
        for (auto& c : rec_cb_) {
            if (!c.aoi) {
                (*c.cb)(s, rev_, ra, rb);
            } else if (aoi_ && gpu_.ObjectGroup(sa.obj) >= 0) {  // AOI:270-276: no sync for group < 0
                ++aoi_device_calls_;
                aoi_->DeviceRecordEvent(s, rev_, ra, rb, Recipients(sa));
            }
        }
    }

    uint8_t& State(int o) {
        if ((size_t)o >= mstate_.size())
            mstate_.resize((size_t)gpu_.ObjectCount() + 1024, eager_all_ ? (uint8_t)(kEager | kMirrorAll) : (uint8_t)0);
        return mstate_[(size_t)o];
    }
    void Written(const nfgpu::NFGUID& g) {
        const int o = gpu_.ObjectIndex(g);
        if (o < 0) return;  // (being created: its creation values are the device's)
        uint8_t& m = State(o);
        if (!(m & kWritten)) {
            m |= kWritten;
            written_.push_back(o);
        }
    }
    void MarkEager(const NFGUID& self, bool all) {
        const uint8_t bits = all ? (uint8_t)(kEager | kMirrorAll) : (uint8_t)kEager;
        const int o = gpu_.ObjectIndex(to_gpu(self));
        if (o < 0) {
            if (GetElement(self)) pre_eager_[self] |= bits;  // (being created: applied by MirrorObject)
            return;
        }
        SyncObject(self);
        State(o) |= bits;
    }

    // After the device frame (the frame hook), before the heartbeat functors: eager objects take the
    // frame's values with their per-object callbacks fired once per accepted Set of the frame's
    // heartbeat programs in the reference's order; every other evented object is marked stale.
    void OnFrame(const nfk_frame_host& f) {
        prof_.Start();
        // objects the host wrote this window: stale, whatever their events (a program may have put a
        // written value back where the frame started, with no event).  An eager one's watched
        // properties are brought up to date below with their callbacks, so its refresh on the next
        // host access (SyncObject) finds them equal and fires nothing
        for (int o : written_) State(o) = (uint8_t)((State(o) & ~kWritten) | kStale);
        written_.clear();
        std::vector<int64_t>& ep = fr_ep_;
        std::vector<int64_t>& er = fr_er_;
        ep.clear();
        er.clear();
        for (int64_t e = 0; e < f.n_ev; e++) {
            uint8_t& m = State(f.ev_obj[e]);
            if (m & kEager) ep.push_back(e);
            else m |= kStale;
        }
        for (int64_t e = 0; e < f.n_re; e++) {
            uint8_t& m = State(f.re_obj[e]);
            if (m & kEager) er.push_back(e);
            else m |= kStale;
        }
        if (ep.empty() && er.empty()) return;
        prof_.Mark(0);
        // the Sets with callbacks, keyed (NFGUID, kind, op, row): the watched properties' per-Set log,
        // and the record cells a record op changed (one op per record column: at most one change per
        // cell and frame, so the frame's event is that Set)
        std::vector<Fire>& fires = fr_fire_;
        fires.clear();
        // (the log comes in the walk's order, nfk_read_chain; it may hold properties no callback
        // here watches: the plugin's own walk-order reads)
        const std::vector<nfgpu::NFGPUKernelModule::ChainEntry>& ch = gpu_.LastChain();
        for (size_t i = 0; i < ch.size(); i++)
            if ((State(ch[i].obj) & kEager) && WatchedPid(ch[i].pid)) fires.push_back({ch[i].obj, ch[i].kind, ch[i].op, -1, (int64_t)i});
        const size_t n_prop_fires = fires.size();
        for (int64_t e : er) {
            const uint32_t rrc = f.re_rrc[e];
            if ((rrc >> 24) & 3) continue;  // row events: the host record made them (AddRow / Remove / Clear)
            auto it = rec_op_.find((uint16_t)((((rrc >> 16) & 0xFF) << 8) | (rrc & 0xFF)));
            if (it == rec_op_.end()) continue;  // a SetRecord cell: the host record holds its value already
            fires.push_back({f.re_obj[e], it->second.first, it->second.second, (int32_t)((rrc >> 8) & 0xFF), e});
        }
        auto walk_less = [this](const Fire& x, const Fire& y) {
            if (x.o != y.o) {
                const nfgpu::NFGUID &gx = gpu_.ObjectGuid(x.o), &gy = gpu_.ObjectGuid(y.o);
                return gx < gy;
            }
            if (x.kind != y.kind) return x.kind < y.kind;
            if (x.op != y.op) return x.op < y.op;
            return x.row < y.row;
        };
        if (fires.size() > n_prop_fires) {  // the record ops' cells (device slot order) merged into the log's order
            std::stable_sort(fires.begin() + (std::ptrdiff_t)n_prop_fires, fires.end(), walk_less);
            std::inplace_merge(fires.begin(), fires.begin() + (std::ptrdiff_t)n_prop_fires, fires.end(), walk_less);
        }
        prof_.Mark(1);
        // the fires' host objects are scattered over the host heap (NFGUID order is not allocation order):
        // their table entries are prefetched kFar fires ahead, the property objects kNear ahead
        constexpr size_t kFar = 24, kNear = 8;
        for (size_t q = 0; q < fires.size(); q++) {
            if (q + kFar < fires.size()) PrefetchFire(fires[q + kFar], false);
            if (q + kNear < fires.size()) PrefetchFire(fires[q + kNear], true);
            const Fire& fi = fires[q];
            const NFGUID self = to_ref(gpu_.ObjectGuid(fi.o));
            NFIObject* ob = HostObject(fi.o);
            if (!ob) continue;
            if (fi.row < 0) {  // NFCProperty::SetInt / SetFloat of one Set (PR:254-334): its callbacks fire
                const auto& c = ch[(size_t)fi.i];
                const std::string& name = gpu_.PropertyName(c.pid);
                NFIProperty* p = HostProperty(fi.o, c.pid, name);
                if (!p) continue;
                Mirror(self, name, -1, -1, [&] {
                    if (p->GetType() == TDATA_INT) p->SetInt((NFINT64)c.new_bits);
                    else if (p->GetType() == TDATA_FLOAT) p->SetFloat(dbl(c.new_bits));
                });
                n_chain_fired_++;
            } else {  // NFCRecord::SetInt (RC:182)
                const uint32_t rrc = f.re_rrc[fi.i];
                const std::string& rn = gpu_.RecordName((int)((rrc >> 16) & 0xFF));
                NF_SHARE_PTR<NFIRecord> r = ob->GetRecordManager()->GetElement(rn);
                const int row = (int)((rrc >> 8) & 0xFF), col = (int)(rrc & 0xFF);
                if (r && r->IsUsed(row) && r->GetColType(col) == TDATA_INT && r->GetInt(row, col) != (NFINT64)f.re_new[fi.i]) {
                    Mirror(self, rn, row, col, [&] { r->SetInt(row, col, (NFINT64)f.re_new[fi.i]); });
                    n_chain_fired_++;
                }
            }
        }
        prof_.Mark(2);
        // the eager objects' other evented properties: the frame's value (an unwatched property has no
        // per-object callback that could tell the Sets apart) when the host object is read directly
        // (kMirrorAll); otherwise the object is stale for them, as any other object (its watched
        // properties are current: the log's callbacks above wrote them)
        WatchedPid(0);  // (the watched-property table current: read directly in the loop below)
        const uint8_t* const wpid = watched_pid_.data();
        const size_t n_wpid = watched_pid_.size();
        for (int64_t e : ep) {
            // (mstate_ is sized for every evented object by the marks above; indexed afresh each time:
            // a mirror write's callbacks below may create objects and grow it)
            uint8_t& m = mstate_[(size_t)f.ev_obj[e]];
            if (!(m & kMirrorAll)) {
                const int32_t pid = f.ev_pid[e];
                if (!(pid >= 0 && (size_t)pid < n_wpid && wpid[pid])) m |= kStale;
                continue;
            }
            const NFGUID self = to_ref(gpu_.ObjectGuid(f.ev_obj[e]));
            NF_SHARE_PTR<NFIObject> ob = GetElement(self);
            const std::string& name = gpu_.PropertyName(f.ev_pid[e]);
            NF_SHARE_PTR<NFIProperty> p = ob ? ob->GetPropertyManager()->GetElement(name) : nullptr;
            if (!p) continue;
            Mirror(self, name, -1, -1, [&] {
                if (p->GetType() == TDATA_OBJECT) {
                    const NFGUID v(f.ev_new_h ? (int64_t)f.ev_new_h[e] : 0, (int64_t)f.ev_new[e]);
                    if (p->GetObject() != v) p->SetObject(v);
                } else {
                    PutValue(p, f.ev_new[e]);
                }
            });
        }
        prof_.Mark(3);
        prof_.Report(fires.size(), ep.size());
        // (record cells: a cell no record op writes changed only through the host record's own calls,
        // which the host record holds already — the frame's coalesced event of such a cell can carry a
        // SetRecord value an AddRow later overwrote, nfgpu.h nfk_set_records)
    }
    // (measurement, NFGPU_ADAPTER_PROF=1) OnFrame's parts per frame on stderr: state marks, the fire
    // list, the per-Set callbacks, the eager objects' other events
    struct FrameProf {
        bool on = getenv("NFGPU_ADAPTER_PROF") != nullptr;
        std::chrono::steady_clock::time_point t0;
        double ms[4] = {0, 0, 0, 0};
        void Start() {
            if (on) t0 = std::chrono::steady_clock::now();
        }
        void Mark(int i) {
            if (!on) return;
            const auto t = std::chrono::steady_clock::now();
            ms[i] = std::chrono::duration<double, std::milli>(t - t0).count();
            t0 = t;
        }
        void Report(size_t nf, size_t nep) {
            if (on) fprintf(stderr, "[onframe] marks %.3f fires %.3f callbacks %.3f others %.3f ms (%zu fires, %zu eager events)\n",
                            ms[0], ms[1], ms[2], ms[3], nf, nep);
        }
    } prof_;
    // (OnFrame) a fire's table entries (far), then the host property they point to (near)
    void PrefetchFire(const Fire& fi, bool near) {
        const size_t o = (size_t)fi.o;
        if (!near) {
            __builtin_prefetch(&gpu_.ObjectGuid(fi.o));
            if (o < host_obj_.size()) __builtin_prefetch(&host_obj_[o]);
            if (fi.row < 0 && watched_slots_) {
                const int w = WatchedSlotFast(FirePid(fi));
                if (w >= 0 && o * watched_slots_ + (size_t)w < prop_cache_.size())
                    __builtin_prefetch(&prop_cache_[o * watched_slots_ + (size_t)w]);
            }
            return;
        }
        if (fi.row < 0 && watched_slots_) {
            const int w = WatchedSlotFast(FirePid(fi));
            const size_t at = o * watched_slots_ + (size_t)w;
            if (w >= 0 && at < prop_cache_.size() && prop_cache_[at]) {
                const char* p = (const char*)prop_cache_[at];
                __builtin_prefetch(p);
                __builtin_prefetch(p + 64);
                __builtin_prefetch(p + 128);
            }
        } else if (o < host_obj_.size() && host_obj_[o]) {
            __builtin_prefetch(host_obj_[o]);
        }
    }
    // the property of a per-Set fire (row < 0: fi.i indexes the frame's per-Set log)
    int FirePid(const Fire& fi) const { return gpu_.LastChain()[(size_t)fi.i].pid; }
    int WatchedSlotFast(int pid) const {
        return pid >= 0 && (size_t)pid < watched_slot_.size() ? watched_slot_[(size_t)pid] : -1;
    }
    // whether a device property id has a per-object callback somewhere (watched_, by device id)
    bool WatchedPid(int pid) {
        if (watched_pid_.size() != (size_t)gpu_.PropertyCount(nfgpu::TDATA_INT) + gpu_.PropertyCount(nfgpu::TDATA_FLOAT) +
                                       gpu_.PropertyCount(nfgpu::TDATA_OBJECT) || watched_n_ != watched_.size()) {
            watched_pid_.assign((size_t)gpu_.PropertyCount(nfgpu::TDATA_INT) + gpu_.PropertyCount(nfgpu::TDATA_FLOAT) +
                                    gpu_.PropertyCount(nfgpu::TDATA_OBJECT), 0);
            watched_slot_.assign(watched_pid_.size(), -1);
            watched_slots_ = 0;
            for (const std::string& nm : watched_) {
                watched_pid_[(size_t)gpu_.PropertyId(nm)] = 1;
                watched_slot_[(size_t)gpu_.PropertyId(nm)] = (int)watched_slots_++;
            }
            watched_n_ = watched_.size();
            prop_cache_.clear();  // (slots renumbered)
        }
        return pid >= 0 && (size_t)pid < watched_pid_.size() && watched_pid_[(size_t)pid];
    }
    // One write of the mirror: the first host common hook it raises is NFCKernelModule's (registered on
    // every property / record at creation, KM:166 / KM:186, before any per-object callback) and is the
    // adapter's own, not forwarded; what the per-object callbacks write meanwhile is forwarded as usual.
    struct MirrorMark {
        bool on = false;
        NFGUID self;
        const std::string* name = nullptr;
        int row = -1, col = -1;
    };
    template <class F>
    void Mirror(const NFGUID& self, const std::string& name, int row, int col, F&& f) {
        mw_.on = true;
        mw_.self = self;
        mw_.name = &name;
        mw_.row = row;
        mw_.col = col;
        mirroring_ = true;
        f();
        mirroring_ = false;
        mw_.on = false;
    }
    // the property the running mirror write sets (a device property of a device object: its host common
    // callbacks receive nothing, as DevProp would say after an NFGUID lookup)
    bool MirrorTarget(const NFGUID& self, const std::string& name) const {
        return mirroring_ && mw_.row < 0 && self == mw_.self && name == *mw_.name;
    }
    bool mirroring_ = false;  // inside Mirror (mw_ keeps its target after OwnWrite cleared mw_.on)
    bool OwnWrite(const NFGUID& self, const std::string& name, int row, int col) {
        if (!mw_.on || self != mw_.self || row != mw_.row || col != mw_.col || name != *mw_.name) return false;
        mw_.on = false;
        return true;
    }
    // an int / f64 host property set to a device value (bits)
    static void PutValue(const NF_SHARE_PTR<NFIProperty>& p, uint64_t bits) {
        if (p->GetType() == TDATA_INT) {
            if (p->GetInt() != (NFINT64)bits) p->SetInt((NFINT64)bits);
        } else if (p->GetType() == TDATA_FLOAT) {
            const double v = dbl(bits), h = p->GetFloat();
            if (memcmp(&h, &v, 8) != 0 && !p->SetFloat(v)) {
                // (a coalesced change within NFCProperty::SetFloat's 1e-15, PR:314: stored as is)
                NFIDataList::TData t;
                t.SetFloat(v);
                p->SetValue(t);
            }
        }
    }

    // A stale object's host mirror brought up to date from the device (its device properties and the
    // used rows' int cells of its device records, batched device reads), each write quiet for the common
    // hook.  Nothing of it has a per-object callback (that object would be eager).
    void SyncObject(const NFGUID& self) {
        if (!DevObject(self)) return;
        const int o = gpu_.ObjectIndex(to_gpu(self));
        if (o < 0 || (size_t)o >= mstate_.size() || !(mstate_[(size_t)o] & kStale)) return;
        mstate_[(size_t)o] &= (uint8_t)~kStale;
        NF_SHARE_PTR<NFIObject> ob = GetElement(self);
        if (!ob) return;
        n_syncs_++;
        std::vector<NF_SHARE_PTR<NFIProperty>>& ps = sy_props_;
        std::vector<int32_t>& pid = sy_pid_;
        ps.clear();
        pid.clear();
        NF_SHARE_PTR<NFIPropertyManager> pm = ob->GetPropertyManager();
        for (NF_SHARE_PTR<NFIProperty> p = pm->First(); p; p = pm->Next()) {
            if (!dev_props_.count(p->GetKey())) continue;
            ps.push_back(p);
            pid.push_back(gpu_.PropertyId(p->GetKey()));
        }
        const int ob0 = gpu_.PropertyCount(nfgpu::TDATA_INT) + gpu_.PropertyCount(nfgpu::TDATA_FLOAT);
        std::vector<int64_t> h, d, vh, vd;
        std::vector<int32_t> qp;
        std::vector<uint64_t> v;
        for (int pass = 0; pass < 2; pass++) {  // int / f64 words, then the object columns' NFGUIDs
            h.clear();
            d.clear();
            qp.clear();
            for (size_t i = 0; i < ps.size(); i++)
                if ((pid[i] >= ob0) == (pass == 1)) {
                    h.push_back(self.nHead64);
                    d.push_back(self.nData64);
                    qp.push_back(pid[i]);
                }
            if (qp.empty()) continue;
            v.assign(qp.size(), 0);
            vh.assign(qp.size(), 0);
            vd.assign(qp.size(), 0);
            gpu_.Flush();
            const int rc = pass ? nfk_get_objects(gpu_.World(), (int32_t)qp.size(), h.data(), d.data(), qp.data(), vh.data(), vd.data())
                                : nfk_get_props(gpu_.World(), (int32_t)qp.size(), h.data(), d.data(), qp.data(), v.data());
            if (rc != NFK_OK) throw std::runtime_error(std::string("host mirror read: ") + nfk_last_error());
            for (size_t i = 0, j = 0; i < ps.size(); i++) {
                if ((pid[i] >= ob0) != (pass == 1)) continue;
                Mirror(self, ps[i]->GetKey(), -1, -1, [&] {
                    if (pass) {
                        const NFGUID g(vh[j], vd[j]);
                        if (ps[i]->GetObject() != g) ps[i]->SetObject(g);
                    } else {
                        PutValue(ps[i], v[j]);
                    }
                });
                j++;
            }
        }
        // int cells of the used rows of its device records
        NF_SHARE_PTR<NFIRecordManager> rm = ob->GetRecordManager();
        std::vector<NF_SHARE_PTR<NFIRecord>> rs;
        std::vector<int32_t> cr, crow, ccol;
        h.clear();
        d.clear();
        for (NF_SHARE_PTR<NFIRecord> r = rm->First(); r; r = rm->Next()) {
            if (!dev_records_.count(r->GetName())) continue;
            const int rid = gpu_.RecordId(r->GetName());
            for (int row = 0; row < r->GetRows(); row++) {
                if (!r->IsUsed(row)) continue;
                for (int c = 0; c < r->GetCols(); c++) {
                    if (r->GetColType(c) != TDATA_INT) continue;
                    rs.push_back(r);
                    h.push_back(self.nHead64);
                    d.push_back(self.nData64);
                    cr.push_back(rid);
                    crow.push_back(row);
                    ccol.push_back(c);
                }
            }
        }
        if (!rs.empty()) {
            v.assign(rs.size(), 0);
            if (nfk_get_records(gpu_.World(), (int32_t)rs.size(), h.data(), d.data(), cr.data(), crow.data(), ccol.data(),
                                v.data()) != NFK_OK)
                throw std::runtime_error(std::string("host mirror read: ") + nfk_last_error());
            for (size_t i = 0; i < rs.size(); i++)
                if (rs[i]->GetInt(crow[i], ccol[i]) != (NFINT64)v[i])
                    Mirror(self, rs[i]->GetName(), crow[i], ccol[i], [&] { rs[i]->SetInt(crow[i], ccol[i], (NFINT64)v[i]); });
        }
    }

    // the host object's device properties as the device object's creation-time values
    void MirrorObject(const NF_SHARE_PTR<NFIObject>& o) {
        std::map<std::string, nfgpu::TData> init;
        NF_SHARE_PTR<NFIPropertyManager> pm = o->GetPropertyManager();
        for (NF_SHARE_PTR<NFIProperty> p = pm->First(); p; p = pm->Next()) {
            if (!dev_props_.count(p->GetKey())) continue;
            nfgpu::TData v;
            v.type = to_gpu(p->GetType());
            v.i = p->GetInt();
            v.f = p->GetFloat();
            v.o = to_gpu(p->GetObject());
            init[p->GetKey()] = v;
        }
        const std::string cls = o->GetPropertyString(NFrame::IObject::ClassName());
        const NFGUID self = o->Self();
        gpu_.CreateObject(to_gpu(self), (int)o->GetPropertyInt(NFrame::IObject::SceneID()),
                          (int)o->GetPropertyInt(NFrame::IObject::GroupID()), cls, init);
        const int idx = gpu_.ObjectIndex(to_gpu(self));
        if (idx >= 0) {
            uint8_t& m = State(idx);
            auto pe = pre_eager_.find(self);
            m = eager_all_ ? (uint8_t)(kEager | kMirrorAll) : pe != pre_eager_.end() ? pe->second : (uint8_t)0;
            if (pe != pre_eager_.end()) pre_eager_.erase(pe);
        }
    }
    // (before AfterInit) the rows the host object's device records already hold: their state at frame 0
    void MirrorRecords(const NF_SHARE_PTR<NFIObject>& o) {
        NF_SHARE_PTR<NFIRecordManager> rm = o->GetRecordManager();
        for (NF_SHARE_PTR<NFIRecord> r = rm->First(); r; r = rm->Next()) {
            if (!dev_records_.count(r->GetName())) continue;
            const int rows = r->GetRows(), cols = r->GetCols();
            uint64_t used = 0;
            std::vector<uint64_t> cells((size_t)rows * cols, 0);
            for (int row = 0; row < rows; row++) {
                if (!r->IsUsed(row)) continue;
                used |= 1ull << row;
                for (int c = 0; c < cols; c++) {
                    uint64_t b;
                    if (r->GetColType(c) == TDATA_INT) {
                        b = (uint64_t)r->GetInt(row, c);
                    } else {
                        const double v = r->GetFloat(row, c);
                        memcpy(&b, &v, 8);
                    }
                    cells[(size_t)c * rows + row] = b;
                }
            }
            if (used) gpu_.SetCreationRecord(to_gpu(o->Self()), r->GetName(), used, cells);
        }
    }
    // A call goes to the device when the object is in the device world and the property / record is
    // one of the device's; an object being created (before MirrorObject) is the host's alone, so the
    // class-event handlers and the AOI module's creation-time reads and writes (KM:146-267, AOI:227-258)
    // see the host object, exactly as in the reference, and its final values enter the device.
    bool DevObject(const NFGUID& self) const { return gpu_.ObjectIndex(to_gpu(self)) >= 0; }
    // (asked by the common-callback wrappers on every host property / record event: one hash, not a tree walk)
    bool DevProp(const NFGUID& self, const std::string& name) const { return dev_prop_ix_.find(name) >= 0 && DevObject(self); }
    bool DevRecord(const NFGUID& self, const std::string& rec) const { return dev_rec_ix_.find(rec) >= 0 && DevObject(self); }
    int ColOf(const std::string& rec, const std::string& tag) const {  // NFCRecord::GetCol (RC:1319)
        auto r = col_tags_.find(rec);
        if (r == col_tags_.end()) return -1;
        auto c = r->second.find(tag);
        return c == r->second.end() ? -1 : c->second;
    }

    void FlushCreationSchedules() {
        if (creation_sched_.empty()) return;
        std::vector<DeferredSchedule> q;
        q.swap(creation_sched_);
        for (DeferredSchedule& d : q) {
            if (!DevObject(d.self)) {  // (still being created: an outer CreateObject's own objects)
                creation_sched_.push_back(std::move(d));
                continue;
            }
            const nfgpu::NFGUID g = to_gpu(d.self);
            if (d.op == 1) gpu_.AddSchedule(g, d.name, d.cb, d.t, d.count, d.now);
            else if (d.op == 2) gpu_.RemoveSchedule(g, d.name);
            else gpu_.RemoveSchedule(g);
        }
    }
    void DropCreationSchedules(const NFGUID& self) {
        creation_sched_.erase(std::remove_if(creation_sched_.begin(), creation_sched_.end(),
                                             [&](const DeferredSchedule& d) { return d.self == self; }),
                              creation_sched_.end());
    }
    // the host object of a device object index (OnFrame's per-Set callbacks: no NFGUID map walk per Set),
    // and the NFIProperty of a watched property (WatchedSlot) per object
    NFIObject* HostObject(int o) {
        if ((size_t)o < host_obj_.size() && host_obj_[(size_t)o]) return host_obj_[(size_t)o];
        NF_SHARE_PTR<NFIObject> ob = GetElement(to_ref(gpu_.ObjectGuid(o)));
        if (!ob) return nullptr;
        if ((size_t)o >= host_obj_.size()) host_obj_.resize((size_t)gpu_.ObjectCount() + 1024, nullptr);
        host_obj_[(size_t)o] = ob.get();  // (NFCKernelModule holds it until DestroyObject, which clears this)
        return ob.get();
    }
    // a device object's host object, brought up to date first (SyncObject); null for any other object
    NFIObject* SyncedHostObject(const NFGUID& self) {
        const int o = gpu_.ObjectIndex(to_gpu(self));
        if (o < 0) {
            SyncObject(self);
            return nullptr;
        }
        if ((size_t)o < mstate_.size() && (mstate_[(size_t)o] & kStale)) SyncObject(self);
        return HostObject(o);
    }
    NFIProperty* HostProperty(int o, int pid, const std::string& name) {
        const int w = WatchedSlot(pid);
        const size_t at = (size_t)o * watched_slots_ + (size_t)w;
        if (w >= 0 && at < prop_cache_.size() && prop_cache_[at]) return prop_cache_[at];
        NFIObject* ob = HostObject(o);
        NF_SHARE_PTR<NFIProperty> p = ob ? ob->GetPropertyManager()->GetElement(name) : nullptr;
        if (!p) return nullptr;
        if (w >= 0) {
            if (at >= prop_cache_.size()) prop_cache_.resize(((size_t)gpu_.ObjectCount() + 1024) * watched_slots_, nullptr);
            prop_cache_[at] = p.get();  // (the object's property manager holds it)
        }
        return p.get();
    }
    int WatchedSlot(int pid) {
        WatchedPid(pid);  // (the table current)
        return pid >= 0 && (size_t)pid < watched_slot_.size() ? watched_slot_[(size_t)pid] : -1;
    }
    void ForgetHostObject(const NFGUID& self) {
        const int o = gpu_.ObjectIndex(to_gpu(self));
        if (o < 0) return;
        if ((size_t)o < host_obj_.size()) host_obj_[(size_t)o] = nullptr;
        for (size_t w = 0; w < watched_slots_; w++)
            if ((size_t)o * watched_slots_ + w < prop_cache_.size()) prop_cache_[(size_t)o * watched_slots_ + w] = nullptr;
    }

    NFIClassModule* m_pClassModule = nullptr;
    std::set<std::string> dev_props_, dev_records_;
    nfgpu_detail::NameIndex dev_prop_ix_, dev_rec_ix_;  // (the same names: DevProp / DevRecord)
    std::map<std::string, std::map<std::string, int>> col_tags_;
    std::set<int> scenes_;
    NFGUID obj_scratch_;
    int quiet_ = 0;  // > 0: host writes are the adapter's own (SwitchScene), not forwarded
    MirrorMark mw_;
    std::vector<Common<PROPERTY_EVENT_FUNCTOR_PTR>> prop_cb_;
    std::vector<Common<RECORD_EVENT_FUNCTOR_PTR>> rec_cb_;
    NFGPUDeviceAOI* aoi_ = nullptr;
    bool aoi_registering_ = false;
    int64_t aoi_host_calls_ = 0, aoi_host_device_calls_ = 0, aoi_device_calls_ = 0;
    int64_t n_syncs_ = 0, n_chain_fired_ = 0;
    NFCDataList rl_, none_;  // the recipient list last built, and the empty one
    bool rl_valid_ = false;
    RECORD_EVENT_DATA rev_;
    // host mirror state per device object index (kStale / kEager), objects made eager before they
    // reached the device, watched device properties
    std::vector<uint8_t> mstate_;
    std::unordered_map<NFGUID, uint8_t, GuidHash> pre_eager_;
    bool eager_all_ = false;
    std::set<std::string> watched_;
    std::vector<uint8_t> watched_pid_;  // (WatchedPid's table, rebuilt when watched_ grows)
    std::vector<int> watched_slot_;     // device pid -> index among the watched properties (-1: none)
    size_t watched_n_ = 0, watched_slots_ = 0;
    std::vector<NFIObject*> host_obj_;    // (HostObject)
    std::vector<NFIProperty*> prop_cache_;  // (HostProperty: [object][watched slot])
    std::vector<NFGUID> creating_;        // CreateObject calls in progress (nested: class callbacks may create)
    std::vector<DeferredSchedule> creation_sched_;
    std::vector<std::string> watch_pending_;
    std::map<uint16_t, std::pair<int, int>> rec_op_;  // (rec << 8 | col) -> (kind, op index)
    std::unordered_map<NFGUID, NF_SHARE_PTR<NFIObject>, GuidHash> handles_;
    std::set<std::string> class_names_;
    std::unordered_map<NFGUID, const std::string*, GuidHash> class_of_;
    NFCDataList gl_scratch_;
    std::set<NFGUID> has_components_;  // objects whose component manager was handed out (Execute walks them)
    std::vector<NFGUID> walk_;          // Execute's copy of has_components_
    NFGUID cur_exe_;                    // the object whose components Execute is running (KM's mnCurExeObject)
    // (scratch kept across frames)
    std::vector<int64_t> fr_ep_, fr_er_;
    std::vector<int> written_;  // objects with kWritten (OnFrame)
    std::vector<Fire> fr_fire_;
    std::vector<NF_SHARE_PTR<NFIProperty>> sy_props_;
    std::vector<int32_t> sy_pid_;
};

// The object handle NFGPUKernelAdapter hands out (GetObject, CreateObject): the host NFCObject behind
// it, brought up to date from the device before any read or write; a per-object callback registered
// through it (NFIObject::AddPropertyCallBack / AddRecordCallBack, NFIObject.h:155-157 — what
// NFIKernelModule::AddPropertyCallBack calls, NFIKernelModule.h:40-45) makes the object eager and its
// device property watched (per-Set callbacks, see the header).  Its managers handed out make it eager.
class NFGPUObject : public NFIObject {
public:
    NFGPUObject(NFGPUKernelAdapter* k, const NFGUID& self, const NF_SHARE_PTR<NFIObject>& in)
        : NFIObject(self), k_(k), self_(self), in_(in) {}
    NFIObject* Inner() const { return in_.get(); }

    bool Execute() override { return in_->Execute(); }
    NFGUID Self() override { return self_; }
    CLASS_OBJECT_EVENT GetState() override { return in_->GetState(); }
    bool SetState(const CLASS_OBJECT_EVENT e) override { return in_->SetState(e); }
    bool FindProperty(const std::string& n) override { return in_->FindProperty(n); }

    bool SetPropertyInt(const std::string& n, const NFINT64 v) override { return T()->SetPropertyInt(n, v); }
    bool SetPropertyFloat(const std::string& n, const double v) override { return T()->SetPropertyFloat(n, v); }
    bool SetPropertyString(const std::string& n, const std::string& v) override {
        const bool ok = T()->SetPropertyString(n, v);
        if (n == NFrame::IObject::ClassName()) k_->ClassNameChanged(self_);
        return ok;
    }
    bool SetPropertyObject(const std::string& n, const NFGUID& v) override { return T()->SetPropertyObject(n, v); }
    bool SetPropertyVector2(const std::string& n, const NFVector2& v) override { return T()->SetPropertyVector2(n, v); }
    bool SetPropertyVector3(const std::string& n, const NFVector3& v) override { return T()->SetPropertyVector3(n, v); }
    NFINT64 GetPropertyInt(const std::string& n) override {
        return k_->WalkRead(self_, n) ? k_->GetPropertyInt(self_, n) : T()->GetPropertyInt(n);
    }
    double GetPropertyFloat(const std::string& n) override {
        return k_->WalkRead(self_, n) ? k_->GetPropertyFloat(self_, n) : T()->GetPropertyFloat(n);
    }
    const std::string& GetPropertyString(const std::string& n) override { return in_->GetPropertyString(n); }
    const NFGUID& GetPropertyObject(const std::string& n) override { return T()->GetPropertyObject(n); }
    const NFVector2& GetPropertyVector2(const std::string& n) override { return in_->GetPropertyVector2(n); }
    const NFVector3& GetPropertyVector3(const std::string& n) override { return in_->GetPropertyVector3(n); }

    bool FindRecord(const std::string& r) override { return in_->FindRecord(r); }
    bool SetRecordInt(const std::string& r, const int row, const int col, const NFINT64 v) override { return T()->SetRecordInt(r, row, col, v); }
    bool SetRecordFloat(const std::string& r, const int row, const int col, const double v) override { return T()->SetRecordFloat(r, row, col, v); }
    bool SetRecordString(const std::string& r, const int row, const int col, const std::string& v) override { return in_->SetRecordString(r, row, col, v); }
    bool SetRecordObject(const std::string& r, const int row, const int col, const NFGUID& v) override { return in_->SetRecordObject(r, row, col, v); }
    bool SetRecordVector2(const std::string& r, const int row, const int col, const NFVector2& v) override { return in_->SetRecordVector2(r, row, col, v); }
    bool SetRecordVector3(const std::string& r, const int row, const int col, const NFVector3& v) override { return in_->SetRecordVector3(r, row, col, v); }
    bool SetRecordInt(const std::string& r, const int row, const std::string& t, const NFINT64 v) override { return T()->SetRecordInt(r, row, t, v); }
    bool SetRecordFloat(const std::string& r, const int row, const std::string& t, const double v) override { return T()->SetRecordFloat(r, row, t, v); }
    bool SetRecordString(const std::string& r, const int row, const std::string& t, const std::string& v) override { return in_->SetRecordString(r, row, t, v); }
    bool SetRecordObject(const std::string& r, const int row, const std::string& t, const NFGUID& v) override { return in_->SetRecordObject(r, row, t, v); }
    bool SetRecordVector2(const std::string& r, const int row, const std::string& t, const NFVector2& v) override { return in_->SetRecordVector2(r, row, t, v); }
    bool SetRecordVector3(const std::string& r, const int row, const std::string& t, const NFVector3& v) override { return in_->SetRecordVector3(r, row, t, v); }
    NFINT64 GetRecordInt(const std::string& r, const int row, const int col) override { return T()->GetRecordInt(r, row, col); }
    double GetRecordFloat(const std::string& r, const int row, const int col) override { return T()->GetRecordFloat(r, row, col); }
    const std::string& GetRecordString(const std::string& r, const int row, const int col) override { return in_->GetRecordString(r, row, col); }
    const NFGUID& GetRecordObject(const std::string& r, const int row, const int col) override { return in_->GetRecordObject(r, row, col); }
    const NFVector2& GetRecordVector2(const std::string& r, const int row, const int col) override { return in_->GetRecordVector2(r, row, col); }
    const NFVector3& GetRecordVector3(const std::string& r, const int row, const int col) override { return in_->GetRecordVector3(r, row, col); }
    NFINT64 GetRecordInt(const std::string& r, const int row, const std::string& t) override { return T()->GetRecordInt(r, row, t); }
    double GetRecordFloat(const std::string& r, const int row, const std::string& t) override { return T()->GetRecordFloat(r, row, t); }
    const std::string& GetRecordString(const std::string& r, const int row, const std::string& t) override { return in_->GetRecordString(r, row, t); }
    const NFGUID& GetRecordObject(const std::string& r, const int row, const std::string& t) override { return in_->GetRecordObject(r, row, t); }
    const NFVector2& GetRecordVector2(const std::string& r, const int row, const std::string& t) override { return in_->GetRecordVector2(r, row, t); }
    const NFVector3& GetRecordVector3(const std::string& r, const int row, const std::string& t) override { return in_->GetRecordVector3(r, row, t); }

    // handed out: whatever is registered on or read from them later, the object stays current
    NF_SHARE_PTR<NFIRecordManager> GetRecordManager() override {
        k_->Watched(self_, "");
        return in_->GetRecordManager();
    }
    NF_SHARE_PTR<NFIPropertyManager> GetPropertyManager() override {
        k_->Watched(self_, "");
        return in_->GetPropertyManager();
    }
    NF_SHARE_PTR<NFIComponentManager> GetComponentManager() override {  // (components run in KM's walk)
        k_->HasComponents(self_);
        return in_->GetComponentManager();
    }
    // (what NFCObject::AddRecordCallBack / AddPropertyCallBack do, NFCObject.cpp:49-73: NFIObject
    // declares them protected)
    bool AddRecordCallBack(const std::string& r, const RECORD_EVENT_FUNCTOR_PTR& cb) override {
        k_->Watched(self_, "");
        NF_SHARE_PTR<NFIRecord> rec = in_->GetRecordManager()->GetElement(r);
        if (!rec) return false;
        rec->AddRecordHook(cb);
        return true;
    }
    bool AddPropertyCallBack(const std::string& p, const PROPERTY_EVENT_FUNCTOR_PTR& cb) override {
        k_->Watched(self_, p);
        NF_SHARE_PTR<NFIProperty> prop = in_->GetPropertyManager()->GetElement(p);
        if (!prop) return false;
        prop->RegisterCallback(cb);
        return true;
    }

private:
    NFIObject* T() {  // (the host object, current)
        k_->Touch(self_);
        return in_.get();
    }
    NFGPUKernelAdapter* k_;
    NFGUID self_;
    NF_SHARE_PTR<NFIObject> in_;
};

NF_SHARE_PTR<NFIObject> NFGPUKernelAdapter::Handle(const NFGUID& self, const NF_SHARE_PTR<NFIObject>& o) {
    auto it = handles_.find(self);
    if (it != handles_.end() && static_cast<NFGPUObject*>(it->second.get())->Inner() == o.get()) return it->second;
    NF_SHARE_PTR<NFIObject> h(new NFGPUObject(this, self, o));
    handles_[self] = h;
    return h;
}

// NFISceneAOIModule (NFISceneAOIModule.h) as the reference's NFCSceneAOIModule, with device events
// taken from the device frame: OnPropertyCommonEvent / OnRecordCommonEvent (AOI:227-288) without
// GetBroadCastObject — the device computed the recipient list (k_tick / k_records fan-out of
// GetBroadCastObject's rules, AOI:531-593) — straight to the protected OnPropertyEvent / OnRecordEvent
// (AOI:703-727), which call the AddPropertyEventCallBack / AddRecordEventCallBack functors.
class NFGPUSceneAOIAdapter : public NFCSceneAOIModule, public NFGPUDeviceAOI {
public:
    explicit NFGPUSceneAOIAdapter(NFIPluginManager* p) : NFCSceneAOIModule(p) {}
    bool Init() override {
        // the common callbacks NFCSceneAOIModule::Init registers (AOI.cpp:20-22) are marked as this
        // module's: the kernel adapter hands device events to DevicePropertyEvent / DeviceRecordEvent
        kernel_ = dynamic_cast<NFGPUKernelAdapter*>(pPluginManager->FindModule<NFIKernelModule>());
        if (kernel_) kernel_->BeginAOIRegistration(this);
        const bool ok = NFCSceneAOIModule::Init();
        if (kernel_) kernel_->EndAOIRegistration();
        return ok;
    }
    // AOI:227-256 for a device property: GroupID / SceneID run the enter / leave handlers; a device
    // object has finished its creation (the COE_CREATE_FINISH test of AOI:240-247 holds); an empty
    // list makes no call (AOI:250)
    void DevicePropertyEvent(const NFGUID& self, const std::string& name, const NFIDataList::TData& oldVar,
                             const NFIDataList::TData& newVar, const NFIDataList& to) override {
        if (NFrame::Player::GroupID() == name) OnGroupEvent(self, name, oldVar, newVar);
        if (NFrame::Player::SceneID() == name) OnSceneEvent(self, name, oldVar, newVar);
        if (to.GetCount() <= 0) return;
        OnPropertyEvent(self, name, oldVar, newVar, to);
    }
    // AOI:260-288 for a device record (the kernel adapter applied the GroupID < 0 test, AOI:270-276)
    void DeviceRecordEvent(const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& oldVar,
                           const NFIDataList::TData& newVar, const NFIDataList& to) override {
        OnRecordEvent(self, ev.strRecordName, ev, oldVar, newVar, to);
    }

private:
    NFGPUKernelAdapter* kernel_ = nullptr;
};

class NFGPUScheduleAdapter : public NFIScheduleModule {
public:
    explicit NFGPUScheduleAdapter(NFIPluginManager* p) : host_(p) { pPluginManager = p; }
    bool Init() override { return host_.Init(); }

    // ---- module schedules (NFIScheduleModule.h:23-25): the reference's own NFCScheduleModule ----
    bool AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR_PTR& cb, const float fTime,
                     const int nCount) override {
        return host_.AddSchedule(name, cb, fTime, nCount);
    }
    bool RemoveSchedule(const std::string& name) override { return host_.RemoveSchedule(name); }
    bool ExistSchedule(const std::string& name) override { return host_.ExistSchedule(name); }

    // ---- object schedules (NFIScheduleModule.h:36-39): a name with a device program runs on the
    // device (its functor after the device frame); any other name — a functor-only heartbeat such as
    // Tutorial3's OnHeartBeat (HelloWorld3Module.cpp:47) — on the host NFCScheduleModule, whose
    // Execute runs at this module's Execute as in the reference ----
    bool AddSchedule(const NFGUID self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR_PTR& cb,
                     const float fTime, const int nCount) override {  // SM:257
        if (!gpu().HasHeartBeat(name)) return host_.AddSchedule(self, name, cb, fTime, nCount);
        nfgpu::OBJECT_SCHEDULE_FUNCTOR f = [cb](const nfgpu::NFGUID& g, const std::string& n, const float t, const int c) {
            return (*cb)(to_ref(g), n, t, c);
        };
        if (kernel()->DeferSchedule(self)) {  // (its object is being created: made once it is on the device)
            kernel()->QueueCreationSchedule({1, self, name, f, fTime, nCount, NFGetTime()});
            return true;
        }
        return gpu().AddSchedule(to_gpu(self), name, f, fTime, nCount);
    }
    bool RemoveSchedule(const NFGUID self) override {  // SM:240
        if (kernel()->DeferSchedule(self)) kernel()->QueueCreationSchedule({3, self, "", nullptr, 0.f, 0, 0});
        const bool d = gpu().RemoveSchedule(to_gpu(self));
        const bool h = host_.RemoveSchedule(self);
        return d || h;
    }
    bool RemoveSchedule(const NFGUID self, const std::string& name) override {  // SM:245
        if (!gpu().HasHeartBeat(name)) return host_.RemoveSchedule(self, name);
        if (kernel()->DeferSchedule(self)) {
            kernel()->QueueCreationSchedule({2, self, name, nullptr, 0.f, 0, 0});
            return true;
        }
        return gpu().RemoveSchedule(to_gpu(self), name);
    }
    bool ExistSchedule(const NFGUID self, const std::string& name) override {  // SM:276
        if (!gpu().HasHeartBeat(name)) return host_.ExistSchedule(self, name);
        // (SM:276 sees an AddSchedule only after the Execute that applies it: one queued at creation is not there yet)
        if (kernel()->DeferSchedule(self)) return false;
        return gpu().ExistSchedule(to_gpu(self), name);
    }
    // the device frame (its object schedules) runs in NFGPUKernelAdapter::Execute; the host
    // schedules here
    bool Execute() override { return host_.Execute(); }

private:
    NFGPUKernelAdapter* kernel() { return dynamic_cast<NFGPUKernelAdapter*>(pPluginManager->FindModule<NFIKernelModule>()); }
    nfgpu::NFGPUKernelModule& gpu() { return kernel()->gpu_; }
    NFCScheduleModule host_;
};

class NFGPUKernelPlugin : public NFIPlugin {
public:
    explicit NFGPUKernelPlugin(NFIPluginManager* p) { pPluginManager = p; }
    const int GetPluginVersion() override { return 0; }
    const std::string GetPluginName() override { return GET_CLASS_NAME(NFGPUKernelPlugin); }
    void Install() override {
        REGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFGPUSceneAOIAdapter)  // enter / leave, client sync
        REGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        REGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        REGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
    }
    void Uninstall() override {
        UNREGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
        UNREGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        UNREGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        UNREGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFGPUSceneAOIAdapter)
    }
};

#ifdef NF_DYNAMIC_PLUGIN
NF_EXPORT void DllStartPlugin(NFIPluginManager* pm) { CREATE_PLUGIN(pm, NFGPUKernelPlugin) }
NF_EXPORT void DllStopPlugin(NFIPluginManager* pm) { DESTROY_PLUGIN(pm, NFGPUKernelPlugin) }
#endif
