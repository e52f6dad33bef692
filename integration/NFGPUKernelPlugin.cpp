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
//   NFGPUScheduleAdapter  NFIScheduleModule (NFIScheduleModule.h:23-39): object schedules on the
//                         device, module schedules on the host.
//   NFGPUKernelPlugin     the NFIPlugin that registers both (NFKernelPlugin.cpp:40-46 pattern).
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCSceneAOIModule.h"
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
}  // namespace

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
                dev_props_.insert(p->GetKey());
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
        return gpu_.AfterInit();
    }

    bool Execute() override {  // NFCKernelModule::Execute (KM:70) + NFCScheduleModule::Execute (SM:49) + AOI fan-out
        NFCKernelModule::Execute();
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
    NF_SHARE_PTR<NFIObject> CreateObject(const NFGUID& self, const int nSceneID, const int nGroupID,
                                         const std::string& strClassName, const std::string& strConfigIndex,
                                         const NFIDataList& arg) override {
        NF_SHARE_PTR<NFIObject> o = NFCKernelModule::CreateObject(self, nSceneID, nGroupID, strClassName, strConfigIndex, arg);
        if (o && !dev_props_.empty()) MirrorObject(o);
        return o;
    }

    // the reference's DestroyObject reads SceneID / GroupID through GetPropertyInt (KM:283-284),
    // which this adapter answers from the device: it runs while the object is still there
    bool DestroyObject(const NFGUID& self) override {  // KM:273
        const bool ok = NFCKernelModule::DestroyObject(self);
        gpu_.DestroyObject(to_gpu(self));
        return ok;
    }

    bool SetPropertyInt(const NFGUID& self, const std::string& name, const NFINT64 v) override {  // KM:323
        return DevProp(self, name) ? gpu_.SetPropertyInt(to_gpu(self), name, v) : NFCKernelModule::SetPropertyInt(self, name, v);
    }
    bool SetPropertyFloat(const NFGUID& self, const std::string& name, const double v) override {  // KM:336
        return DevProp(self, name) ? gpu_.SetPropertyFloat(to_gpu(self), name, v)
                                      : NFCKernelModule::SetPropertyFloat(self, name, v);
    }
    bool SetPropertyObject(const NFGUID& self, const std::string& name, const NFGUID& v) override {  // KM:362
        return DevProp(self, name) ? gpu_.SetPropertyObject(to_gpu(self), name, to_gpu(v))
                                      : NFCKernelModule::SetPropertyObject(self, name, v);
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

    bool ClearRecord(const NFGUID& self, const std::string& rec) override {  // KM:492
        return DevRecord(self, rec) ? gpu_.ClearRecord(to_gpu(self), rec) : NFCKernelModule::ClearRecord(self, rec);
    }
    bool SetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const int nCol,
                      const NFINT64 v) override {  // KM:505
        return DevRecord(self, rec) ? gpu_.SetRecordInt(to_gpu(self), rec, nRow, nCol, v)
                                       : NFCKernelModule::SetRecordInt(self, rec, nRow, nCol, v);
    }
    bool SetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const int nCol,
                        const double v) override {  // KM:545
        return DevRecord(self, rec) ? gpu_.SetRecordFloat(to_gpu(self), rec, nRow, nCol, v)
                                       : NFCKernelModule::SetRecordFloat(self, rec, nRow, nCol, v);
    }
    // the column-tag forms (NFIKernelModule.h:127-128, KM:525): NFCRecord::GetCol of the tag
    bool SetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag,
                      const NFINT64 v) override {
        if (!DevRecord(self, rec)) return NFCKernelModule::SetRecordInt(self, rec, nRow, tag, v);
        const int c = ColOf(rec, tag);
        return c >= 0 && gpu_.SetRecordInt(to_gpu(self), rec, nRow, c, v);
    }
    bool SetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const std::string& tag,
                        const double v) override {
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
        NFCKernelModule::SwitchScene(self, scene, group, fX, fY, fZ, fOrient, arg);  // host-side scene lists
        return gpu_.SwitchScene(to_gpu(self), scene, group, fX, fY, fZ, fOrient);
    }

    nfgpu::NFGPUKernelModule gpu_;

protected:
    // Common property / record callbacks (NFIKernelModule.h:181-182): the device's coalesced events
    // for its properties and records (delivered by Execute), the host's for the rest (strings,
    // vectors, host-only records).  The AOI module registers its OnPropertyCommonEvent /
    // OnRecordCommonEvent (AOI:227, 260) here, so its client sync runs from the device event list.
    bool RegisterCommonPropertyEvent(const PROPERTY_EVENT_FUNCTOR_PTR& cb) override {
        PROPERTY_EVENT_FUNCTOR_PTR host(new PROPERTY_EVENT_FUNCTOR(
            [this, cb](const NFGUID& self, const std::string& name, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                return DevProp(self, name) ? 0 : (*cb)(self, name, a, b);
            }));
        NFCKernelModule::RegisterCommonPropertyEvent(host);
        return gpu_.RegisterCommonPropertyEvent(
            [cb](const nfgpu::NFGUID& self, const std::string& name, const nfgpu::TData& a, const nfgpu::TData& b) {
                return (*cb)(to_ref(self), name, to_ref(a), to_ref(b));
            });
    }
    bool RegisterCommonRecordEvent(const RECORD_EVENT_FUNCTOR_PTR& cb) override {
        RECORD_EVENT_FUNCTOR_PTR host(new RECORD_EVENT_FUNCTOR(
            [this, cb](const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                return DevRecord(self, ev.strRecordName) ? 0 : (*cb)(self, ev, a, b);
            }));
        NFCKernelModule::RegisterCommonRecordEvent(host);
        return gpu_.RegisterCommonRecordEvent(
            [cb](const nfgpu::NFGUID& self, const nfgpu::RECORD_EVENT_DATA& e, const nfgpu::TData& a, const nfgpu::TData& b) {
                RECORD_EVENT_DATA ev;
                ev.nOpType = (RECORD_EVENT_DATA::RecordOptype)e.nOpType;
                ev.nRow = e.nRow;
                ev.nCol = e.nCol;
                ev.strRecordName = e.strRecordName;
                return (*cb)(to_ref(self), ev, to_ref(a), to_ref(b));
            });
    }

private:
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
        gpu_.CreateObject(to_gpu(o->Self()), (int)o->GetPropertyInt(NFrame::IObject::SceneID()),
                          (int)o->GetPropertyInt(NFrame::IObject::GroupID()), cls, init);
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
    bool DevProp(const NFGUID& self, const std::string& name) const {
        return dev_props_.count(name) && gpu_.ObjectIndex(to_gpu(self)) >= 0;
    }
    bool DevRecord(const NFGUID& self, const std::string& rec) const {
        return dev_records_.count(rec) && gpu_.ObjectIndex(to_gpu(self)) >= 0;
    }
    int ColOf(const std::string& rec, const std::string& tag) const {  // NFCRecord::GetCol (RC:1319)
        auto r = col_tags_.find(rec);
        if (r == col_tags_.end()) return -1;
        auto c = r->second.find(tag);
        return c == r->second.end() ? -1 : c->second;
    }

    NFIClassModule* m_pClassModule = nullptr;
    std::set<std::string> dev_props_, dev_records_;
    std::map<std::string, std::map<std::string, int>> col_tags_;
    std::set<int> scenes_;
    NFGUID obj_scratch_;
};

class NFGPUScheduleAdapter : public NFIScheduleModule {
public:
    explicit NFGPUScheduleAdapter(NFIPluginManager* p) { pPluginManager = p; }

    // ---- module schedules (NFIScheduleModule.h:23-25) ----
    bool AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR_PTR& cb, const float fTime,
                     const int nCount) override {
        return gpu().AddSchedule(name,
                                 [cb](const std::string& n, const float t, const int c) { return (*cb)(n, t, c); },
                                 fTime, nCount);
    }
    bool RemoveSchedule(const std::string& name) override { return gpu().RemoveSchedule(name); }
    bool ExistSchedule(const std::string& name) override { return gpu().ExistSchedule(name); }

    // ---- object schedules (NFIScheduleModule.h:36-39) ----
    bool AddSchedule(const NFGUID self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR_PTR& cb,
                     const float fTime, const int nCount) override {  // SM:257
        return gpu().AddSchedule(
            to_gpu(self), name,
            [cb](const nfgpu::NFGUID& g, const std::string& n, const float t, const int c) { return (*cb)(to_ref(g), n, t, c); },
            fTime, nCount);
    }
    bool RemoveSchedule(const NFGUID self) override { return gpu().RemoveSchedule(to_gpu(self)); }  // SM:240
    bool RemoveSchedule(const NFGUID self, const std::string& name) override {                       // SM:245
        return gpu().RemoveSchedule(to_gpu(self), name);
    }
    bool ExistSchedule(const NFGUID self, const std::string& name) override {  // SM:276
        return gpu().ExistSchedule(to_gpu(self), name);
    }
    // the frame (object and module schedules) runs in NFGPUKernelAdapter::Execute
    bool Execute() override { return true; }

private:
    nfgpu::NFGPUKernelModule& gpu() {
        return dynamic_cast<NFGPUKernelAdapter*>(pPluginManager->FindModule<NFIKernelModule>())->gpu_;
    }
};

class NFGPUKernelPlugin : public NFIPlugin {
public:
    explicit NFGPUKernelPlugin(NFIPluginManager* p) { pPluginManager = p; }
    const int GetPluginVersion() override { return 0; }
    const std::string GetPluginName() override { return GET_CLASS_NAME(NFGPUKernelPlugin); }
    void Install() override {
        REGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFCSceneAOIModule)  // enter / leave, client sync
        REGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        REGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        REGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
    }
    void Uninstall() override {
        UNREGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
        UNREGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        UNREGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        UNREGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFCSceneAOIModule)
    }
};

#ifdef NF_DYNAMIC_PLUGIN
NF_EXPORT void DllStartPlugin(NFIPluginManager* pm) { CREATE_PLUGIN(pm, NFGPUKernelPlugin) }
NF_EXPORT void DllStopPlugin(NFIPluginManager* pm) { DESTROY_PLUGIN(pm, NFGPUKernelPlugin) }
#endif
