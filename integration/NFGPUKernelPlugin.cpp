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
//                         The host objects stay a mirror of the device ones (below), so per-object
//                         callbacks and direct NFIObject / NFIRecord access keep working.
//   NFGPUScheduleAdapter  NFIScheduleModule (NFIScheduleModule.h:23-39): object schedules whose name
//                         has a device program on the device; every other schedule (functor-only
//                         heartbeats, module schedules) on the reference's own NFCScheduleModule.
//
// Host objects as a mirror of the device (NFIKernelModule.h:28-45 AddPropertyCallBack /
// AddRecordCallBack register on the host NFCObject's NFCProperty / NFCRecord, NFCProperty.h:71):
//   * every write to a device property or int record cell goes to the HOST object first — through
//     NFIKernelModule (SetPropertyInt / Float / Object, SetRecordInt, ClearRecord) or straight
//     through the object (GetObject(self)->SetPropertyInt, FindRecord(self, r)->SetInt / AddRow /
//     Remove) — so the reference's change predicates and per-object callbacks run at call time as in
//     the reference; the host common event of that write is forwarded to the device (queued there)
//     instead of reaching the common callbacks;
//   * the common callbacks (the AOI module's client sync) receive the device's coalesced frame
//     events (the dirty-sync list), exactly as before;
//   * when Execute returns, every (object, property) and int cell that had a device event or a host
//     write this window is read back from the device and written into the host object where it
//     differs: the heartbeat programs' effects reach GetObject(self)->Get* and fire the per-object
//     callbacks (old = the host value, new = the device value).
//   f64 record cells are the exception: NFCRecord::SetFloat stores a double into the int64 alternative
//   of the cell (RC:243-297; tests/test_oracle.py::test_reference_record_setfloat_bug), so they are
//   device-only (SetRecordFloat / GetRecordFloat through NFIKernelModule read and write the device).
//   NFGPUKernelPlugin     the NFIPlugin that registers both (NFKernelPlugin.cpp:40-46 pattern).
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <tuple>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCScheduleModule.h"
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
        // host writes of device state -> the device (first in the host common lists: the modules
        // register their common callbacks in their own AfterInit, after this one)
        NFCKernelModule::RegisterCommonPropertyEvent(PROPERTY_EVENT_FUNCTOR_PTR(new PROPERTY_EVENT_FUNCTOR(
            [this](const NFGUID& self, const std::string& name, const NFIDataList::TData&, const NFIDataList::TData& v) {
                return ForwardProperty(self, name, v);
            })));
        NFCKernelModule::RegisterCommonRecordEvent(RECORD_EVENT_FUNCTOR_PTR(new RECORD_EVENT_FUNCTOR(
            [this](const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData&, const NFIDataList::TData&) {
                return ForwardRecord(self, ev);
            })));
        // the device's frame events -> the common callbacks, and their (object, property / cell) to
        // the host mirror when Execute returns
        gpu_.RegisterCommonPropertyEvent(
            [this](const nfgpu::NFGUID& self, const std::string& name, const nfgpu::TData& a, const nfgpu::TData& b) {
                const NFGUID s = to_ref(self);
                for (auto& cb : prop_cb_) (*cb)(s, name, to_ref(a), to_ref(b));
                sync_props_.emplace_back(s, name);
                return 0;
            });
        gpu_.RegisterCommonRecordEvent(
            [this](const nfgpu::NFGUID& self, const nfgpu::RECORD_EVENT_DATA& e, const nfgpu::TData& a, const nfgpu::TData& b) {
                RECORD_EVENT_DATA ev;
                ev.nOpType = (RECORD_EVENT_DATA::RecordOptype)e.nOpType;
                ev.nRow = e.nRow;
                ev.nCol = e.nCol;
                ev.strRecordName = e.strRecordName;
                const NFGUID s = to_ref(self);
                for (auto& cb : rec_cb_) (*cb)(s, ev, to_ref(a), to_ref(b));
                if (e.nOpType == nfgpu::RECORD_EVENT_DATA::Update && b.type == nfgpu::TDATA_INT)
                    sync_cells_.push_back({s, e.strRecordName, e.nRow, e.nCol});
                return 0;
            });
        return gpu_.AfterInit();
    }

    bool Execute() override {  // NFCKernelModule::Execute (KM:70) + NFCScheduleModule::Execute (SM:49) + AOI fan-out
        NFCKernelModule::Execute();
        const bool ok = gpu_.Execute();
        SyncHostObjects();
        return ok;
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

    // SetPropertyInt / Float / Object, SetRecordInt (by column and by tag), ClearRecord: the
    // reference's own NFCKernelModule on the host object (KM:323-372, 492-544); ForwardProperty /
    // ForwardRecord queue the accepted writes on the device.
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
        ++quiet_;
        NFCKernelModule::SwitchScene(self, scene, group, fX, fY, fZ, fOrient, arg);
        --quiet_;
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
        prop_cb_.push_back(cb);
        return true;
    }
    bool RegisterCommonRecordEvent(const RECORD_EVENT_FUNCTOR_PTR& cb) override {
        RECORD_EVENT_FUNCTOR_PTR host(new RECORD_EVENT_FUNCTOR(
            [this, cb](const NFGUID& self, const RECORD_EVENT_DATA& ev, const NFIDataList::TData& a, const NFIDataList::TData& b) {
                return DevRecord(self, ev.strRecordName) ? 0 : (*cb)(self, ev, a, b);
            }));
        NFCKernelModule::RegisterCommonRecordEvent(host);
        rec_cb_.push_back(cb);
        return true;
    }

private:
    struct Cell {
        NFGUID self;
        std::string rec;
        int row, col;
    };

    // an accepted host write of a device property (NFCProperty::SetInt / SetFloat / SetObject raised
    // the common event): queued on the device in call order
    int ForwardProperty(const NFGUID& self, const std::string& name, const NFIDataList::TData& v) {
        if (quiet_ || !DevProp(self, name)) return 0;
        const nfgpu::NFGUID g = to_gpu(self);
        if (v.GetType() == TDATA_INT) gpu_.SetPropertyInt(g, name, v.GetInt());
        else if (v.GetType() == TDATA_FLOAT) gpu_.SetPropertyFloat(g, name, v.GetFloat());
        else if (v.GetType() == TDATA_OBJECT) gpu_.SetPropertyObject(g, name, to_gpu(v.GetObject()));
        else return 0;
        sync_props_.emplace_back(self, name);
        return 0;
    }
    // an accepted host write of a device record (NFCRecord's Update / Add / Cover / Del events,
    // RC:170-177, 225-231, 1092-1098): the same call queued on the device
    int ForwardRecord(const NFGUID& self, const RECORD_EVENT_DATA& ev) {
        if (quiet_ || !DevRecord(self, ev.strRecordName)) return 0;
        NF_SHARE_PTR<NFIRecord> r = NFCKernelModule::FindRecord(self, ev.strRecordName);
        if (!r) return 0;
        const nfgpu::NFGUID g = to_gpu(self);
        switch (ev.nOpType) {
            case RECORD_EVENT_DATA::Update:
                // (an f64 cell written on the host holds the double in the int64 alternative and
                // cannot be read back: f64 record cells are device-only)
                if (r->GetColType(ev.nCol) == TDATA_INT) {
                    gpu_.SetRecordInt(g, ev.strRecordName, ev.nRow, ev.nCol, r->GetInt(ev.nRow, ev.nCol));
                    sync_cells_.push_back({self, ev.strRecordName, ev.nRow, ev.nCol});
                }
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

    // When Execute returns: the device values of the window's written and evented properties and
    // int cells, written into the host objects where they differ (one batched device read each);
    // the host NFCProperty / NFCRecord then fires the per-object callbacks for the difference.
    void SyncHostObjects() {
        gpu_.Flush();  // (this reads the world through the C-ABI)
        std::vector<std::pair<NFGUID, std::string>> props;
        props.swap(sync_props_);
        std::vector<Cell> cells;
        cells.swap(sync_cells_);
        std::sort(props.begin(), props.end());
        props.erase(std::unique(props.begin(), props.end()), props.end());
        std::vector<int64_t> gh, gd, oh;
        std::vector<int32_t> pid;
        std::vector<uint64_t> val;
        std::vector<size_t> at;  // props index of each device read
        for (size_t i = 0; i < props.size(); i++) {
            if (!DevProp(props[i].first, props[i].second)) continue;  // (destroyed / left the shard)
            at.push_back(i);
            gh.push_back(props[i].first.nHead64);
            gd.push_back(props[i].first.nData64);
            pid.push_back(gpu_.PropertyId(props[i].second));
        }
        if (!at.empty()) {
            // int / f64 words, and the object columns' NFGUIDs (nfk_get_props refuses those)
            std::vector<size_t> w, o;
            for (size_t k = 0; k < at.size(); k++) (pid[k] < ObjectBase() ? w : o).push_back(k);
            val.assign(at.size(), 0);
            oh.assign(at.size(), 0);
            auto gather = [&](const std::vector<size_t>& ks, bool obj) {
                if (ks.empty()) return;
                std::vector<int64_t> h(ks.size()), d(ks.size()), vh(ks.size()), vd(ks.size());
                std::vector<int32_t> p(ks.size());
                std::vector<uint64_t> v(ks.size());
                for (size_t j = 0; j < ks.size(); j++) {
                    h[j] = gh[ks[j]];
                    d[j] = gd[ks[j]];
                    p[j] = pid[ks[j]];
                }
                const int rc = obj ? nfk_get_objects(gpu_.World(), (int32_t)ks.size(), h.data(), d.data(), p.data(), vh.data(), vd.data())
                                   : nfk_get_props(gpu_.World(), (int32_t)ks.size(), h.data(), d.data(), p.data(), v.data());
                if (rc != NFK_OK) throw std::runtime_error(std::string("host mirror read: ") + nfk_last_error());
                for (size_t j = 0; j < ks.size(); j++) {
                    val[ks[j]] = obj ? (uint64_t)vd[j] : v[j];
                    oh[ks[j]] = obj ? vh[j] : 0;
                }
            };
            gather(w, false);
            gather(o, true);
        }
        ++quiet_;
        for (size_t k = 0; k < at.size(); k++) {
            const NFGUID& self = props[at[k]].first;
            const std::string& name = props[at[k]].second;
            NF_SHARE_PTR<NFIObject> ob = GetElement(self);
            NF_SHARE_PTR<NFIProperty> p = ob ? ob->GetPropertyManager()->GetElement(name) : nullptr;
            if (!p) continue;
            if (p->GetType() == TDATA_INT) {
                if (p->GetInt() != (NFINT64)val[k]) p->SetInt((NFINT64)val[k]);
            } else if (p->GetType() == TDATA_FLOAT) {
                double v;
                memcpy(&v, &val[k], 8);
                const double h = p->GetFloat();
                if (memcmp(&h, &v, 8) != 0 && !p->SetFloat(v)) {
                    // (a coalesced change within NFCProperty::SetFloat's 1e-15, PR:314: stored as is)
                    NFIDataList::TData t;
                    t.SetFloat(v);
                    p->SetValue(t);
                }
            } else if (p->GetType() == TDATA_OBJECT) {
                const NFGUID v(oh[k], (int64_t)val[k]);
                if (p->GetObject() != v) p->SetObject(v);
            }
        }
        // int record cells
        std::sort(cells.begin(), cells.end(), [](const Cell& a, const Cell& b) {
            return std::tie(a.self, a.rec, a.row, a.col) < std::tie(b.self, b.rec, b.row, b.col);
        });
        cells.erase(std::unique(cells.begin(), cells.end(), [](const Cell& a, const Cell& b) {
            return a.self == b.self && a.rec == b.rec && a.row == b.row && a.col == b.col;
        }), cells.end());
        std::vector<int64_t> ch, cd;
        std::vector<int32_t> cr, crow, ccol;
        std::vector<const Cell*> live;
        for (const Cell& c : cells) {
            if (!DevRecord(c.self, c.rec)) continue;
            live.push_back(&c);
            ch.push_back(c.self.nHead64);
            cd.push_back(c.self.nData64);
            cr.push_back(gpu_.RecordId(c.rec));
            crow.push_back(c.row);
            ccol.push_back(c.col);
        }
        if (!live.empty()) {
            std::vector<uint64_t> cv(live.size());
            if (nfk_get_records(gpu_.World(), (int32_t)live.size(), ch.data(), cd.data(), cr.data(), crow.data(),
                                ccol.data(), cv.data()) != NFK_OK)
                throw std::runtime_error(std::string("host mirror read: ") + nfk_last_error());
            for (size_t k = 0; k < live.size(); k++) {
                NF_SHARE_PTR<NFIRecord> r = NFCKernelModule::FindRecord(live[k]->self, live[k]->rec);
                if (r && r->IsUsed(live[k]->row) && r->GetInt(live[k]->row, live[k]->col) != (NFINT64)cv[k])
                    r->SetInt(live[k]->row, live[k]->col, (NFINT64)cv[k]);
            }
        }
        --quiet_;
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
    int ObjectBase() const {  // the first object property id (int, then float, then object ids)
        return gpu_.PropertyCount(nfgpu::TDATA_INT) + gpu_.PropertyCount(nfgpu::TDATA_FLOAT);
    }

    NFIClassModule* m_pClassModule = nullptr;
    std::set<std::string> dev_props_, dev_records_;
    std::map<std::string, std::map<std::string, int>> col_tags_;
    std::set<int> scenes_;
    NFGUID obj_scratch_;
    int quiet_ = 0;  // > 0: host writes are the adapter's own (mirror, SwitchScene), not forwarded
    std::vector<PROPERTY_EVENT_FUNCTOR_PTR> prop_cb_;
    std::vector<RECORD_EVENT_FUNCTOR_PTR> rec_cb_;
    std::vector<std::pair<NFGUID, std::string>> sync_props_;  // this window's written / evented pairs
    std::vector<Cell> sync_cells_;
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
        return gpu().AddSchedule(
            to_gpu(self), name,
            [cb](const nfgpu::NFGUID& g, const std::string& n, const float t, const int c) { return (*cb)(to_ref(g), n, t, c); },
            fTime, nCount);
    }
    bool RemoveSchedule(const NFGUID self) override {  // SM:240
        const bool d = gpu().RemoveSchedule(to_gpu(self));
        const bool h = host_.RemoveSchedule(self);
        return d || h;
    }
    bool RemoveSchedule(const NFGUID self, const std::string& name) override {  // SM:245
        return gpu().HasHeartBeat(name) ? gpu().RemoveSchedule(to_gpu(self), name) : host_.RemoveSchedule(self, name);
    }
    bool ExistSchedule(const NFGUID self, const std::string& name) override {  // SM:276
        return gpu().HasHeartBeat(name) ? gpu().ExistSchedule(to_gpu(self), name) : host_.ExistSchedule(self, name);
    }
    // the device frame (its object schedules) runs in NFGPUKernelAdapter::Execute; the host
    // schedules here
    bool Execute() override { return host_.Execute(); }

private:
    nfgpu::NFGPUKernelModule& gpu() {
        return dynamic_cast<NFGPUKernelAdapter*>(pPluginManager->FindModule<NFIKernelModule>())->gpu_;
    }
    NFCScheduleModule host_;
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
