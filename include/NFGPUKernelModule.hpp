// NFGPUKernelModule.hpp — C++ host plugin over the nfgpu C-ABI, with the reference's
// plugin API names for the tick path, so a NoahGameFrame game server swaps it in for
// NFCKernelModule + NFCScheduleModule + the NFCSceneAOIModule property fan-out.
//
// Reference interfaces mirrored (flyish/NoahGameFrame):
//   NFComm/NFPluginModule/NFIKernelModule.h     CreateScene, CreateObject (before or after AfterInit),
//                                               DestroyObject, SwitchScene, SetPropertyInt/Float,
//                                               GetPropertyInt/Float, RegisterCommonPropertyEvent,
//                                               Execute (NFCKernelModule.cpp:70)
//   NFComm/NFPluginModule/NFIScheduleModule.h   AddSchedule(self, name, cb, fTime, nCount),
//                                               RemoveSchedule(self[, name]), ExistSchedule
//   NFComm/NFPluginModule/NFISceneAOIModule.h   AddPropertyEventCallBack / AddRecordEventCallBack
//                                               (the recipient-list events, AOI.cpp:703-727)
//   NFComm/NFPluginModule/NFIModule.h           Init / AfterInit / Execute / BeforeShut / Shut
//   NFComm/NFPluginModule/NFIRankRedisModule.h  GetRange (leaderboard over a property)
//
// Differences a plugin author must know:
//   * A heartbeat's state change is a device effect program (nfk_op list) registered once per
//     schedule name before AfterInit (an empty list for a functor-only heartbeat); the C++
//     functor passed to AddSchedule still runs, after the device frame, with the reference's
//     arguments (self, name, fTime, nCount), objects in NFGUID order and each object's schedules
//     in name order, as NFCScheduleModule::Execute walks its maps (SM:52-80).  Its own Set,
//     SwitchScene, Create/Destroy and Add/RemoveSchedule calls take effect in the same Execute
//     (a second device pass, nfk_execute_calls; SetFunctorCallsSameFrame(false) defers them to the
//     next frame).
//   * SetProperty* calls are queued and applied at the start of the next Execute, in call order,
//     through the reference's change predicates; GetProperty* sees them at once (read-your-writes);
//     callbacks see coalesced (first old, last new) events once per frame, in (scene, group,
//     guid, property) order.
//   * Time comes from SetTimeSource (default: NFGetTime(), system clock milliseconds,
//     NFPlatform.h:367), read by AddSchedule and Execute like the reference.
//   * Limits: 64 int + 64 float + 32 object frame properties (128 in all), 15 classes, 32 schedule names, 8 records of at
//     most 64 rows x 16 columns, 4 ops per heartbeat program, 12 properties written by programs,
//     16383 players per scene group (nfgpu.h).
//   * String / Vector properties stay host-side (not on the frame path); object (NFGUID) properties
//     are device columns like the int / float ones.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "nfgpu.h"
#include "nfgpu_guidmap.hpp"
#include "NFGPUSceneShard.hpp"

namespace nfgpu_detail {
// property / record name -> index for the per-call API: open addressing on an FNV-1a hash of the
// name's bytes, the table at most a quarter full (a lookup is one hash and, mostly, one compare;
// std::unordered_map<std::string> cost ~25 ns per SetProperty call, profiles/r10e_*)
class NameIndex {
public:
    void insert(const std::string& k, int v) {
        if ((n_ + 1) * 4 > t_.size()) grow();
        put(k, v);
    }
    int find(const std::string& k) const {
        if (t_.empty()) return -1;
        for (size_t i = hash(k.data(), k.size()) & mask_;; i = (i + 1) & mask_) {
            const E& e = t_[i];
            if (e.v < 0) return -1;
            if (e.k.size() == k.size() && std::memcmp(e.k.data(), k.data(), k.size()) == 0) return e.v;
        }
    }

private:
    struct E {
        std::string k;
        int v = -1;
    };
    static uint64_t hash(const char* p, size_t n) {
        uint64_t h = 0xcbf29ce484222325ull;
        for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
        return h ^ (h >> 29);
    }
    void put(const std::string& k, int v) {
        for (size_t i = hash(k.data(), k.size()) & mask_;; i = (i + 1) & mask_) {
            E& e = t_[i];
            if (e.v < 0) {
                e.k = k;
                e.v = v;
                n_++;
                return;
            }
            if (e.k == k) {
                e.v = v;
                return;
            }
        }
    }
    void grow() {
        std::vector<E> old;
        old.swap(t_);
        t_.assign(std::max<size_t>(16, old.size() * 2), E{});
        mask_ = t_.size() - 1;
        n_ = 0;
        for (E& e : old)
            if (e.v >= 0) put(e.k, e.v);
    }
    std::vector<E> t_;
    size_t mask_ = 0, n_ = 0;
};
// A few persistent worker threads for data-parallel host loops that run no game code (gathers of
// scattered reads into dense arrays): Run(n, fn) calls fn(0) .. fn(n-1) on the workers and the
// calling thread and returns when every call has returned; Start(n, fn) hands the calls to the
// workers alone and returns at once (claimed in index order), Wait(job) returns when every call has
// returned (the calling thread takes what is left).
class WorkerPool {
public:
    // one job's calls: a worker holding a finished job finds no index left and never calls fn
    struct Job {
        std::function<void(int64_t)> own;  // (Start: the job keeps its function)
        const std::function<void(int64_t)>* fn = nullptr;
        int64_t n = 0;
        std::atomic<int64_t> next{0}, done{0};
    };
    explicit WorkerPool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this] { Loop(); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int Workers() const { return (int)th_.size(); }
    void Run(int64_t n, const std::function<void(int64_t)>& fn) {
        if (n <= 0) return;
        auto job = std::make_shared<Job>();
        job->fn = &fn;
        job->n = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = job;
        }
        cv_.notify_all();
        Wait(job);
    }
    std::shared_ptr<Job> Start(int64_t n, std::function<void(int64_t)> fn) {
        auto job = std::make_shared<Job>();
        job->own = std::move(fn);
        job->fn = &job->own;
        job->n = std::max<int64_t>(n, 0);
        if (n > 0) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                job_ = job;
            }
            cv_.notify_all();
        }
        return job;
    }
    void Wait(const std::shared_ptr<Job>& job) {
        if (!job) return;
        Work(*job);
        while (job->done.load(std::memory_order_acquire) < job->n) std::this_thread::yield();
        std::lock_guard<std::mutex> lk(mu_);
        if (job_ == job) job_.reset();
    }

private:
    static void Work(Job& j) {
        int64_t i;
        while ((i = j.next.fetch_add(1, std::memory_order_relaxed)) < j.n) {
            (*j.fn)(i);
            j.done.fetch_add(1, std::memory_order_release);
        }
    }
    void Loop() {
        std::shared_ptr<Job> last;
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (job_ && job_ != last); });
                if (stop_) return;
                j = last = job_;
            }
            Work(*j);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::shared_ptr<Job> job_;
    bool stop_ = false;
};
}  // namespace nfgpu_detail

namespace nfgpu {

struct NFGUID {
    int64_t nData64 = 0;
    int64_t nHead64 = 0;
    NFGUID() = default;
    NFGUID(int64_t head, int64_t data) : nData64(data), nHead64(head) {}
    bool IsNull() const { return nData64 == 0 && nHead64 == 0; }
    bool operator==(const NFGUID& o) const { return nData64 == o.nData64 && nHead64 == o.nHead64; }
    bool operator!=(const NFGUID& o) const { return !(*this == o); }
    bool operator<(const NFGUID& o) const {  // NFGUID.h:83
        return nHead64 == o.nHead64 ? nData64 < o.nData64 : nHead64 < o.nHead64;
    }
};

enum TDATA_TYPE { TDATA_UNKNOWN, TDATA_INT, TDATA_FLOAT, TDATA_STRING, TDATA_OBJECT };

struct TData {
    TDATA_TYPE type = TDATA_UNKNOWN;
    int64_t i = 0;
    double f = 0.0;
    NFGUID o;
    TDATA_TYPE GetType() const { return type; }
    int64_t GetInt() const { return type == TDATA_INT ? i : 0; }
    double GetFloat() const { return type == TDATA_FLOAT ? f : 0.0; }
    NFGUID GetObject() const { return type == TDATA_OBJECT ? o : NFGUID(); }
};

struct RECORD_EVENT_DATA {
    enum RecordOptype { Add = 0, Del, Swap, Create, Update, Cleared, Sort, Cover, UNKNOW };
    RecordOptype nOpType = Update;
    int nRow = 0, nCol = 0;
    std::string strRecordName;
};

using PROPERTY_EVENT_FUNCTOR = std::function<int(const NFGUID&, const std::string&, const TData&, const TData&)>;
using RECORD_EVENT_FUNCTOR =
    std::function<int(const NFGUID&, const RECORD_EVENT_DATA&, const TData&, const TData&)>;
using OBJECT_SCHEDULE_FUNCTOR = std::function<int(const NFGUID&, const std::string&, const float, const int)>;
using MODULE_SCHEDULE_FUNCTOR = std::function<int(const std::string&, const float, const int)>;
using PROPERTY_SINGLE_EVENT_FUNCTOR = std::function<int(const NFGUID&, const std::string&, const TData&,
                                                        const TData&, const std::vector<NFGUID>&)>;
using RECORD_SINGLE_EVENT_FUNCTOR = std::function<int(const NFGUID&, const std::string&, const RECORD_EVENT_DATA&,
                                                      const TData&, const TData&, const std::vector<NFGUID>&)>;

// Module schedules of NFIScheduleModule (no object: AddSchedule(name, cb, fTime, nCount),
// RemoveSchedule(name), ExistSchedule(name)), restating NFCScheduleModule (SM:123-176 Execute,
// SM:184-216 calls) on the host: they are not entity state, so they stay off the device.
class ModuleScheduler {
public:
    struct Element {  // NFCScheduleElement of a module schedule
        std::string name;
        float interval = 0.f;
        int64_t next = 0, start = 0;
        int remain = 0, all = 0;
        bool forever = false;
        MODULE_SCHEDULE_FUNCTOR cb;
    };
    bool AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR& cb, float fTime, int nCount,
                     int64_t now) {
        Element e;
        e.name = name;
        e.interval = fTime;
        e.next = now + (int64_t)(fTime * 1000);
        e.start = now;
        e.remain = e.all = nCount;
        e.forever = nCount < 0;
        e.cb = cb;
        add_.push_back(e);  // mModuleAddList
        return true;
    }
    bool RemoveSchedule(const std::string& name) {
        remove_.push_back(name);  // mModuleRemoveList
        return true;
    }
    bool ExistSchedule(const std::string& name) const { return map_.count(name) != 0; }
    // the module part of NFCScheduleModule::Execute: fire (name order), remove list, add list (an
    // add replaces a schedule of the same name)
    void Execute(const std::function<int64_t()>& now) {
        for (auto& kv : map_) {
            Element& e = kv.second;
            if (!(now() > e.next) || !(e.remain > 0 || e.forever)) continue;
            e.remain--;
            if (e.cb) e.cb(e.name, e.interval, e.remain);
            if (e.remain <= 0 && !e.forever)
                remove_.push_back(e.name);
            else
                e.next = e.start + (int64_t)(e.interval * 1000) * (int64_t)(e.all - e.remain);
        }
        for (const auto& nm : remove_) map_.erase(nm);
        remove_.clear();
        for (auto& e : add_) map_[e.name] = e;
        add_.clear();
    }

private:
    std::map<std::string, Element> map_;  // mModuleScheduleMap (name order)
    std::vector<Element> add_;
    std::vector<std::string> remove_;
};

class NFGPUKernelModule {
public:
    struct PropertyDef { std::string name; TDATA_TYPE type; };
    struct ClassDef {
        std::string name;
        std::map<std::string, uint8_t> prop_flags;   // NFK_PUBLIC | NFK_PRIVATE | NFK_UPLOAD
        std::map<std::string, uint8_t> record_flags;
    };
    struct RecordDef { std::string name; int rows; std::vector<TDATA_TYPE> cols; };
    struct HeartBeatDef {
        std::string name;
        std::vector<nfk_op> ops;
        std::vector<std::string> props, records;  // symbolic operands (empty: ids)
        bool symbolic = false;
    };

    // ---- schema (what NFIClassModule loads from Struct/Class/*.xml) ----
    explicit NFGPUKernelModule(int capacity, void* hip_stream = nullptr);
    ~NFGPUKernelModule();
    int AddProperty(const std::string& name, TDATA_TYPE type);  // TDATA_INT / FLOAT / OBJECT; returns its index
    int AddClass(const std::string& name);
    void SetPropertyFlags(const std::string& cls, const std::string& prop, bool pub, bool priv, bool upload);
    int AddRecord(const std::string& name, int rows, const std::vector<TDATA_TYPE>& cols);
    void SetRecordFlags(const std::string& cls, const std::string& rec, bool pub, bool priv, bool upload);
    // the device-side effect of a heartbeat name (see nfgpu.h op list): operands as device
    // property ids (PropertyId) and record ids
    void AddHeartBeatProgram(const std::string& name, const std::vector<nfk_op>& ops);
    // the same with operands by NAME, for a module that registers its programs before the schema
    // exists (before AfterInit, e.g. the reference-side adapter, whose schema comes from the class
    // module): a property operand (dst of a property op, a / lo / hi under NFK_A_PROP / NFK_LO_PROP /
    // NFK_HI_PROP, FLERP's a, the guard's property under NFK_GUARD and, with NFK_GUARD_PROP, the
    // property it is compared to in guard >> 19) is an index into props, a record
    // op's dst is index << 8 | column with the index into records; resolved at AfterInit (a
    // guard's constant, NFK_GUARD_K, is kept as it is)
    void AddHeartBeatProgram(const std::string& name, const std::vector<nfk_op>& ops,
                             const std::vector<std::string>& props, const std::vector<std::string>& records = {});
    int PropertyId(const std::string& name) const;
    // whether a schedule name has a device program (AddHeartBeatProgram, before or after AfterInit)
    bool HasHeartBeat(const std::string& name) const;
    // whether a heartbeat program writes property pid / record rec's column col (after AfterInit)
    bool ProgramWrites(int pid) const { return pid >= 0 && (size_t)pid < prog_props_.size() && prog_props_[(size_t)pid]; }
    bool ProgramWritesRecord(int rec, int col) const { return prog_cells_.count((rec << 8) | col) != 0; }
    bool ProgramWritesRecord(int rec) const { return prog_recs_.count(rec) != 0; }
    // properties of one type (device ids: int [0, n_int), float [n_int, n_int + n_flt), object after)
    int PropertyCount(TDATA_TYPE type) const;
    int RecordId(const std::string& name) const { return record_id_.at(name); }

    // ---- NFIModule lifecycle ----
    bool Init();
    bool AfterInit();  // commits the layout (objects created before AfterInit)
    bool Execute();    // one frame at the time source's now
    bool BeforeShut();
    bool Shut();
    // the clock AddSchedule and Execute read (NFGetTime() by default)
    void SetTimeSource(std::function<int64_t()> now_ms);
    // Calls that heartbeat functors make during Execute (Set*, SwitchScene, Create/Destroy,
    // Add/RemoveSchedule) take effect within the same Execute, as in NFCScheduleModule::Execute
    // (SM:65, SM:83-119): after the functors run, a second device pass applies them and their
    // events are delivered before Execute returns (nfk_execute_calls).  Off: they land in the
    // next frame.  Default on.
    void SetFunctorCallsSameFrame(bool on) { same_frame_ = on; }
    int64_t Now() const { return clock_(); }

    // ---- NFIKernelModule ----
    bool CreateScene(int nSceneID);
    bool CreateObject(const NFGUID& self, int nSceneID, int nGroupID, const std::string& strClassName,
                      const std::map<std::string, TData>& init = {});
    // Before AfterInit: an object's creation-time record contents (the rows game logic filled before
    // the layout, cells [cols][rows] as int64 / f64 bit patterns, the used-row mask); they are the
    // record's state at frame 0, not events.  After AfterInit use AddRow.
    bool SetCreationRecord(const NFGUID& self, const std::string& strRecordName, uint64_t used,
                           const std::vector<uint64_t>& cells);
    bool SetPropertyInt(const NFGUID& self, const std::string& name, int64_t v);
    bool SetPropertyFloat(const NFGUID& self, const std::string& name, double v);
    int64_t GetPropertyInt(const NFGUID& self, const std::string& name);
    double GetPropertyFloat(const NFGUID& self, const std::string& name);
    // NFIKernelModule::SetPropertyObject / GetPropertyObject (KM:362 / KM:440): an NFGUID column on
    // the device (16 bytes per entity), queued and read like the int / float properties
    bool SetPropertyObject(const NFGUID& self, const std::string& name, const NFGUID& v);
    NFGUID GetPropertyObject(const NFGUID& self, const std::string& name);
    // NFIKernelModule::SetRecordInt / SetRecordFloat (NFIKernelModule.h:120-121): queued like the
    // property setters and applied at the next Execute through NFCRecord::SetInt / SetFloat.  False
    // for a row the record does not use (RC:194: its used-row mask as the reference holds it now,
    // nfk_get_used_rows, one device read per (object, record) per frame); true once queued otherwise
    // (the reference also returns false for a value the cell already holds: such a call changes
    // nothing and raises no event)
    bool SetRecordInt(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol, int64_t nValue);
    bool SetRecordFloat(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol, double dwValue);
    // Record rows (NFCRecord::AddRow / Remove / IsUsed, NFIKernelModule::ClearRecord; RC:111, 1086,
    // 1209, KM:492), queued in call order with the SetRecord calls; Add / Del / Cover record events
    // are delivered with the frame.  AddRow returns the row it takes (-1 = the first unused row; no
    // unused row or a row outside the record: -1), values per column (none: the initial 0s).
    int AddRow(const NFGUID& self, const std::string& strRecordName, int nRow, const std::vector<TData>& values = {});
    bool RemoveRow(const NFGUID& self, const std::string& strRecordName, int nRow);
    bool ClearRecord(const NFGUID& self, const std::string& strRecordName);
    bool IsUsed(const NFGUID& self, const std::string& strRecordName, int nRow);
    // NFIKernelModule::GetRecordInt / GetRecordFloat (NFIKernelModule.h:134-135): read-your-writes
    // like GetProperty*; 0 for an unused row (NFCRecord::GetInt, RC:623)
    int64_t GetRecordInt(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol);
    double GetRecordFloat(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol);
    // NFCKernelModule::SwitchScene (KM:901-951); writes SceneID/GroupID/X/Y/Z when the schema has
    // them; like the reference, fOrient and arg are not used
    bool SwitchScene(const NFGUID& self, int nTargetSceneID, int nTargetGroupID, float fX, float fY, float fZ,
                     float fOrient = 0.0f, const std::vector<TData>& arg = {});
    // NFCKernelModule::DestroyObject (KM:273-308): leaves its group, its schedules go with it
    bool DestroyObject(const NFGUID& self);
    bool RegisterCommonPropertyEvent(const PROPERTY_EVENT_FUNCTOR& cb);
    bool RegisterCommonRecordEvent(const RECORD_EVENT_FUNCTOR& cb);

    // ---- NFIScheduleModule: object schedules (SM:218-285) ----
    bool AddSchedule(const NFGUID& self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb, float fTime,
                     int nCount);
    // the same call made at time now_ms (NFGetTime() of the original call, for a caller that queued it)
    bool AddSchedule(const NFGUID& self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb, float fTime,
                     int nCount, int64_t now_ms);
    bool RemoveSchedule(const NFGUID& self, const std::string& name);
    bool RemoveSchedule(const NFGUID& self);
    bool ExistSchedule(const NFGUID& self, const std::string& name);
    // ---- NFIScheduleModule: module schedules (SM:123-216; host-side, not entity state) ----
    bool AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR& cb, float fTime, int nCount);
    bool RemoveSchedule(const std::string& name);
    bool ExistSchedule(const std::string& name);

    // ---- scene shards (include/NFGPUSceneShard.hpp): one process per GPU, a scene range each ----
    // With a shard attached, SwitchScene into a scene another shard owns queues the entity's
    // departure.  Execute ends by starting the all-gather of the departures' tickets
    // (SceneShard::EndFrame, on an exchange frame; off the world's stream) and the next Execute begins
    // by moving their rows (SceneShard::BeginFrame, collective: every rank's Execute makes it; no
    // collective when no rank has a departure): the entity leaves at the start of the frame after the
    // one its SwitchScene was queued before, with its state after that frame, and enters the owner's
    // world with the SwitchScene property writes.  Until its row leaves it is this module's: its
    // heartbeats fire here with their functors and calls on it apply here (they travel with the row: a
    // window with calls while an entity is departing applies them in a device pass of its own, their
    // events delivered, before the rows leave); another SwitchScene or a DestroyObject of it returns
    // false (Departing).  Arrivals' schedules call
    // the functor registered for their name with SetKindFunctor (functors cannot cross processes).
    void AttachShard(SceneShard* shard) { shard_ = shard; }
    // the departures queued so far leave now and the arrivals enter (synchronous; collective: every
    // rank calls it the same number of times), so calls made after it in the window find the
    // arrivals here
    void MigrateNow() {
        if (shard_) MigrateShard(true);
    }
    void SetKindFunctor(const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb, float fTime);
    int64_t MigratedOut() const { return shard_ ? shard_->migrated_out : 0; }
    // a cross-shard SwitchScene of it is queued and its row has not left yet
    bool Departing(const NFGUID& g) const { return departing_.count(g.nHead64, g.nData64) != 0; }
    int64_t MigratedIn() const { return shard_ ? shard_->migrated_in : 0; }

    // ---- NFIRankRedisModule::GetRange(type, 0, k - 1, memberScoreVec) over a property: this world's
    // entities, or with a shard attached every shard's (collective then: SceneShard::RankTop) ----
    bool GetRange(const std::string& prop, int k, std::vector<std::pair<std::string, double>>& memberScoreVec);

    // ---- NFISceneAOIModule recipient-list events ----
    bool AddPropertyEventCallBack(const PROPERTY_SINGLE_EVENT_FUNCTOR& cb);
    bool AddRecordEventCallBack(const RECORD_SINGLE_EVENT_FUNCTOR& cb);

    // ---- per-Set chains (nfk_watch_props).  The reference fires a property's per-object callbacks
    // once per accepted Set (NFCProperty::SetInt / SetFloat, PR:254-334); the frame's events are
    // coalesced per (entity, property).  For the watched properties every Execute also reads the log
    // of the Sets the frame's heartbeat programs made, ordered as NFCScheduleModule::Execute runs the
    // functors: objects in NFGUID order, each object's schedules in name (kind id) order, each
    // program's ops in order (SM:52-80).  LastChain() holds it from the frame hook on. ----
    struct ChainEntry {
        int32_t obj, kind, op, pid;  // object index, heartbeat kind, op index in its program, device property id
        uint64_t old_bits, new_bits;
    };
    void WatchProperty(const std::string& name);  // int / float properties; before or after AfterInit
    const std::vector<ChainEntry>& LastChain() const { return chain_; }
    // Walk-order reads.  NFCScheduleModule::Execute runs each object's functors in turn (SM:52-80), so a
    // functor's GetPropertyInt(other, p) sees the Sets of the functors before it in the walk and none
    // after.  Here the device programs (the functors' Sets) all run before the host functors, so by
    // default such a read sees every object's programs of the frame.  On: every property
    // a program writes is logged per Set (nfk_watch_props: k_chain runs every frame), and during the
    // functor walk GetPropertyInt / GetPropertyFloat of a program-written property answer from the log
    // as of the running functor's place — an object later in NFGUID order (or a later schedule name of
    // the running object) before its programs' Sets — unless a functor of this walk set that property
    // itself (its queued Set is read, as always).  Before or after AfterInit.
    void SetWalkOrderReads(bool on);
    bool WalkOrderReads() const { return walk_reads_; }
    bool InFunctorWalk() const { return in_walk_; }
    // called by Execute once the device frame's outputs are read back, before the heartbeat functors
    // run: the frame's events (fh) and its chain are final (a reference-side adapter brings its host
    // objects up to date here, so the functors and their callbacks see the frame's values)
    void SetFrameHook(std::function<void(const nfk_frame_host&)> hook) { frame_hook_ = std::move(hook); }
    // One call per event of every device pass, after the common callbacks: the object index, the
    // event's recipient run (GetBroadCastObject, AOI:531-593) as NFGUIDs — empty for an event with
    // none — and whether that run equals the last non-empty one passed, so a caller keeps what it
    // built from it.  A reference-side adapter dispatches the reference's common and AOI callbacks
    // from here in its own registration order.
    struct SyncArgs {
        int32_t obj;
        const std::vector<NFGUID>* rcpt;
        bool same;
    };
    using PROPERTY_SYNC_FUNCTOR = std::function<void(const NFGUID&, int /*device pid*/, const TData&, const TData&, const SyncArgs&)>;
    using RECORD_SYNC_FUNCTOR = std::function<void(const NFGUID&, const RECORD_EVENT_DATA&, const TData&, const TData&, const SyncArgs&)>;
    bool AddPropertySyncCallBack(const PROPERTY_SYNC_FUNCTOR& cb);
    bool AddRecordSyncCallBack(const RECORD_SYNC_FUNCTOR& cb);
    // object and schema accessors (object index = creation order in this module)
    const NFGUID& ObjectGuid(int o) const { return guids_[(size_t)o]; }
    int ObjectGroup(int o) const { return group_[(size_t)o]; }
    int ObjectCount() const { return (int)guids_.size(); }
    const std::string& PropertyName(int dev_pid) const { return props_[(size_t)def_of_pid_[(size_t)dev_pid]].name; }
    TDATA_TYPE PropertyType(int dev_pid) const { return props_[(size_t)def_of_pid_[(size_t)dev_pid]].type; }
    const std::string& RecordName(int rec) const { return records_[(size_t)rec].name; }
    int RecordCount() const { return (int)records_.size(); }
    int HeartBeatCount() const { return (int)heartbeats_.size(); }
    // kind k's program with device operand ids (after AfterInit)
    const std::vector<nfk_op>& HeartBeatOps(int k) const { return heartbeats_[(size_t)k].ops; }

    // ---- frame batch consumers: one call per device pass instead of one per event ----
    // The pass's outputs as arrays (nfk_read_frame's nfk_frame_host: the fired list, property and
    // record events, the recipient CSR, all in object-index terms; objects[i] is object i's
    // NFGUID), called after the per-event callbacks of the same pass.  `what` = the NFK_READ_* bits
    // the consumer needs (fired in NFGUID order only with NFK_READ_FIRED_GUID_ORDER).  A network
    // layer that packs the dirty-sync messages itself reads them this way: the per-event std::function
    // calls of the reference's callback API then cost nothing.  The arrays are valid during the call.
    using FRAME_FUNCTOR = std::function<void(const nfk_frame_host&, const NFGUID* objects)>;
    bool AddFrameCallBack(const FRAME_FUNCTOR& cb, uint32_t what);

    // the world (nfk C-ABI); Flush() first hands it the buffered SetProperty calls
    void* World() const { return world_; }
    void Flush();
    const nfk_summary& LastSummary() const { return summary_; }
    // host wall time of the last Execute by phase (ms): the device frame (nfk_execute and the wait
    // for its counters), the heartbeat functors (fired list read + order + calls), the event lists
    // (read back), their delivery to the callbacks, the functors' own calls (second device pass
    // and its delivery) and module schedules
    struct FrameStats {
        double device, functors, events_read, deliver, calls, total;
        double gather;  // (of functors: the worker pool's gather of the frame's scattered reads)
        double mirror;  // the frame hook (the drop-in adapter's mirror and per-Set callbacks)
    };
    const FrameStats& LastFrameStats() const { return stats_; }
    int ObjectIndex(const NFGUID& g) const;

private:
    void check(int rc, const char* what) const;
    void DeliverEvents(const nfk_frame_host& f, const NFGUID* ev_self = nullptr, const NFGUID* re_self = nullptr,
                       const uint8_t* ev_same = nullptr);
    uint64_t UsedRows(const NFGUID& self, int rec);
    void TakeAddedSchedules();
    bool same_frame_ = true;
    int64_t pending_calls_ = 0;  // calls queued since the last device pass
    void* world_ = nullptr;
    int capacity_;
    void* stream_;
    bool committed_ = false;
    std::vector<PropertyDef> props_;
    std::unordered_map<std::string, int> prop_id_;
    nfgpu_detail::NameIndex prop_ix_;  // prop_id_ for the per-call API
    // SetPropertyInt / Float calls buffered on the host in call order (property checked, object
    // not yet: no NFGUID lookup per call) and handed to the world in one nfk_set_props before
    // anything that must see them (Flush); the world looks a large batch up on the device
    std::vector<int64_t> qs_h_, qs_d_;
    std::vector<int32_t> qs_pid_;
    std::vector<uint64_t> qs_bits_;
    std::vector<int> dev_pid_;  // props_ index -> device property id (AfterInit)
    std::vector<ClassDef> classes_;
    std::map<std::string, int> class_id_;
    std::vector<RecordDef> records_;
    std::unordered_map<std::string, int> record_id_;
    std::vector<HeartBeatDef> heartbeats_;
    std::vector<bool> prog_props_;         // property ids a heartbeat program writes (AfterInit)
    std::set<int> prog_cells_, prog_recs_;  // record rec << 8 | column, and records, a program writes
    std::unordered_map<std::string, int> hb_id_;
    std::map<int, bool> scenes_;
    // objects
    template <class T>
    using HVec = std::vector<T, nfgpu_detail::HugeAlloc<T>>;  // (tables read at random: huge pages)
    HVec<NFGUID> guids_;
    nfgpu_detail::GuidMap obj_of_;  // NFGUID -> object index (open addressing)
    std::vector<int32_t> scene_, group_;
    std::vector<uint8_t> cls_, isplayer_;
    std::vector<std::vector<uint64_t>> init_;
    std::map<std::pair<int, int>, std::pair<uint64_t, std::vector<uint64_t>>> rec_init_;  // (object, record)
    // callbacks
    std::vector<PROPERTY_EVENT_FUNCTOR> common_prop_cb_;
    std::vector<RECORD_EVENT_FUNCTOR> common_rec_cb_;
    std::vector<PROPERTY_SINGLE_EVENT_FUNCTOR> aoi_prop_cb_;
    std::vector<RECORD_SINGLE_EVENT_FUNCTOR> aoi_rec_cb_;
    std::vector<FRAME_FUNCTOR> frame_cb_;
    std::vector<PROPERTY_SYNC_FUNCTOR> sync_prop_cb_;
    std::vector<RECORD_SYNC_FUNCTOR> sync_rec_cb_;
    std::function<void(const nfk_frame_host&)> frame_hook_;
    std::vector<std::string> watch_names_;  // WatchProperty before AfterInit
    std::vector<int32_t> watch_pids_;
    std::vector<ChainEntry> chain_;
    void ReadChain();
    uint32_t frame_what_ = 0;  // union of the frame consumers' NFK_READ_* bits
    uint32_t ReadMask(bool per_event_fired) const;
    // the functor of each (object, kind) schedule: cb_slot_[object * n_kind + kind] indexes
    // cb_pool_ / cb_time_ (-1: none); freed entries are reused
    HVec<int32_t> cb_slot_;
    HVec<OBJECT_SCHEDULE_FUNCTOR> cb_pool_;
    HVec<float> cb_time_;
    std::vector<int32_t> cb_free_;
    int64_t n_cb_ = 0;
    void SetFunctor(int o, int k, const OBJECT_SCHEDULE_FUNCTOR& f, float t);
    void DropFunctors(int o);
    std::vector<int> def_of_pid_;  // device property id -> props_ index
    // pending functors of AddSchedule calls in this window ((NFGUID, kind), first call wins)
    struct PendingAdd {
        int64_t h, d;
        int32_t kind;
        OBJECT_SCHEDULE_FUNCTOR cb;
        float t;
    };
    std::vector<PendingAdd> sched_add_;  // in call order; the first call of a key wins
    struct AddKey {  // (NFGUID, kind, call index) of a pending add
        int64_t h, d;
        int32_t kind, i;
        bool operator<(const AddKey& o) const {
            return h != o.h ? h < o.h : d != o.d ? d < o.d : kind != o.kind ? kind < o.kind : i < o.i;
        }
    };
    // (TakeAddedSchedules' buffers, kept: a fresh large allocation per frame costs page faults)
    std::vector<AddKey> ta_key_;
    std::vector<int64_t> ta_h_, ta_d_;
    std::vector<int32_t> ta_k_, ta_ord_;
    // schedule calls buffered like the Sets, by NFGUID (nfk_schedule_calls in Flush)
    std::vector<int32_t> qh_op_, qh_kind_, qh_cnt_;
    std::vector<int64_t> qh_h_, qh_d_;
    std::vector<float> qh_t_;
    std::vector<int64_t> qh_now_;
    nfgpu_detail::NameIndex hb_ix_;  // schedule name -> kind (AfterInit)
    void QueueScheduleCall(int32_t op, const NFGUID& self, int32_t kind, float t, int32_t cnt, int64_t now);
    void DropPendingAdds(const NFGUID& g);
    // objects with a queued cross-shard departure whose rows have not left the world yet (still this
    // module's: see AttachShard)
    nfgpu_detail::GuidMap departing_;
    int FlushSets();
    int FlushScheduleCalls();
    // the functor walk's and the deliveries' scattered host reads (functor slot, NFGUID, interval
    // per fired schedule; NFGUID per event) gathered into dense arrays by worker threads
    // (NFGPU_PLUGIN_THREADS workers, default 8), so the calls themselves stream.  The gather runs
    // beside the walk: the fired list in chunks ahead of it (fg_ready_), the events while it
    // runs.  The workers read guids_, cb_slot_ and cb_time_: every write to those waits for the
    // gather first (WaitGather), so a functor that creates objects or drops schedules sees no race.
    std::unique_ptr<nfgpu_detail::WorkerPool> pool_;
    std::shared_ptr<nfgpu_detail::WorkerPool::Job> gather_job_;
    std::unique_ptr<std::atomic<uint8_t>[]> fg_ready_;  // [fired chunk] gathered
    size_t fg_ready_cap_ = 0;
    HVec<int32_t> fg_c_;
    HVec<NFGUID> fg_g_, ev_self_, re_self_;
    HVec<float> fg_t_;
    HVec<uint8_t> ev_same_;
    bool in_walk_ = false;  // (freed functor entries are not reused while the fired list is walked)
    // walk-order reads (SetWalkOrderReads): the running functor's (object, kind), the log's range of
    // each object (built on the walk's first such read), the (object, property) a functor of the walk set
    bool walk_reads_ = false;
    int32_t walk_o_ = -1, walk_k_ = -1;
    bool walk_ix_built_ = false;
    std::unordered_map<int32_t, std::pair<uint32_t, uint32_t>> walk_ix_;
    std::unordered_map<uint64_t, uint8_t> walk_set_;
    void WatchProgramProperties();
    bool WalkRead(const NFGUID& self, int32_t pid, uint64_t* bits);
    void WalkWrote(const NFGUID& self, int32_t pid);
    static constexpr int64_t kGatherChunk = 1 << 14;
    bool GatherFrame(const nfk_frame_host& fh, int64_t nfi);
    void WaitGather();
    ModuleScheduler module_sched_;
    SceneShard* shard_ = nullptr;
    std::map<std::string, std::pair<OBJECT_SCHEDULE_FUNCTOR, float>> kind_cb_;  // arrivals' functors
    void MigrateShard(bool sync);
    void CallsPass();
    // (with a shard) the objects the calls since the last device pass named, and whether one of those
    // calls named an entity in transit (NoteCall, Depart)
    std::unordered_set<uint64_t> touched_;
    bool transit_calls_ = false;
    static uint64_t TouchKey(const NFGUID& g) { return (uint64_t)g.nData64 * 0x9E3779B97F4A7C15ull ^ (uint64_t)g.nHead64; }
    void NoteCall(const NFGUID& self);
    // cross-shard SwitchScene of an entity whose membership changed in this window (spawned, or
    // switched within the shard): deferred until the frame has applied that change (an export of
    // it would be refused, and every rank would fail the exchange)
    struct DeferredSwitch {
        NFGUID self;
        int scene, group;
        float x, y, z;
    };
    std::vector<DeferredSwitch> deferred_;
    std::vector<uint8_t> moved_flag_;  // [object] membership changed in this window (with a shard)
    std::vector<int> moved_;
    void MarkMoved(int o);
    void DropDeferred(const NFGUID& self);
    void Depart(int o, const NFGUID& self, int scene, int group, float x, float y, float z);
    void WindowApplied();
    std::function<int64_t()> clock_;
    nfk_summary summary_{};
    FrameStats stats_{};
};

}  // namespace nfgpu
