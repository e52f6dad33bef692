// NFGPUKernelModule.cpp — host plugin over the C-ABI (see include/NFGPUKernelModule.hpp).
#include "NFGPUKernelModule.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <numeric>

namespace nfgpu {

static uint64_t bits_of(double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; }
static double dbl_of(uint64_t u) { double d; std::memcpy(&d, &u, 8); return d; }

// NFGetTime() (NFPlatform.h:367): system clock milliseconds since the epoch
static int64_t nf_get_time() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
}

NFGPUKernelModule::NFGPUKernelModule(int capacity, void* hip_stream)
    : capacity_(capacity), stream_(hip_stream), clock_(nf_get_time) {}

void NFGPUKernelModule::SetTimeSource(std::function<int64_t()> now_ms) { clock_ = now_ms ? now_ms : nf_get_time; }

NFGPUKernelModule::~NFGPUKernelModule() {
    WaitGather();
    pool_.reset();
    if (world_) nfk_destroy(world_);
}

void NFGPUKernelModule::check(int rc, const char* what) const {
    if (rc != NFK_OK) throw std::runtime_error(std::string(what) + ": " + nfk_last_error());
}

int NFGPUKernelModule::AddProperty(const std::string& name, TDATA_TYPE type) {
    if (committed_) throw std::runtime_error("AddProperty after AfterInit");
    if (type != TDATA_INT && type != TDATA_FLOAT && type != TDATA_OBJECT)
        throw std::runtime_error("frame-path properties are int, float or object");
    auto it = prop_id_.find(name);
    if (it != prop_id_.end()) return it->second;
    props_.push_back({name, type});
    prop_id_[name] = (int)props_.size() - 1;
    prop_ix_.insert(name, (int)props_.size() - 1);
    return prop_id_[name];
}

int NFGPUKernelModule::AddClass(const std::string& name) {
    auto it = class_id_.find(name);
    if (it != class_id_.end()) return it->second;
    classes_.push_back({name, {}, {}});
    class_id_[name] = (int)classes_.size() - 1;
    return class_id_[name];
}

void NFGPUKernelModule::SetPropertyFlags(const std::string& cls, const std::string& prop, bool pub, bool priv,
                                         bool upload) {
    classes_.at(class_id_.at(cls)).prop_flags[prop] =
        (pub ? NFK_PUBLIC : 0) | (priv ? NFK_PRIVATE : 0) | (upload ? NFK_UPLOAD : 0);
}

int NFGPUKernelModule::AddRecord(const std::string& name, int rows, const std::vector<TDATA_TYPE>& cols) {
    records_.push_back({name, rows, cols});
    record_id_[name] = (int)records_.size() - 1;
    return record_id_[name];
}

void NFGPUKernelModule::SetRecordFlags(const std::string& cls, const std::string& rec, bool pub, bool priv,
                                       bool upload) {
    classes_.at(class_id_.at(cls)).record_flags[rec] =
        (pub ? NFK_PUBLIC : 0) | (priv ? NFK_PRIVATE : 0) | (upload ? NFK_UPLOAD : 0);
}

void NFGPUKernelModule::AddHeartBeatProgram(const std::string& name, const std::vector<nfk_op>& ops) {
    if (committed_) throw std::runtime_error("AddHeartBeatProgram after AfterInit");
    heartbeats_.push_back({name, ops, {}, {}, false});
}

void NFGPUKernelModule::AddHeartBeatProgram(const std::string& name, const std::vector<nfk_op>& ops,
                                            const std::vector<std::string>& props,
                                            const std::vector<std::string>& records) {
    if (committed_) throw std::runtime_error("AddHeartBeatProgram after AfterInit");
    heartbeats_.push_back({name, ops, props, records, true});
}

// a symbolic program's operands as device ids (AfterInit, once the schema is complete)
static void resolve_program(std::vector<nfk_op>& ops, const std::vector<std::string>& props,
                            const std::vector<std::string>& records, const std::function<int(const std::string&)>& pid,
                            const std::function<int(const std::string&)>& rid) {
    for (nfk_op& op : ops) {
        auto P = [&](int64_t i) {
            if (i < 0 || i >= (int64_t)props.size()) throw std::runtime_error("heartbeat program: property operand out of range");
            return (int64_t)pid(props[(size_t)i]);
        };
        if (op.flags & NFK_GUARD) {
            op.guard = (op.guard & ~0xFFFFu) | (uint32_t)P(op.guard & 0xFFFF);
            if (op.guard & NFK_GUARD_PROP)  // (the compared property, guard >> 19)
                op.guard = (op.guard & 0x7FFFFu) | ((uint32_t)P(op.guard >> 19) << 19);
        }
        switch (op.code) {
            case NFK_OP_IADD_CLAMP:
                op.dst = (uint16_t)P(op.dst);
                if (op.flags & NFK_A_PROP) op.a = P(op.a);
                if (op.flags & NFK_LO_PROP) op.b = P(op.b);
                if (op.flags & NFK_HI_PROP) op.c = P(op.c);
                break;
            case NFK_OP_FLERP:
                op.dst = (uint16_t)P(op.dst);
                op.a = P(op.a);
                break;
            case NFK_OP_FAFFINE:
                op.dst = (uint16_t)P(op.dst);
                break;
            case NFK_OP_ISET:
            case NFK_OP_FSET:
                op.dst = (uint16_t)P(op.dst);
                if (op.flags & NFK_A_PROP) op.a = P(op.a);
                break;
            case NFK_OP_RIADD_CLAMP:
            case NFK_OP_RFAFFINE: {
                const size_t r = op.dst >> 8;
                if (r >= records.size()) throw std::runtime_error("heartbeat program: record operand out of range");
                op.dst = (uint16_t)((rid(records[r]) << 8) | (op.dst & 0xFF));
                break;
            }
            default:
                break;
        }
    }
}

bool NFGPUKernelModule::HasHeartBeat(const std::string& name) const {
    if (committed_) return hb_id_.count(name) != 0;
    for (const HeartBeatDef& h : heartbeats_)
        if (h.name == name) return true;
    return false;
}

int NFGPUKernelModule::PropertyCount(TDATA_TYPE type) const {
    int n = 0;
    for (const PropertyDef& p : props_) n += p.type == type;
    return n;
}

// property ids on the device: int properties first, then float ones, then object ones, each in
// definition order
int NFGPUKernelModule::PropertyId(const std::string& name) const {
    const int pid = prop_id_.at(name);
    if (committed_) return dev_pid_[(size_t)pid];
    int n[3] = {0, 0, 0}, before = 0;
    const int t = props_[pid].type == TDATA_INT ? 0 : props_[pid].type == TDATA_FLOAT ? 1 : 2;
    for (int i = 0; i < (int)props_.size(); i++) {
        const int ti = props_[i].type == TDATA_INT ? 0 : props_[i].type == TDATA_FLOAT ? 1 : 2;
        n[ti]++;
        if (ti == t && i < pid) before++;
    }
    return (t >= 1 ? n[0] : 0) + (t == 2 ? n[1] : 0) + before;
}

// a property's value as its row words (int / f64 bits: one; NFGUID: data then head)
static void put_words(std::vector<uint64_t>& row, int at, TDATA_TYPE type, const TData& v) {
    if (type == TDATA_INT) row[at] = (uint64_t)v.GetInt();
    else if (type == TDATA_FLOAT) row[at] = bits_of(v.GetFloat());
    else {
        row[at] = (uint64_t)v.GetObject().nData64;
        row[at + 1] = (uint64_t)v.GetObject().nHead64;
    }
}

bool NFGPUKernelModule::Init() { return true; }

bool NFGPUKernelModule::CreateScene(int nSceneID) {
    if (scenes_.count(nSceneID)) return false;  // NFCKernelModule::CreateScene (KM:981)
    scenes_[nSceneID] = true;
    return true;
}

bool NFGPUKernelModule::CreateObject(const NFGUID& self, int nSceneID, int nGroupID, const std::string& cls,
                                     const std::map<std::string, TData>& init) {
    Flush();  // (the buffered Set calls first: call order)
    if (!scenes_.count(nSceneID)) return false;  // "There is no scene" (KM:107)
    if (committed_) {
        // after AfterInit: the entity enters at the start of the next frame (nfk_spawn_objects)
        if (obj_of_.count(self.nHead64, self.nData64)) return false;  // "The object has Exists" (KM:131)
        auto c = class_id_.find(cls);
        if (c == class_id_.end()) return false;
        int n_if = 0;
        for (auto& p : props_) n_if += p.type != TDATA_OBJECT;
        std::vector<uint64_t> row(props_.size() * 2, 0);  // property words (nfk_spawn_objects)
        for (auto& kv : init) {
            const int p = prop_id_.at(kv.first), id = PropertyId(kv.first);
            put_words(row, id < n_if ? id : n_if + 2 * (id - n_if), props_[p].type, kv.second);
        }
        for (const char* nm : {"SceneID", "GroupID"}) {  // CreateObject sets them (KM:248-249)
            auto it = prop_id_.find(nm);
            if (it != prop_id_.end() && props_[it->second].type == TDATA_INT)
                row[PropertyId(nm)] = (uint64_t)(int64_t)(nm[0] == 'S' ? nSceneID : nGroupID);
        }
        const uint8_t cl = (uint8_t)c->second, pl = cls == "Player";
        check(nfk_spawn_objects(world_, 1, &self.nHead64, &self.nData64, &nSceneID, &nGroupID, &cl, &pl, row.data()),
              "nfk_spawn_objects");
        pending_calls_++;
        WaitGather();  // (the gather's workers read guids_)
        obj_of_.insert(self.nHead64, self.nData64, (int)guids_.size());
        guids_.push_back(self);
        scene_.push_back(nSceneID);
        group_.push_back(nGroupID);
        cls_.push_back(cl);
        isplayer_.push_back(pl);
        MarkMoved((int)guids_.size() - 1);
        return true;
    }
    if (obj_of_.count(self.nHead64, self.nData64)) return false;       // "The object has Exists" (KM:131)
    auto c = class_id_.find(cls);
    if (c == class_id_.end()) return false;
    WaitGather();  // (the gather's workers read guids_)
    int o = (int)guids_.size();
    guids_.push_back(self);
    obj_of_.insert(self.nHead64, self.nData64, o);
    scene_.push_back(nSceneID);
    group_.push_back(nGroupID);
    cls_.push_back((uint8_t)c->second);
    isplayer_.push_back(cls == "Player");  // NFCKernelModule.cpp:146
    if (init_.size() < props_.size()) init_.resize(props_.size());
    for (size_t p = 0; p < init_.size(); p++) init_[p].resize(init_[p].size() + (props_[p].type == TDATA_OBJECT ? 2 : 1), 0);
    for (auto& kv : init) {
        const int p = prop_id_.at(kv.first);
        std::vector<uint64_t>& v = init_[p];
        put_words(v, (int)v.size() - (props_[p].type == TDATA_OBJECT ? 2 : 1), props_[p].type, kv.second);
    }
    return true;
}

bool NFGPUKernelModule::SetCreationRecord(const NFGUID& self, const std::string& strRecordName, uint64_t used,
                                          const std::vector<uint64_t>& cells) {
    auto it = record_id_.find(strRecordName);
    const int o = ObjectIndex(self);
    if (committed_ || it == record_id_.end() || o < 0) return false;
    const RecordDef& rd = records_[it->second];
    if (cells.size() != (size_t)rd.rows * rd.cols.size()) return false;
    rec_init_[{o, it->second}] = {used & (rd.rows >= 64 ? ~0ull : ((1ull << rd.rows) - 1)), cells};
    return true;
}

bool NFGPUKernelModule::AfterInit() {
    int n_int = 0, n_flt = 0, n_obj = 0;
    for (auto& p : props_) (p.type == TDATA_INT ? n_int : p.type == TDATA_FLOAT ? n_flt : n_obj)++;
    nfk_config cfg{};
    cfg.capacity = std::max(capacity_, 1);
    cfg.n_int = n_int;
    cfg.n_flt = n_flt;
    cfg.n_obj = n_obj;
    cfg.n_class = (int)classes_.size();
    cfg.n_kind = (int)heartbeats_.size();
    cfg.n_rec = (int)records_.size();
    cfg.stream = stream_;
    check(nfk_create(&cfg, &world_), "nfk_create");
    const int np = n_int + n_flt + n_obj;
    for (int c = 0; c < (int)classes_.size(); c++) {
        std::vector<uint8_t> fl(np, 0);
        for (auto& kv : classes_[c].prop_flags) fl[PropertyId(kv.first)] = kv.second;
        check(nfk_set_prop_flags(world_, c, fl.data()), "nfk_set_prop_flags");
    }
    for (int r = 0; r < (int)records_.size(); r++) {
        std::vector<uint8_t> ct, fl(classes_.size(), 0);
        for (auto t : records_[r].cols) ct.push_back(t == TDATA_FLOAT ? 1 : 0);
        for (int c = 0; c < (int)classes_.size(); c++) {
            auto it = classes_[c].record_flags.find(records_[r].name);
            if (it != classes_[c].record_flags.end()) fl[c] = it->second;
        }
        check(nfk_define_record(world_, r, records_[r].rows, (int)records_[r].cols.size(), ct.data(), fl.data()),
              "nfk_define_record");
    }
    // schedule names -> kind ids in lexical order (NFMapEx<std::string, NFCScheduleElement> order)
    std::sort(heartbeats_.begin(), heartbeats_.end(),
              [](const HeartBeatDef& a, const HeartBeatDef& b) { return a.name < b.name; });
    for (int k = 0; k < (int)heartbeats_.size(); k++) {
        hb_id_[heartbeats_[k].name] = k;
        hb_ix_.insert(heartbeats_[k].name, k);
        if (heartbeats_[k].symbolic)
            resolve_program(heartbeats_[k].ops, heartbeats_[k].props, heartbeats_[k].records,
                            [this](const std::string& n) { return PropertyId(n); },
                            [this](const std::string& n) { return record_id_.at(n); });
        check(nfk_define_kind(world_, k, heartbeats_[k].ops.data(), (int)heartbeats_[k].ops.size()),
              "nfk_define_kind");
        for (const nfk_op& op : heartbeats_[k].ops) {  // (ProgramWrites)
            if (op.code == NFK_OP_RIADD_CLAMP || op.code == NFK_OP_RFAFFINE) {
                prog_cells_.insert(op.dst);
                prog_recs_.insert(op.dst >> 8);
            } else if (op.code != NFK_OP_NOP) {
                if (prog_props_.size() <= op.dst) prog_props_.resize((size_t)op.dst + 1, false);
                prog_props_[op.dst] = true;
            }
        }
    }
    const int n = (int)guids_.size();
    std::vector<int64_t> gh(n), gd(n);
    for (int i = 0; i < n; i++) {
        gh[i] = guids_[i].nHead64;
        gd[i] = guids_[i].nData64;
    }
    check(nfk_create_objects(world_, n, gh.data(), gd.data(), scene_.data(), group_.data(), cls_.data(),
                             isplayer_.data()),
          "nfk_create_objects");
    for (int p = 0; p < (int)props_.size(); p++) {
        if (p >= (int)init_.size() || init_[p].empty()) continue;
        if (props_[p].type != TDATA_OBJECT) {
            check(nfk_load_prop(world_, PropertyId(props_[p].name), init_[p].data()), "nfk_load_prop");
            continue;
        }
        std::vector<int64_t> h(n), d(n);  // init_ holds (data, head) per object
        for (int i = 0; i < n; i++) {
            d[i] = (int64_t)init_[p][2 * (size_t)i];
            h[i] = (int64_t)init_[p][2 * (size_t)i + 1];
        }
        check(nfk_load_object(world_, PropertyId(props_[p].name), h.data(), d.data()), "nfk_load_object");
    }
    for (int r = 0; r < (int)records_.size(); r++) {  // creation-time record contents
        const size_t per = (size_t)records_[r].rows * records_[r].cols.size();
        std::vector<uint64_t> cells(per * (size_t)n, 0), used((size_t)n, 0);
        bool any = false;
        for (auto& kv : rec_init_) {
            if (kv.first.second != r) continue;
            any = true;
            used[kv.first.first] = kv.second.first;
            std::copy(kv.second.second.begin(), kv.second.second.end(), cells.begin() + per * kv.first.first);
        }
        if (any) check(nfk_load_record(world_, r, cells.data(), used.data()), "nfk_load_record");
    }
    rec_init_.clear();
    check(nfk_commit(world_), "nfk_commit");
    {
        auto pid_of = [&](const char* nm, TDATA_TYPE t) {
            auto it = prop_id_.find(nm);
            return (it != prop_id_.end() && props_[it->second].type == t) ? PropertyId(nm) : -1;
        };
        check(nfk_set_scene_props(world_, pid_of("SceneID", TDATA_INT), pid_of("GroupID", TDATA_INT),
                                  pid_of("X", TDATA_FLOAT), pid_of("Y", TDATA_FLOAT), pid_of("Z", TDATA_FLOAT)),
              "nfk_set_scene_props");
    }
    def_of_pid_.assign(props_.size(), 0);
    dev_pid_.assign(props_.size(), 0);
    for (int p = 0; p < (int)props_.size(); p++) {
        dev_pid_[p] = PropertyId(props_[p].name);
        def_of_pid_[dev_pid_[p]] = p;
    }
    committed_ = true;
    for (const std::string& nm : watch_names_) WatchProperty(nm);
    watch_names_.clear();
    if (walk_reads_) WatchProgramProperties();
    return true;
}

void NFGPUKernelModule::SetWalkOrderReads(bool on) {
    walk_reads_ = on;
    if (on && committed_) WatchProgramProperties();
}

// every int / f64 property a heartbeat program writes joins the per-Set log
void NFGPUKernelModule::WatchProgramProperties() {
    bool added = false;
    for (int32_t pid = 0; pid < (int32_t)prog_props_.size(); pid++) {
        if (!prog_props_[(size_t)pid] || PropertyType(pid) == TDATA_OBJECT) continue;
        if (std::find(watch_pids_.begin(), watch_pids_.end(), pid) != watch_pids_.end()) continue;
        watch_pids_.push_back(pid);
        added = true;
    }
    if (added) check(nfk_watch_props(world_, (int32_t)watch_pids_.size(), watch_pids_.data()), "nfk_watch_props");
}

// (walk-order reads) the value of (self, pid) as of the running functor's place in the walk, from the
// frame's per-Set log: an object before it in NFGUID order has made all its Sets (the device's value),
// one after it none (its first logged Set's old value), the running object those of its schedules up
// to the running one (SM:52-80).  False: read the device (no logged Set, or a functor of this walk set
// the property: its queued Set is what the reference's read returns).
bool NFGPUKernelModule::WalkRead(const NFGUID& self, int32_t pid, uint64_t* bits) {
    if (!walk_reads_ || !in_walk_ || walk_o_ < 0 || !ProgramWrites(pid)) return false;
    const int32_t o = ObjectIndex(self);
    if (o < 0 || walk_set_.count(((uint64_t)(uint32_t)o << 8) | (uint32_t)pid)) return false;
    if (o != walk_o_ && guids_[(size_t)o] < guids_[(size_t)walk_o_]) return false;
    if (!walk_ix_built_) {
        walk_ix_.clear();
        for (uint32_t i = 0; i < (uint32_t)chain_.size(); i++) {
            auto it = walk_ix_.find(chain_[i].obj);
            if (it == walk_ix_.end()) walk_ix_.emplace(chain_[i].obj, std::make_pair(i, i + 1));
            else it->second.second = i + 1;  // (an object's entries are contiguous in the walk's order)
        }
        walk_ix_built_ = true;
    }
    auto it = walk_ix_.find(o);
    if (it == walk_ix_.end()) return false;
    const ChainEntry* first = nullptr;
    const ChainEntry* last_before = nullptr;
    for (uint32_t i = it->second.first; i < it->second.second; i++) {
        const ChainEntry& c = chain_[i];
        if (c.pid != pid) continue;
        if (!first) first = &c;
        if (o == walk_o_ && c.kind <= walk_k_) last_before = &c;
    }
    if (!first) return false;
    *bits = last_before ? last_before->new_bits : first->old_bits;
    return true;
}

void NFGPUKernelModule::WalkWrote(const NFGUID& self, int32_t pid) {
    if (!walk_reads_ || !in_walk_) return;
    const int32_t o = ObjectIndex(self);
    if (o >= 0) walk_set_[((uint64_t)(uint32_t)o << 8) | (uint32_t)pid] = 1;
}

void NFGPUKernelModule::WatchProperty(const std::string& name) {
    if (!committed_) {
        watch_names_.push_back(name);
        return;
    }
    auto it = prop_id_.find(name);
    if (it == prop_id_.end() || props_[(size_t)it->second].type == TDATA_OBJECT) return;  // (programs write int / f64)
    const int32_t pid = dev_pid_[(size_t)it->second];
    if (std::find(watch_pids_.begin(), watch_pids_.end(), pid) != watch_pids_.end()) return;
    watch_pids_.push_back(pid);
    check(nfk_watch_props(world_, (int32_t)watch_pids_.size(), watch_pids_.data()), "nfk_watch_props");
}

// the frame's per-Set log in the order the reference's heartbeat walk makes the Sets: objects in
// NFGUID order, then kind (name order), then op (SM:52-80), as nfk_read_chain hands it over
void NFGPUKernelModule::ReadChain() {
    chain_.clear();
    if (watch_pids_.empty()) return;
    int32_t n = 0;
    check(nfk_read_chain(world_, 0, &n, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr), "nfk_read_chain");
    if (!n) return;
    std::vector<int32_t> o((size_t)n), k((size_t)n), op((size_t)n), pid((size_t)n);
    std::vector<uint64_t> a((size_t)n), b((size_t)n);
    int32_t m = 0;
    check(nfk_read_chain(world_, n, &m, o.data(), k.data(), op.data(), pid.data(), a.data(), b.data()), "nfk_read_chain");
    chain_.resize((size_t)n);  // (in the walk's order already: nfk_read_chain sorts it on the device)
    for (int32_t i = 0; i < n; i++) chain_[(size_t)i] = {o[(size_t)i], k[(size_t)i], op[(size_t)i], pid[(size_t)i], a[(size_t)i], b[(size_t)i]};
}

bool NFGPUKernelModule::SwitchScene(const NFGUID& self, int nTargetSceneID, int nTargetGroupID, float fX, float fY,
                                    float fZ, float /*fOrient*/, const std::vector<TData>& /*arg*/) {
    Flush();  // (the buffered Set calls first: call order)
    if (!committed_ || ObjectIndex(self) < 0) return false;  // "There is no object" (KM:948)
    if (departing_.count(self.nHead64, self.nData64)) return false;  // (on its way to another shard)
    if (shard_ && !shard_->Owns(nTargetSceneID)) {          // into another shard's scene
        const int o = ObjectIndex(self);
        // an entity spawned or switched in this window has no row to export until the frame applies
        // that: its departure is deferred to the end of the next Execute's device frame
        if ((size_t)o < moved_flag_.size() && moved_flag_[(size_t)o]) {
            deferred_.push_back({self, nTargetSceneID, nTargetGroupID, fX, fY, fZ});
            return true;
        }
        Depart(o, self, nTargetSceneID, nTargetGroupID, fX, fY, fZ);
        return true;
    }
    if (!scenes_.count(nTargetSceneID)) return false;       // "no this container" (KM:917)
    DropDeferred(self);  // (a later switch within the shard supersedes a deferred departure)
    check(nfk_switch_scene(world_, self.nHead64, self.nData64, nTargetSceneID, nTargetGroupID, fX, fY, fZ),
          "nfk_switch_scene");
    pending_calls_++;
    const int o = ObjectIndex(self);
    scene_[o] = nTargetSceneID;
    group_[o] = nTargetGroupID;
    MarkMoved(o);
    return true;
}

// The entity stays this module's until the exchange exports its row (MigrateNow, or the next Execute's
// SceneShard::BeginFrame after the gather its Execute starts): its heartbeats fire with their functors
// on this shard until then, and calls on it apply here and travel with its row (with the
// asynchronous gather the entity ticks here one more device frame, whose functor calls were lost when
// the functors were dropped at the SwitchScene)
void NFGPUKernelModule::Depart(int o, const NFGUID& self, int scene, int group, float x, float y, float z) {
    shard_->QueueSwitch(self.nHead64, self.nData64, cls_[o], isplayer_[o], scene, group, x, y, z);
    departing_.insert(self.nHead64, self.nData64, o);
    if (touched_.count(TouchKey(self))) transit_calls_ = true;  // (calls on it earlier in this window)
}

// (with a shard) a call on self was queued: whether it is an entity in transit (its row may leave before
// the next device pass applies the call: MigrateShard applies the window's calls first)
void NFGPUKernelModule::NoteCall(const NFGUID& self) {
    if (departing_.size() && departing_.count(self.nHead64, self.nData64)) transit_calls_ = true;
    else touched_.insert(TouchKey(self));
}

void NFGPUKernelModule::DropDeferred(const NFGUID& self) {
    for (size_t i = 0; i < deferred_.size();)
        if (deferred_[i].self == self) deferred_.erase(deferred_.begin() + (std::ptrdiff_t)i);
        else i++;
}

void NFGPUKernelModule::MarkMoved(int o) {
    if (!shard_) return;
    if (moved_flag_.size() <= (size_t)o) moved_flag_.resize((size_t)o + 1 + moved_flag_.size() / 2, 0);
    if (!moved_flag_[(size_t)o]) {
        moved_flag_[(size_t)o] = 1;
        moved_.push_back(o);
    }
}

// after the device frame applied the window's membership changes: nothing has moved in the new
// window yet, and the departures deferred in the last one leave now (still objects of this module
// unless the game destroyed or departed them since)
void NFGPUKernelModule::WindowApplied() {
    for (int o : moved_) moved_flag_[(size_t)o] = 0;
    moved_.clear();
    std::vector<DeferredSwitch> dv;
    dv.swap(deferred_);
    for (const DeferredSwitch& q : dv) {
        const int o = ObjectIndex(q.self);
        if (o >= 0) Depart(o, q.self, q.scene, q.group, q.x, q.y, q.z);
    }
}

bool NFGPUKernelModule::DestroyObject(const NFGUID& self) {
    Flush();  // (the buffered Set calls first: call order)
    const int o = ObjectIndex(self);
    if (!committed_ || o < 0 || departing_.count(self.nHead64, self.nData64)) return false;
    DropDeferred(self);
    check(nfk_destroy_objects(world_, 1, &self.nHead64, &self.nData64), "nfk_destroy_objects");
    pending_calls_++;
    obj_of_.erase(self.nHead64, self.nData64);  // its object index stays reserved; later calls find no object
    DropFunctors(o);
    DropPendingAdds(self);
    return true;
}

bool NFGPUKernelModule::GetRange(const std::string& prop, int k,
                                 std::vector<std::pair<std::string, double>>& memberScoreVec) {
    Flush();  // (the buffered Set calls first: call order)
    memberScoreVec.clear();
    if (!committed_ || !prop_id_.count(prop) || k <= 0) return false;
    if (shard_) {  // every shard's entities (collective: SceneShard::RankTop)
        std::vector<SceneShard::RankRow> rows;
        check(shard_->RankTop(PropertyId(prop), k, &rows), "SceneShard::RankTop");
        for (const auto& q : rows)  // member = NFGUID::ToString() (NFGUID.h:93)
            memberScoreVec.emplace_back(std::to_string(q.guid_head) + "-" + std::to_string(q.guid_data), q.score);
        return true;
    }
    std::vector<int64_t> gh(k), gd(k);
    std::vector<double> sc(k);
    int32_t n = 0;
    check(nfk_rank_top(world_, PropertyId(prop), k, &n, gh.data(), gd.data(), sc.data()), "nfk_rank_top");
    for (int i = 0; i < n; i++)  // member = NFGUID::ToString() (NFGUID.h:93)
        memberScoreVec.emplace_back(std::to_string(gh[i]) + "-" + std::to_string(gd[i]), sc[i]);
    return true;
}

int NFGPUKernelModule::ObjectIndex(const NFGUID& g) const { return obj_of_.find(g.nHead64, g.nData64); }

// The call is checked here (the property is an int one) and buffered by NFGUID; Flush hands the
// buffer to the world in one nfk_set_props, whose NFGUID lookups of a large batch run on the
// device.  A call on an object this module does not have is dropped there (NFCKernelModule logs
// "There is no object" and returns false, KM:331; this returns true, as it does for a value the
// property already holds, where NFCProperty::SetInt returns false, PR:273).
bool NFGPUKernelModule::SetPropertyInt(const NFGUID& self, const std::string& name, int64_t v) {
    const int p = prop_ix_.find(name);
    if (!committed_ || p < 0 || props_[(size_t)p].type != TDATA_INT) return false;
    if (walk_reads_ && in_walk_) WalkWrote(self, dev_pid_[(size_t)p]);
    qs_h_.push_back(self.nHead64);
    qs_d_.push_back(self.nData64);
    qs_pid_.push_back(dev_pid_[(size_t)p]);
    qs_bits_.push_back((uint64_t)v);
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

void NFGPUKernelModule::Flush() {
    if (!qs_h_.empty()) {
        const int rc = FlushSets();
        qs_h_.clear();
        qs_d_.clear();
        qs_pid_.clear();
        qs_bits_.clear();
        check(rc, "nfk_set_props");
    }
    if (!qh_op_.empty()) {
        const int rc = FlushScheduleCalls();
        for (auto* v : {&qh_op_, &qh_kind_, &qh_cnt_}) v->clear();
        qh_h_.clear();
        qh_d_.clear();
        qh_t_.clear();
        qh_now_.clear();
        check(rc, "nfk_schedule_calls");
    }
}

// the buffered Sets: one nfk_set_props (it rejects a batch naming an object the world does not
// have, queueing none of it); then the calls on objects this module has, resolved here, by object
// index.
int NFGPUKernelModule::FlushSets() {
    const int32_t n = (int32_t)qs_h_.size();
    if (!n) return NFK_OK;
    const int rc = nfk_set_props(world_, n, qs_h_.data(), qs_d_.data(), qs_pid_.data(), qs_bits_.data());
    if (rc != NFK_ERR_NOTFOUND) return rc;
    std::vector<int32_t> obj, pid;
    std::vector<uint64_t> bits;
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = obj_of_.find(qs_h_[i], qs_d_[i]);
        if (o < 0) continue;  // "There is no object" (KM:331)
        obj.push_back(o);
        pid.push_back(qs_pid_[i]);
        bits.push_back(qs_bits_[i]);
    }
    return obj.empty() ? NFK_OK : nfk_set_props_obj(world_, (int32_t)obj.size(), obj.data(), pid.data(), bits.data());
}

// the buffered schedule calls, as FlushSets (the reference's schedule module keeps no object
// table: a call naming no object of this module changes nothing)
int NFGPUKernelModule::FlushScheduleCalls() {
    const int32_t n = (int32_t)qh_op_.size();
    if (!n) return NFK_OK;
    const int rc = nfk_schedule_calls(world_, n, qh_op_.data(), qh_h_.data(), qh_d_.data(), qh_kind_.data(),
                                      qh_t_.data(), qh_cnt_.data(), qh_now_.data());
    if (rc != NFK_ERR_NOTFOUND) return rc;
    int32_t k = 0;
    std::vector<int32_t> obj;
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = obj_of_.find(qh_h_[i], qh_d_[i]);
        if (o < 0) continue;
        obj.push_back(o);
        qh_op_[k] = qh_op_[i];
        qh_kind_[k] = qh_kind_[i];
        qh_t_[k] = qh_t_[i];
        qh_cnt_[k] = qh_cnt_[i];
        qh_now_[k] = qh_now_[i];
        k++;
    }
    return k ? nfk_schedule_calls_obj(world_, k, qh_op_.data(), obj.data(), qh_kind_.data(), qh_t_.data(),
                                      qh_cnt_.data(), qh_now_.data())
             : NFK_OK;
}

bool NFGPUKernelModule::SetRecordInt(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol,
                                     int64_t nValue) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (it == record_id_.end() || ObjectIndex(self) < 0) return false;
    const RecordDef& rd = records_[it->second];
    // NFCRecord::SetInt: ValidPos and the column type (RC:184-192)
    if (nRow < 0 || nRow >= rd.rows || nCol < 0 || nCol >= (int)rd.cols.size() || rd.cols[nCol] != TDATA_INT)
        return false;
    if (!((UsedRows(self, it->second) >> nRow) & 1)) return false;  // RC:194
    const int32_t rec = it->second, row = nRow, col = nCol;
    const uint8_t f = 0;
    const uint64_t b = (uint64_t)nValue;
    if (nfk_set_records(world_, 1, &self.nHead64, &self.nData64, &rec, &row, &col, &f, &b) != NFK_OK) return false;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

bool NFGPUKernelModule::SetRecordFloat(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol,
                                       double dwValue) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (it == record_id_.end() || ObjectIndex(self) < 0) return false;
    const RecordDef& rd = records_[it->second];
    if (nRow < 0 || nRow >= rd.rows || nCol < 0 || nCol >= (int)rd.cols.size() || rd.cols[nCol] != TDATA_FLOAT)
        return false;
    if (!((UsedRows(self, it->second) >> nRow) & 1)) return false;  // RC:255
    const int32_t rec = it->second, row = nRow, col = nCol;
    const uint8_t f = 1;
    uint64_t b;
    memcpy(&b, &dwValue, 8);
    if (nfk_set_records(world_, 1, &self.nHead64, &self.nData64, &rec, &row, &col, &f, &b) != NFK_OK) return false;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

uint64_t NFGPUKernelModule::UsedRows(const NFGUID& self, int rec) {
    const int32_t r = rec;
    uint64_t m = 0;
    check(nfk_get_used_rows(world_, 1, &self.nHead64, &self.nData64, &r, &m), "nfk_get_used_rows");
    return m;
}

bool NFGPUKernelModule::IsUsed(const NFGUID& self, const std::string& strRecordName, int nRow) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (!committed_ || it == record_id_.end() || ObjectIndex(self) < 0 || nRow < 0 || nRow >= records_[it->second].rows)
        return false;
    return (UsedRows(self, it->second) >> nRow) & 1;
}

// NFCRecord::AddRow (RC:111-180): the row it takes is known here from the used-row mask as the
// reference holds it now, so the call is queued with that explicit row
int NFGPUKernelModule::AddRow(const NFGUID& self, const std::string& strRecordName, int nRow,
                              const std::vector<TData>& values) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (!committed_ || it == record_id_.end() || ObjectIndex(self) < 0) return -1;
    const RecordDef& rd = records_[it->second];
    if (nRow >= rd.rows || nRow < -1) return -1;
    if (!values.empty() && values.size() != rd.cols.size()) return -1;  // RC:120
    for (size_t c = 0; c < values.size(); c++)
        if (values[c].GetType() != rd.cols[c]) return -1;  // RC:149-155
    if (nRow < 0) {
        const uint64_t used = UsedRows(self, it->second);
        const uint64_t fr = ~used & (rd.rows >= 64 ? ~0ull : ((1ull << rd.rows) - 1));
        if (!fr) return -1;
        nRow = __builtin_ctzll(fr);
    }
    uint64_t v[NFK_MAX_REC_COLS] = {};
    for (size_t c = 0; c < values.size(); c++)
        v[c] = rd.cols[c] == TDATA_INT ? (uint64_t)values[c].GetInt() : bits_of(values[c].GetFloat());
    const int32_t rec = it->second, op = 1, row = nRow;
    if (nfk_record_rows(world_, 1, &self.nHead64, &self.nData64, &rec, &op, &row, values.empty() ? nullptr : v) != NFK_OK)
        return -1;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return nRow;
}

// NFCRecord::Remove (RC:1086): true when the row was used
bool NFGPUKernelModule::RemoveRow(const NFGUID& self, const std::string& strRecordName, int nRow) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (!committed_ || it == record_id_.end() || ObjectIndex(self) < 0 || nRow < 0 || nRow >= records_[it->second].rows)
        return false;
    if (!((UsedRows(self, it->second) >> nRow) & 1)) return false;
    const int32_t rec = it->second, op = 2, row = nRow;
    if (nfk_record_rows(world_, 1, &self.nHead64, &self.nData64, &rec, &op, &row, nullptr) != NFK_OK) return false;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

// NFCKernelModule::ClearRecord (KM:492) -> NFCRecord::Clear (RC:1109)
bool NFGPUKernelModule::ClearRecord(const NFGUID& self, const std::string& strRecordName) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (!committed_ || it == record_id_.end() || ObjectIndex(self) < 0) return false;
    const int32_t rec = it->second, op = 3, row = 0;
    if (nfk_record_rows(world_, 1, &self.nHead64, &self.nData64, &rec, &op, &row, nullptr) != NFK_OK) return false;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

int64_t NFGPUKernelModule::GetRecordInt(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (it == record_id_.end() || ObjectIndex(self) < 0) return 0;
    const RecordDef& rd = records_[it->second];
    if (nRow < 0 || nRow >= rd.rows || nCol < 0 || nCol >= (int)rd.cols.size() || rd.cols[nCol] != TDATA_INT) return 0;
    const int32_t rec = it->second, row = nRow, col = nCol;
    uint64_t b = 0;
    if (nfk_get_records(world_, 1, &self.nHead64, &self.nData64, &rec, &row, &col, &b) != NFK_OK) return 0;
    return (int64_t)b;
}

double NFGPUKernelModule::GetRecordFloat(const NFGUID& self, const std::string& strRecordName, int nRow, int nCol) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = record_id_.find(strRecordName);
    if (it == record_id_.end() || ObjectIndex(self) < 0) return 0.0;
    const RecordDef& rd = records_[it->second];
    if (nRow < 0 || nRow >= rd.rows || nCol < 0 || nCol >= (int)rd.cols.size() || rd.cols[nCol] != TDATA_FLOAT)
        return 0.0;
    const int32_t rec = it->second, row = nRow, col = nCol;
    uint64_t b = 0;
    if (nfk_get_records(world_, 1, &self.nHead64, &self.nData64, &rec, &row, &col, &b) != NFK_OK) return 0.0;
    double v;
    memcpy(&v, &b, 8);
    return v;
}

bool NFGPUKernelModule::SetPropertyFloat(const NFGUID& self, const std::string& name, double v) {
    const int p = prop_ix_.find(name);
    if (!committed_ || p < 0 || props_[(size_t)p].type != TDATA_FLOAT) return false;
    if (walk_reads_ && in_walk_) WalkWrote(self, dev_pid_[(size_t)p]);
    qs_h_.push_back(self.nHead64);
    qs_d_.push_back(self.nData64);
    qs_pid_.push_back(dev_pid_[(size_t)p]);
    qs_bits_.push_back(bits_of(v));
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

// NFCKernelModule::GetPropertyInt/Float (KM:401-425): the value after this window's queued Sets
// (nfk_get_props, one element); an unknown object or property, or one of the other type, reads
// NULL_INT / NULL_FLOAT (TData::GetInt / GetFloat of a mismatched type)
int64_t NFGPUKernelModule::GetPropertyInt(const NFGUID& self, const std::string& name) {
    const int p = prop_ix_.find(name);
    if (!committed_ || ObjectIndex(self) < 0 || p < 0 || props_[(size_t)p].type != TDATA_INT) return 0;
    const int32_t pid = dev_pid_[(size_t)p];
    uint64_t b = 0;
    if (walk_reads_ && WalkRead(self, pid, &b)) return (int64_t)b;
    Flush();
    check(nfk_get_props(world_, 1, &self.nHead64, &self.nData64, &pid, &b), "nfk_get_props");
    return (int64_t)b;
}

double NFGPUKernelModule::GetPropertyFloat(const NFGUID& self, const std::string& name) {
    const int p = prop_ix_.find(name);
    if (!committed_ || ObjectIndex(self) < 0 || p < 0 || props_[(size_t)p].type != TDATA_FLOAT) return 0.0;
    const int32_t pid = dev_pid_[(size_t)p];
    uint64_t b = 0;
    if (walk_reads_ && WalkRead(self, pid, &b)) return dbl_of(b);
    Flush();
    check(nfk_get_props(world_, 1, &self.nHead64, &self.nData64, &pid, &b), "nfk_get_props");
    return dbl_of(b);
}

bool NFGPUKernelModule::SetPropertyObject(const NFGUID& self, const std::string& name, const NFGUID& v) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = prop_id_.find(name);
    if (!committed_ || it == prop_id_.end() || props_[it->second].type != TDATA_OBJECT || ObjectIndex(self) < 0) return false;
    const int32_t pid = dev_pid_[(size_t)it->second];
    if (nfk_set_objects(world_, 1, &self.nHead64, &self.nData64, &pid, &v.nHead64, &v.nData64) != NFK_OK) return false;
    if (shard_) NoteCall(self);
    pending_calls_++;
    return true;
}

// NFCKernelModule::GetPropertyObject (KM:440): NULL_OBJECT for an unknown object or property
NFGUID NFGPUKernelModule::GetPropertyObject(const NFGUID& self, const std::string& name) {
    Flush();  // (the buffered Set calls first: call order)
    auto it = prop_id_.find(name);
    if (!committed_ || ObjectIndex(self) < 0 || it == prop_id_.end() || props_[it->second].type != TDATA_OBJECT)
        return NFGUID();
    const int32_t pid = dev_pid_[(size_t)it->second];
    NFGUID v;
    check(nfk_get_objects(world_, 1, &self.nHead64, &self.nData64, &pid, &v.nHead64, &v.nData64), "nfk_get_objects");
    return v;
}

bool NFGPUKernelModule::RegisterCommonPropertyEvent(const PROPERTY_EVENT_FUNCTOR& cb) {
    common_prop_cb_.push_back(cb);
    return true;
}
bool NFGPUKernelModule::RegisterCommonRecordEvent(const RECORD_EVENT_FUNCTOR& cb) {
    common_rec_cb_.push_back(cb);
    return true;
}
bool NFGPUKernelModule::AddPropertyEventCallBack(const PROPERTY_SINGLE_EVENT_FUNCTOR& cb) {
    aoi_prop_cb_.push_back(cb);
    return true;
}
bool NFGPUKernelModule::AddRecordEventCallBack(const RECORD_SINGLE_EVENT_FUNCTOR& cb) {
    aoi_rec_cb_.push_back(cb);
    return true;
}

bool NFGPUKernelModule::AddPropertySyncCallBack(const PROPERTY_SYNC_FUNCTOR& cb) {
    if (!cb) return false;
    sync_prop_cb_.push_back(cb);
    return true;
}
bool NFGPUKernelModule::AddRecordSyncCallBack(const RECORD_SYNC_FUNCTOR& cb) {
    if (!cb) return false;
    sync_rec_cb_.push_back(cb);
    return true;
}

bool NFGPUKernelModule::AddFrameCallBack(const FRAME_FUNCTOR& cb, uint32_t what) {
    if (!cb) return false;
    frame_cb_.push_back(cb);
    frame_what_ |= what;
    return true;
}

// what one device pass reads back for the registered consumers (nfk_read_frame bits)
uint32_t NFGPUKernelModule::ReadMask(bool per_event_fired) const {
    const bool sync = !sync_prop_cb_.empty() || !sync_rec_cb_.empty();
    const bool cb_events = !common_prop_cb_.empty() || !aoi_prop_cb_.empty() || !common_rec_cb_.empty() ||
                           !aoi_rec_cb_.empty() || sync || (per_event_fired && frame_hook_);
    const bool cb_fan = !aoi_prop_cb_.empty() || !aoi_rec_cb_.empty() || sync;
    uint32_t what = 0;
    if (summary_.n_fired && ((per_event_fired && n_cb_) || (frame_what_ & NFK_READ_FIRED))) {
        what |= NFK_READ_FIRED;
        if ((per_event_fired && n_cb_) || (frame_what_ & NFK_READ_FIRED_GUID_ORDER)) what |= NFK_READ_FIRED_GUID_ORDER;
    }
    if ((cb_events || (frame_what_ & NFK_READ_EVENTS)) && (summary_.n_prop_events || summary_.n_rec_events))
        what |= NFK_READ_EVENTS | ((cb_fan || (frame_what_ & NFK_READ_FANOUT)) ? NFK_READ_FANOUT : 0u);
    return what;
}

// NFCScheduleModule::AddSchedule (SM:257-275): queued, added at the end of the next Execute unless
// the (object, name) still has a schedule then; the functor of the call that creates it is the one
// that fires (nfk_read_added tells which)
// (buffered by NFGUID like the Sets: SM:218-238 returns true without an object table, and a call
// on an object this module does not have is dropped at Flush)
bool NFGPUKernelModule::AddSchedule(const NFGUID& self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb,
                                    float fTime, int nCount) {
    return AddSchedule(self, name, cb, fTime, nCount, clock_());
}

bool NFGPUKernelModule::AddSchedule(const NFGUID& self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb,
                                    float fTime, int nCount, int64_t now_ms) {
    const int kind = hb_ix_.find(name);
    if (!committed_ || kind < 0) return false;
    QueueScheduleCall(1, self, kind, fTime, nCount, now_ms);
    sched_add_.push_back({self.nHead64, self.nData64, kind, cb, fTime});  // the window's first call wins
    return true;
}

// SM:245-249: into the remove list (first call per object per frame owns the key); a name with no
// device program removes nothing but still takes the key
bool NFGPUKernelModule::RemoveSchedule(const NFGUID& self, const std::string& name) {
    if (!committed_) return false;
    QueueScheduleCall(2, self, hb_ix_.find(name), 0.f, 0, 0);
    return true;
}

// SM:240-243: erases the object's schedules at once
bool NFGPUKernelModule::RemoveSchedule(const NFGUID& self) {
    if (!committed_) return false;
    QueueScheduleCall(3, self, 0, 0.f, 0, 0);
    return true;
}

// (buffered; Flush hands them to the world in one nfk_schedule_calls, call order kept)
void NFGPUKernelModule::QueueScheduleCall(int32_t op, const NFGUID& self, int32_t kind, float t, int32_t cnt,
                                          int64_t now) {
    qh_op_.push_back(op);
    qh_h_.push_back(self.nHead64);
    qh_d_.push_back(self.nData64);
    qh_kind_.push_back(kind);
    qh_t_.push_back(t);
    qh_cnt_.push_back(cnt);
    qh_now_.push_back(now);
    if (shard_) NoteCall(self);
    pending_calls_++;
}

void NFGPUKernelModule::DropPendingAdds(const NFGUID& g) {
    sched_add_.erase(std::remove_if(sched_add_.begin(), sched_add_.end(),
                                    [&g](const PendingAdd& a) { return a.h == g.nHead64 && a.d == g.nData64; }),
                     sched_add_.end());
}

// SM:276-285
bool NFGPUKernelModule::ExistSchedule(const NFGUID& self, const std::string& name) {
    Flush();  // (the buffered Set calls first: call order)
    auto k = hb_id_.find(name);
    if (!committed_ || ObjectIndex(self) < 0 || k == hb_id_.end()) return false;
    int32_t e = 0;
    check(nfk_exist_schedule(world_, self.nHead64, self.nData64, k->second, &e), "nfk_exist_schedule");
    return e != 0;
}

// module schedules (SM:184-216): host-side (ModuleScheduler), executed after the object schedules
bool NFGPUKernelModule::AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR& cb, float fTime,
                                    int nCount) {
    return module_sched_.AddSchedule(name, cb, fTime, nCount, clock_());
}

bool NFGPUKernelModule::RemoveSchedule(const std::string& name) { return module_sched_.RemoveSchedule(name); }

bool NFGPUKernelModule::ExistSchedule(const std::string& name) { return module_sched_.ExistSchedule(name); }

namespace {
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

void NFGPUKernelModule::SetKindFunctor(const std::string& name, const OBJECT_SCHEDULE_FUNCTOR& cb, float fTime) {
    kind_cb_[name] = {cb, fTime};
}

// the shard exchange (collective): departures leave, arrivals become this module's objects, their
// schedules with the functors of their names.  sync: gather the tickets now (MigrateNow); else the
// rows of the gather the previous Execute started (SceneShard::BeginFrame)
void NFGPUKernelModule::MigrateShard(bool sync) {
    WaitGather();  // (the gather's workers read guids_)
    // calls made on a departing entity since the last device pass would stay queued in the world while
    // its row leaves (k_pack copies the device row): the window's calls are applied first, in a pass of
    // their own with their events delivered, as the functors' calls are; windows with no call
    // on a departing entity pay nothing (NoteCall, Depart)
    if (transit_calls_ && pending_calls_) CallsPass();
    Flush();  // (the buffered Set calls first: call order)
    std::vector<Ticket> sent, recv;
    if (sync) check(shard_->Migrate(&sent, &recv), "SceneShard::Migrate");
    else check(shard_->BeginFrame(&sent, &recv), "SceneShard::BeginFrame");
    for (const Ticket& k : sent) {  // their rows have left the world: no longer this module's objects
        departing_.erase(k.guid_head, k.guid_data);
        const int o = obj_of_.find(k.guid_head, k.guid_data);
        if (o < 0) continue;
        obj_of_.erase(k.guid_head, k.guid_data);  // (its object index stays reserved)
        DropFunctors(o);
        DropPendingAdds(NFGUID(k.guid_head, k.guid_data));
    }
    for (const Ticket& k : recv) {
        const NFGUID g(k.guid_head, k.guid_data);
        const int o = (int)guids_.size();
        obj_of_.insert(g.nHead64, g.nData64, o);
        guids_.push_back(g);
        scene_.push_back(k.scene);
        group_.push_back(k.group);
        cls_.push_back((uint8_t)k.cls);
        isplayer_.push_back((uint8_t)k.is_player);
        scenes_[k.scene] = true;
        for (auto& kv : kind_cb_) {
            auto h = hb_id_.find(kv.first);
            if (h != hb_id_.end()) SetFunctor(o, h->second, kv.second.first, kv.second.second);
        }
    }
}

bool NFGPUKernelModule::Execute() {
    const auto t0 = std::chrono::steady_clock::now();
    stats_ = FrameStats{};
    if (shard_) MigrateShard(false);
    Flush();
    check(nfk_execute(world_, clock_()), "nfk_execute");
    pending_calls_ = 0;
    touched_.clear();
    transit_calls_ = false;
    if (shard_) WindowApplied();
    check(nfk_summary_get(world_, &summary_), "nfk_summary_get");
    stats_.device = ms_since(t0);
    auto t1 = std::chrono::steady_clock::now();
    TakeAddedSchedules();  // the AddSchedule calls this frame applied: their functors fire from now on
    // the frame's outputs in one read-back (nfk_read_frame): the fired list in the order
    // NFCScheduleModule::Execute walks mObjectScheduleMap — objects in NFGUID order, each object's
    // schedules in name order (SM:52-80), sorted on the device — and the event lists
    const uint32_t what = ReadMask(true);
    nfk_frame_host fh{};
    // (the gather reads fh: it is waited for before fh goes, however Execute leaves)
    struct GatherGuard {
        NFGPUKernelModule* m;
        ~GatherGuard() { m->WaitGather(); }
    } gather_guard{this};
    if (what) check(nfk_read_frame(world_, what, &fh), "nfk_read_frame");
    ReadChain();
    stats_.events_read = ms_since(t1);
    t1 = std::chrono::steady_clock::now();
    if (frame_hook_) frame_hook_(fh);  // (before the functors: they see the frame's values)
    stats_.mirror = ms_since(t1);
    t1 = std::chrono::steady_clock::now();
    // heartbeat functors with the reference's arguments, objects in NFGUID order (the fired list's)
    const int64_t nfi = n_cb_ ? fh.n_fi : 0;  // (a frame consumer may read the list without functors)
    const bool gathered = GatherFrame(fh, nfi);
    double gather_ms = ms_since(t1);
    in_walk_ = true;
    walk_ix_built_ = false;
    walk_set_.clear();
    if (gathered) {
        // the functor entries, NFGUIDs and intervals are dense arrays, gathered chunk by chunk
        // ahead of the walk: only the functor objects themselves are scattered (prefetched ahead)
        constexpr int64_t kPre = 16;
        for (int64_t i0 = 0, k = 0; i0 < nfi; i0 += kGatherChunk, k++) {
            if (!fg_ready_[(size_t)k].load(std::memory_order_acquire)) {
                const auto tw = std::chrono::steady_clock::now();
                // (a functor that wrote guids_ / cb_slot_ / cb_time_ waited for the whole gather)
                while (gather_job_ && !fg_ready_[(size_t)k].load(std::memory_order_acquire)) std::this_thread::yield();
                gather_ms += ms_since(tw);
            }
            const int64_t i1 = std::min(nfi, i0 + kGatherChunk);
            for (int64_t i = i0; i < i1; i++) {
                if (i + kPre < i1 && fg_c_[(size_t)(i + kPre)] >= 0) __builtin_prefetch(&cb_pool_[(size_t)fg_c_[(size_t)(i + kPre)]]);
                const int32_t c = fg_c_[(size_t)i];
                // (empty: a functor earlier in this walk destroyed the object or moved it to another shard)
                if (c >= 0 && cb_pool_[(size_t)c]) {
                    walk_o_ = fh.fi_obj[i];
                    walk_k_ = fh.fi_kind[i];
                    cb_pool_[(size_t)c](fg_g_[(size_t)i], heartbeats_[(size_t)fh.fi_kind[i]].name, fg_t_[(size_t)i], fh.fi_remain[i]);
                }
            }
        }
    } else {
        // (a small frame, or no workers) its (object, kind) functor slots, pooled functors and NFGUIDs
        // are scattered host reads, prefetched two stages ahead
        const size_t nk = heartbeats_.size(), nslot = cb_slot_.size();
        constexpr int64_t kPre = 16;
        for (int64_t i = 0; i < nfi; i++) {
            if (i + 2 * kPre < nfi) {
                const int64_t j = i + 2 * kPre;
                const size_t at = (size_t)fh.fi_obj[j] * nk + (size_t)fh.fi_kind[j];
                if (at < nslot) __builtin_prefetch(&cb_slot_[at]);
                __builtin_prefetch(&guids_[(size_t)fh.fi_obj[j]]);
            }
            if (i + kPre < nfi) {
                const int64_t j = i + kPre;
                const size_t at = (size_t)fh.fi_obj[j] * nk + (size_t)fh.fi_kind[j];
                const int32_t c = at < nslot ? cb_slot_[at] : -1;
                if (c >= 0) {
                    __builtin_prefetch(&cb_pool_[(size_t)c]);
                    __builtin_prefetch(&cb_time_[(size_t)c]);
                }
            }
            const int o = fh.fi_obj[i], k = fh.fi_kind[i];
            const size_t at = (size_t)o * nk + (size_t)k;
            const int32_t c = at < cb_slot_.size() ? cb_slot_[at] : -1;
            if (c >= 0) {
                walk_o_ = o;
                walk_k_ = k;
                cb_pool_[c](guids_[o], heartbeats_[k].name, cb_time_[c], fh.fi_remain[i]);
            }
        }
    }
    in_walk_ = false;
    walk_o_ = walk_k_ = -1;
    {
        const auto tw = std::chrono::steady_clock::now();
        WaitGather();  // the events' part, gathered while the walk ran
        gather_ms += ms_since(tw);
    }
    stats_.functors = ms_since(t1) - gather_ms;
    stats_.gather = gather_ms;
    t1 = std::chrono::steady_clock::now();
    if (what & NFK_READ_EVENTS)
        DeliverEvents(fh, gathered && !ev_self_.empty() ? ev_self_.data() : nullptr,
                      gathered && !re_self_.empty() ? re_self_.data() : nullptr,
                      gathered && !ev_same_.empty() ? ev_same_.data() : nullptr);
    if (what)
        for (auto& fc : frame_cb_) fc(fh, guids_.data());
    stats_.deliver = ms_since(t1);
    // what the functors called takes effect in this Execute (SM:65: their Sets land at once;
    // SM:83-119: their Add/RemoveSchedule calls are applied at the end of the walk)
    t1 = std::chrono::steady_clock::now();
    if (same_frame_ && pending_calls_) CallsPass();
    module_sched_.Execute(clock_);  // module schedules (SM:123-176)
    // the departures queued up to now (this window's and the functors'): their tickets are
    // gathered off the world's stream while the next window's game logic runs
    if (shard_) check(shard_->EndFrame(), "SceneShard::EndFrame");
    stats_.calls = ms_since(t1);
    stats_.total = ms_since(t0);
    return true;
}

// The calls queued since the last device pass applied now (nfk_execute_calls: nothing fires), their
// events delivered
void NFGPUKernelModule::CallsPass() {
    Flush();
    check(nfk_execute_calls(world_), "nfk_execute_calls");
    pending_calls_ = 0;
    touched_.clear();
    transit_calls_ = false;
    check(nfk_summary_get(world_, &summary_), "nfk_summary_get");
    TakeAddedSchedules();
    // the pass fires no heartbeats: only its events
    const uint32_t w2 = ReadMask(false) & ~(NFK_READ_FIRED | NFK_READ_FIRED_GUID_ORDER);
    if (w2) {
        nfk_frame_host f2{};
        check(nfk_read_frame(world_, w2, &f2), "nfk_read_frame");
        DeliverEvents(f2);
        for (auto& fc : frame_cb_) fc(f2, guids_.data());
    }
}

void NFGPUKernelModule::SetFunctor(int o, int k, const OBJECT_SCHEDULE_FUNCTOR& f, float t) {
    WaitGather();  // (the gather's workers read cb_slot_ and cb_time_)
    const size_t nk = heartbeats_.size(), at = (size_t)o * nk + k;
    if (cb_slot_.size() < guids_.size() * nk) cb_slot_.resize(guids_.size() * nk + nk * 1024, -1);
    int32_t c = cb_slot_[at];
    if (!f) {  // a schedule with no host functor (its device program is all it does)
        if (c >= 0) {
            cb_pool_[c] = nullptr;
            cb_free_.push_back(c);
            cb_slot_[at] = -1;
            n_cb_--;
        }
        return;
    }
    if (c < 0) {
        if (!cb_free_.empty() && !in_walk_) {  // (a gathered entry of the walk stays what it was)
            c = cb_free_.back();
            cb_free_.pop_back();
        } else {
            c = (int32_t)cb_pool_.size();
            cb_pool_.emplace_back();
            cb_time_.push_back(0.0f);
        }
        cb_slot_[at] = c;
        n_cb_++;
    }
    cb_pool_[c] = f;
    cb_time_[c] = t;
}

void NFGPUKernelModule::DropFunctors(int o) {
    WaitGather();  // (the gather's workers read cb_slot_)
    const size_t nk = heartbeats_.size();
    for (size_t k = 0; k < nk; k++) {
        const size_t at = (size_t)o * nk + k;
        if (at >= cb_slot_.size() || cb_slot_[at] < 0) continue;
        cb_pool_[cb_slot_[at]] = nullptr;
        cb_free_.push_back(cb_slot_[at]);
        cb_slot_[at] = -1;
        n_cb_--;
    }
}

// AddSchedule calls that the last device pass applied and that created a schedule: their functors
// fire from now on (the first call of a name wins, SM:218-238; nfk_read_added says which)
void NFGPUKernelModule::TakeAddedSchedules() {
    if (sched_add_.empty()) return;
    // by key, call order kept within a key: the first call of each key leads its run
    const int32_t cap = (int32_t)sched_add_.size();
    ta_key_.resize((size_t)cap);
    for (int32_t i = 0; i < cap; i++) ta_key_[(size_t)i] = {sched_add_[(size_t)i].h, sched_add_[(size_t)i].d, sched_add_[(size_t)i].kind, i};
    std::sort(ta_key_.begin(), ta_key_.end());
    ta_h_.resize((size_t)cap);
    ta_d_.resize((size_t)cap);
    ta_k_.resize((size_t)cap);
    int32_t n = 0;
    check(nfk_read_added(world_, cap, &n, ta_h_.data(), ta_d_.data(), ta_k_.data()), "nfk_read_added");
    n = std::min(n, cap);
    // the new functor entries are taken in the order the heartbeat walk reads them (NFGUID, then
    // kind): the pool the walk streams through is then in walk order for every batch of adds (an
    // (object, kind) added again later reuses its entry)
    ta_ord_.resize((size_t)n);
    for (int32_t i = 0; i < n; i++) ta_ord_[(size_t)i] = i;
    static const bool ordered = !(getenv("NFGPU_PLUGIN_POOL_ORDER") && getenv("NFGPU_PLUGIN_POOL_ORDER")[0] == '0');
    if (ordered)
        std::sort(ta_ord_.begin(), ta_ord_.end(), [&](int32_t a, int32_t b) {
            const NFGUID ga(ta_h_[(size_t)a], ta_d_[(size_t)a]), gb(ta_h_[(size_t)b], ta_d_[(size_t)b]);
            return ga < gb || (ga == gb && ta_k_[(size_t)a] < ta_k_[(size_t)b]);
        });
    for (int32_t j = 0; j < n; j++) {
        const int32_t i = ta_ord_[(size_t)j];
        const int o = ObjectIndex(NFGUID(ta_h_[(size_t)i], ta_d_[(size_t)i]));
        if (o < 0) continue;
        const AddKey q{ta_h_[(size_t)i], ta_d_[(size_t)i], ta_k_[(size_t)i], -1};
        auto it = std::lower_bound(ta_key_.begin(), ta_key_.end(), q);
        if (it == ta_key_.end() || it->h != q.h || it->d != q.d || it->kind != q.kind) continue;
        const PendingAdd& pa = sched_add_[(size_t)it->i];
        SetFunctor(o, q.kind, pa.cb, pa.t);
    }
    sched_add_.clear();
}

void NFGPUKernelModule::WaitGather() {
    if (!gather_job_) return;
    pool_->Wait(gather_job_);
    gather_job_.reset();
}

// Started before any functor of the frame runs: the fired list's functor entries, NFGUIDs and
// intervals, and the events' NFGUIDs, gathered in chunks by the worker pool while the walk runs —
// the fired chunks first, in order, each flagged in fg_ready_ when done (the walk waits for its
// chunk), then the events.  No game code writes what the workers read while they run (WaitGather
// before every such write).  False for a frame too small to pay for it, or with no workers.
bool NFGPUKernelModule::GatherFrame(const nfk_frame_host& fh, int64_t nfi) {
    WaitGather();
    const bool ev = !(common_prop_cb_.empty() && aoi_prop_cb_.empty() && common_rec_cb_.empty() && aoi_rec_cb_.empty() &&
                      sync_prop_cb_.empty() && sync_rec_cb_.empty());
    const int64_t nev = ev ? fh.n_ev : 0, nre = ev ? fh.n_re : 0;
    ev_self_.clear();
    re_self_.clear();
    static const int64_t kMin = getenv("NFGPU_PLUGIN_GATHER_MIN") ? atoll(getenv("NFGPU_PLUGIN_GATHER_MIN")) : (1 << 15);
    if (nfi + nev + nre < std::max<int64_t>(kMin, 1)) return false;
    if (!pool_) {
        const char* e = getenv("NFGPU_PLUGIN_THREADS");
        const int nw = e ? atoi(e) : 8;
        if (nw <= 0) return false;
        pool_.reset(new nfgpu_detail::WorkerPool(nw));
    }
    fg_c_.resize((size_t)nfi);
    fg_g_.resize((size_t)nfi);
    fg_t_.resize((size_t)nfi);
    ev_self_.resize((size_t)nev);
    re_self_.resize((size_t)nre);
    // (per property event: its recipient run equals the previous event's, so the delivery reuses the
    // NFGUID list it built; consecutive events of a scene group mostly share their recipients)
    static const bool same_on = !(getenv("NFGPU_PLUGIN_SAME") && getenv("NFGPU_PLUGIN_SAME")[0] == '0');
    const bool runs = same_on && fh.msg_off && (!aoi_prop_cb_.empty() || !sync_prop_cb_.empty());
    ev_same_.resize(runs ? (size_t)nev : 0);
    constexpr int64_t kChunk = kGatherChunk, kPre = 16;
    const int64_t cf = (nfi + kChunk - 1) / kChunk, ce = (nev + kChunk - 1) / kChunk, cr = (nre + kChunk - 1) / kChunk;
    const size_t nk = heartbeats_.size(), nslot = cb_slot_.size();
    if ((size_t)cf > fg_ready_cap_) {
        fg_ready_cap_ = (size_t)cf + (size_t)cf / 4 + 16;
        fg_ready_.reset(new std::atomic<uint8_t>[fg_ready_cap_]);
    }
    for (int64_t k = 0; k < cf; k++) fg_ready_[(size_t)k].store(0, std::memory_order_relaxed);
    // (fh lives until Execute returns; Execute waits for the job before it does)
    const nfk_frame_host* fp = &fh;
    gather_job_ = pool_->Start(cf + ce + cr, [this, fp, nfi, nev, nre, cf, ce, nk, nslot, runs](int64_t q) {
        const nfk_frame_host& fh = *fp;
        if (q < cf) {
            const int64_t i0 = q * kChunk, i1 = std::min(nfi, i0 + kChunk);
            for (int64_t i = i0; i < i1; i++) {
                if (i + kPre < i1) {
                    const size_t at = (size_t)fh.fi_obj[i + kPre] * nk + (size_t)fh.fi_kind[i + kPre];
                    if (at < nslot) __builtin_prefetch(&cb_slot_[at]);
                    __builtin_prefetch(&guids_[(size_t)fh.fi_obj[i + kPre]]);
                }
                const size_t at = (size_t)fh.fi_obj[i] * nk + (size_t)fh.fi_kind[i];
                const int32_t c = at < nslot ? cb_slot_[at] : -1;
                fg_c_[(size_t)i] = c;
                fg_g_[(size_t)i] = guids_[(size_t)fh.fi_obj[i]];
                fg_t_[(size_t)i] = c >= 0 ? cb_time_[(size_t)c] : 0.f;
            }
            fg_ready_[(size_t)q].store(1, std::memory_order_release);
        } else if (q < cf + ce) {
            const int64_t i0 = (q - cf) * kChunk, i1 = std::min(nev, i0 + kChunk);
            for (int64_t i = i0; i < i1; i++) {
                if (i + kPre < i1) __builtin_prefetch(&guids_[(size_t)fh.ev_obj[i + kPre]]);
                ev_self_[(size_t)i] = guids_[(size_t)fh.ev_obj[i]];
            }
            if (runs) {
                // against the last event before it with a non-empty run (the one the delivery's
                // list then holds: events with no recipients make no AOI call)
                int64_t p = i0 - 1;
                while (p >= 0 && fh.msg_off[p + 1] == fh.msg_off[p]) p--;
                for (int64_t i = i0; i < i1; i++) {
                    const uint32_t m0 = fh.msg_off[i], m1 = fh.msg_off[i + 1];
                    if (m1 == m0) {
                        ev_same_[(size_t)i] = 0;
                        continue;
                    }
                    const uint32_t q0 = p >= 0 ? fh.msg_off[p] : 0u, q1 = p >= 0 ? fh.msg_off[p + 1] : 0u;
                    ev_same_[(size_t)i] = p >= 0 && m1 - m0 == q1 - q0 &&
                                          std::memcmp(fh.msg_rcpt + m0, fh.msg_rcpt + q0, (size_t)(m1 - m0) * 4) == 0;
                    p = i;
                }
            }
        } else {
            const int64_t i0 = (q - cf - ce) * kChunk, i1 = std::min(nre, i0 + kChunk);
            for (int64_t i = i0; i < i1; i++) {
                if (i + kPre < i1) __builtin_prefetch(&guids_[(size_t)fh.re_obj[i + kPre]]);
                re_self_[(size_t)i] = guids_[(size_t)fh.re_obj[i]];
            }
        }
    });
    return true;
}

// An event's old / new values as TData: built per event with each field written once and without a
// branch on the type (resetting and rewriting two long-lived TData objects, and a branch that the
// mixed int / float events of a frame mispredict, cost more than the callbacks); the object values
// are the caller's
static inline void TDataOf(TDATA_TYPE t, uint64_t vo, uint64_t vn, TData* a, TData* b) {
    const uint64_t mi = 0 - (uint64_t)(t == TDATA_INT), mf = 0 - (uint64_t)(t == TDATA_FLOAT);
    a->type = b->type = t;
    a->i = (int64_t)(vo & mi);
    b->i = (int64_t)(vn & mi);
    a->f = dbl_of(vo & mf);
    b->f = dbl_of(vn & mf);
}

void NFGPUKernelModule::DeliverEvents(const nfk_frame_host& f, const NFGUID* ev_self, const NFGUID* re_self,
                                      const uint8_t* ev_same) {
    if (common_prop_cb_.empty() && aoi_prop_cb_.empty() && common_rec_cb_.empty() && aoi_rec_cb_.empty() &&
        sync_prop_cb_.empty() && sync_rec_cb_.empty())
        return;
    static const std::vector<NFGUID> kNone;
    const bool sync_p = !sync_prop_cb_.empty(), sync_r = !sync_rec_cb_.empty();
    const bool want_p = f.msg_off && (!aoi_prop_cb_.empty() || sync_p);
    const bool want_r = f.msg_off && (!aoi_rec_cb_.empty() || sync_r);
    std::vector<NFGUID> rcpt;
    uint32_t rcpt_at = 0, rcpt_n = 0xFFFFFFFFu;  // the msg_rcpt run rcpt holds
    constexpr int64_t kPre = 16;  // events are in slot order; their objects' NFGUIDs are scattered
    for (int64_t e = 0; e < f.n_ev; e++) {
        if (!ev_self && e + kPre < f.n_ev) __builtin_prefetch(&guids_[(size_t)f.ev_obj[e + kPre]]);
        const PropertyDef& pd = props_[def_of_pid_[f.ev_pid[e]]];
        TData a, b;
        TDataOf(pd.type, f.ev_old[e], f.ev_new[e], &a, &b);
        if (pd.type == TDATA_OBJECT) {
            a.o = NFGUID((int64_t)f.ev_old_h[e], (int64_t)f.ev_old[e]);
            b.o = NFGUID((int64_t)f.ev_new_h[e], (int64_t)f.ev_new[e]);
        }
        const NFGUID& self = ev_self ? ev_self[e] : guids_[f.ev_obj[e]];
        for (auto& cb : common_prop_cb_) cb(self, pd.name, a, b);
        bool same = false;
        const bool run = want_p && f.msg_off[e + 1] > f.msg_off[e];
        if (run) {  // AOI.cpp:250: no AOI call for an empty list
            // consecutive events of a scene group mostly share their recipients: rebuild the list
            // only when the run differs from the last one delivered (ev_same: compared by the workers)
            const uint32_t m0 = f.msg_off[e], m1 = f.msg_off[e + 1];
            same = ev_same ? ev_same[e] != 0
                           : m1 - m0 == rcpt_n && memcmp(f.msg_rcpt + m0, f.msg_rcpt + rcpt_at, (size_t)(m1 - m0) * 4) == 0;
            if (!same) {
                rcpt.resize(m1 - m0);
                for (uint32_t m = m0; m < m1; m++) rcpt[m - m0] = guids_[f.msg_rcpt[m]];
            }
            rcpt_at = m0;
            rcpt_n = m1 - m0;
            for (auto& cb : aoi_prop_cb_) cb(self, pd.name, a, b, rcpt);
        }
        if (sync_p) {
            const SyncArgs sa{f.ev_obj[e], run ? &rcpt : &kNone, run && same};
            for (auto& cb : sync_prop_cb_) cb(self, f.ev_pid[e], a, b, sa);
        }
    }
    rcpt_n = 0xFFFFFFFFu;  // (the record runs: the first one is built)
    RECORD_EVENT_DATA ev;
    int ev_r = -1;  // the record ev.strRecordName holds (a name copy per event would allocate)
    for (int64_t e = 0; e < f.n_re; e++) {
        const uint32_t rrc = f.re_rrc[e];
        const int r = (rrc >> 16) & 0xFF, row = (rrc >> 8) & 0xFF, col = rrc & 0xFF, op = (rrc >> 24) & 3;
        // row events (AddRow / Remove / Clear) carry empty values, as NFCRecord raises them (RC:177, 1098)
        ev.nOpType = op == 1 ? RECORD_EVENT_DATA::Add : op == 2 ? RECORD_EVENT_DATA::Del
                   : op == 3 ? RECORD_EVENT_DATA::Cover : RECORD_EVENT_DATA::Update;
        ev.nRow = row;
        ev.nCol = col;
        if (r != ev_r) {
            ev.strRecordName = records_[r].name;
            ev_r = r;
        }
        TData a, b;
        TDataOf(op ? TDATA_UNKNOWN : records_[r].cols[col], f.re_old[e], f.re_new[e], &a, &b);
        const NFGUID& self = re_self ? re_self[e] : guids_[f.re_obj[e]];
        for (auto& cb : common_rec_cb_) cb(self, ev, a, b);
        if (want_r) {  // (AOI.cpp:285-287 calls OnRecordEvent with an empty list too)
            const uint32_t m0 = f.msg_off[f.n_ev + e], m1 = f.msg_off[f.n_ev + e + 1];
            bool same = false;
            if (m1 > m0) {
                same = m1 - m0 == rcpt_n && memcmp(f.msg_rcpt + m0, f.msg_rcpt + rcpt_at, (size_t)(m1 - m0) * 4) == 0;
                if (!same) {
                    rcpt.resize(m1 - m0);
                    for (uint32_t m = m0; m < m1; m++) rcpt[m - m0] = guids_[f.msg_rcpt[m]];
                }
                rcpt_at = m0;
                rcpt_n = m1 - m0;
            }
            const std::vector<NFGUID>& rl = m1 > m0 ? rcpt : kNone;
            for (auto& cb : aoi_rec_cb_) cb(self, ev.strRecordName, ev, a, b, rl);
            if (sync_r) {
                const SyncArgs sa{f.re_obj[e], &rl, m1 > m0 && same};
                for (auto& cb : sync_rec_cb_) cb(self, ev, a, b, sa);
            }
        }
    }
}

bool NFGPUKernelModule::BeforeShut() { return true; }

bool NFGPUKernelModule::Shut() {
    WaitGather();
    if (world_) nfk_destroy(world_);
    world_ = nullptr;
    return true;
}

}  // namespace nfgpu
