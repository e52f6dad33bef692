// nfgpu_host.hip — C-ABI implementation (include/nfgpu.h): world lifetime, schema,
// membership layout, queued SetProperty / schedule calls, frame launch, readback.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include <mutex>
#include <thread>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "nfgpu_jit.hpp"
#include "nfgpu_kernels.hip"
#include "../../include/nfgpu_guidmap.hpp"
#include "nfgpu_pool.hpp"

using namespace nfgpu;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t _e = (x);                                                               \
        if (_e != hipSuccess)                                                              \
            return fail(NFK_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e));     \
    } while (0)

using nfgpu_detail::GuidMap;
using nfgpu_detail::HostPool;

template <typename T>
int dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return fail(NFK_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    return NFK_OK;
}

enum { KT_TICK = 0, KT_REC = 1, KT_FAN = 2, KT_AUX = 3, KT_SCAN = 4, KT_MEM = 5, KT_CHAIN = 6, KT_N = 7 };
static_assert(KT_N == NFK_N_KERNEL_TIMERS, "nfk_kernel_times' arrays");

struct PendingTiming {
    int kind;
    hipEvent_t a, b;
    int64_t bytes_before;
};

struct MemPlan;

struct World {
    nfk_config cfg{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int32_t n_obj = 0;
    bool committed = false;
    int n_prop = 0;  // properties: int [0, n_int), f64 [n_int, n_if), object (NFGUID) [n_if, n_prop)
    int n_if = 0;    // n_int + n_flt
    int n_pw = 0;    // property words of a row: n_if + 2 object halves per object property
    // host-mapped error word (Dev::err_host): device error bits, seen without a device read
    unsigned* err_host = nullptr;
    unsigned* err_host_d = nullptr;

    std::vector<int64_t> gh, gd;
    struct Guid { int64_t h, d; };
    std::vector<Guid> guid;  // (gh, gd) side by side: one cache line per NFGUID comparison
    std::vector<int32_t> scene, group;
    std::vector<uint8_t> cls, isplayer;
    GuidMap obj_of;
    std::vector<int32_t> slot_of_obj, obj_of_slot;  // -1: not resident / slack slot
    std::vector<uint8_t> alive;                       // object exists (not destroyed / exported)
    std::vector<int64_t> src_row;                     // >= 0: arrives from row src_row of ins_rows
    std::vector<uint8_t> m_flag;                      // membership changed in this window
    std::vector<int32_t> touched;                     // objects with m_flag set
    // scene-group segments in (scene, group) order; slot range [base, base + cap)
    struct Seg {
        int32_t scene, group, base, cap;
        int32_t np = 0;             // players among objs (set by seg_meta)
        std::vector<int32_t> objs;  // live objects, NFGUID order
        // their NFGUIDs, beside them: a joiner's place is binary-searched in this contiguous array
        // instead of through guid[objs[i]] (one random host read per probe, ~8 per joiner)
        std::vector<Guid> keys;
    };
    std::vector<Seg> segs;
    std::vector<uint64_t> seg_key;  // each segment's (scene, group) as seg_key_of gives it: ascending
    int32_t slack = 16;  // slack slots per 256 live (nfk_config::slack_per_256)
    int32_t pid_scene = -1, pid_group = -1, pid_x = -1, pid_y = -1, pid_z = -1;  // nfk_set_scene_props
    int32_t row_words = 0;
    uint64_t* ins_rows = nullptr;  // rows of entities imported this window
    size_t ins_cap = 0, ins_n = 0;
    uint64_t* mv_rows = nullptr;   // rows of entities moving inside this shard
    size_t mv_cap = 0;
    void* mlist = nullptr;         // device copy of the membership lists
    size_t mlist_cap = 0;
    std::vector<char> mhost;       // host staging of the membership lists
    // pinned double buffer the lists are uploaded from, so no upload waits for the stream
    char* mpin[2] = {nullptr, nullptr};
    size_t mpin_cap[2] = {0, 0};
    hipEvent_t mpin_done[2] = {nullptr, nullptr};
    bool mpin_pending[2] = {false, false};
    int mpin_slot = 0;
    // nfk_export_objects' slot list, read by k_pack straight from pinned host memory (a few
    // hundred rows: no copy, which behind a busy stream could wait for it)
    int32_t* xpin = nullptr;
    int32_t* xpin_dev = nullptr;
    size_t xpin_cap = 0;
    hipEvent_t xpin_done = nullptr;
    bool xpin_pending = false;
    uint64_t* fan_desc_w = nullptr;
    int32_t* pl_slot_w = nullptr;
    int64_t n_relayout_full = 0, n_relayout_seg = 0;
    double ms_relayout_full = 0, ms_relayout_seg = 0;  // host time in plan/commit_membership
    std::unique_ptr<MemPlan> mplan;            // the window's membership plan (scratch kept)
    void* glist = nullptr;  // device-generated membership lists (untouched segments of a full re-layout)
    size_t glist_cap = 0;
    std::vector<std::vector<uint64_t>> init_props;
    std::vector<std::vector<uint64_t>> init_rcells, init_rused;
    std::vector<bool> rec_defined;
    uint8_t rec_ctype[NFK_MAX_RECORDS][NFK_MAX_REC_COLS] = {};  // 0 = int64, 1 = f64

    Tables tab{};
    bool kind_defined[NFK_MAX_KINDS] = {};
    uint64_t dst_union_mask[2] = {0, 0};  // properties written by any program (bit per pid)
    // frame working set of k_tick (Dev::u_*): program destinations / read-only operands
    bool u_ok = false;
    std::vector<int> u_wp, u_rp;
    int n_dst_union = 0;

    Dev d{};
    Tables* tab_d = nullptr;
    Ctrl* ctrl = nullptr;
    int32_t* slot_obj_d = nullptr;
    int32_t nseg = 0;
    std::vector<void*> allocs;
    // dense readback scratch (nfk_read_*), grown on demand
    void* dense = nullptr;
    size_t dense_cap = 0;
    // nfk_read_frame: the dense region on the device and its pinned host copy, device scratch, and
    // the NFGUID order of the objects (guid_sorted; rank_d[object] on the device for rank_n objects)
    void* fr_dev = nullptr;
    char* fr_pin = nullptr;
    size_t fr_cap = 0;
    void* fr_scr = nullptr;
    size_t fr_scap = 0;
    std::vector<int32_t> guid_sorted;
    int32_t* rank_d = nullptr;
    size_t rank_cap = 0;
    int32_t rank_n = 0;

    // queued calls
    // queued calls; `slot` holds the object index until nfk_execute resolves it after the
    // window's membership changes
    struct XOp { uint32_t slot, pid; uint64_t bits; };
    std::vector<XOp> xops;
    std::vector<uint64_t> xops_h;  // the NFGUID head half of each queued call (worlds with object properties)
    // the SetProperty groups are folded on the device (k_xkeys, radix sort, k_scan_heads,
    // k_xgroups): object -> slot after the window's membership changes (rebuilt by k_obj_slots
    // when the membership changed), and the fold's scratch
    int32_t* obj_slot_d = nullptr;
    size_t obj_slot_cap = 0;
    bool obj_slot_dirty = true;
    void* xf_buf = nullptr;
    size_t xf_cap = 0;
    // SetProperty calls of large batches queued on the device (set_props_dev), in two buffers used
    // by alternate windows: the window's first xq_n calls are xq[xq_b][0, xq_n) (XOp records), the
    // host xops the calls queued after them; xq_ev[b]: the frame that folded buffer b read it
    void* xq[2] = {nullptr, nullptr};
    size_t xq_cap[2] = {0, 0};  // records
    hipEvent_t xq_ev[2] = {nullptr, nullptr};
    bool xq_ev_set[2] = {false, false};
    int xq_b = 0;
    size_t xq_n = 0;
    uint8_t* tile_work_d = nullptr;  // a calls-only pass's tiles with SetProperty groups (Dev::tile_work)
    size_t tile_work_cap = 0;
    std::vector<int32_t> look;           // GUID lookups of one batched call
    // GUID lookups of large call batches on the device (find_many_dev): obj_of's device mirror
    // (guid_d, same entries and hash), the log of the entries the host table wrote since the
    // mirror was last brought up to date, the batch's pinned and device buffers, and a stream of
    // their own (the world's stream may be running the previous frame)
    std::vector<uint32_t> guid_log;
    void* guid_d = nullptr;
    size_t guid_dcap = 0;       // bytes
    size_t guid_dmask = 0;      // capacity - 1 of the mirrored table
    bool guid_synced = false;
    hipStream_t look_stream = nullptr;
    char* look_pin = nullptr;
    size_t look_pin_cap = 0;
    void* look_dev = nullptr;
    size_t look_dev_cap = 0;
    size_t dev_look_min = 4096;  // batches from this size on (NFGPU_DEV_LOOKUP; 0 = never)
    // the window's SetProperty calls of properties no program writes, and those properties: they
    // bound a tile's standalone events (nfk_execute)
    int64_t sa_calls = 0;
    uint64_t sa_pids[2] = {0, 0};
    // GetProperty* (nfk_get_props): device values read since the last frame, and the queued
    // SetProperty chain of each (object, property): ov_last[key] = its last xop, ov_prev links back
    std::unordered_map<uint64_t, uint64_t> dcache;
    std::unordered_map<uint64_t, uint32_t> ov_last;
    std::vector<uint32_t> ov_prev;
    uint64_t* gat = nullptr;             // device scratch of gathered reads
    size_t gat_cap = 0;
    uint32_t* moff_tmp = nullptr;        // device scratch of nfk_read_fanout's counted offsets
    size_t moff_tmp_cap = 0;
    // host worker threads for large call batches (NFGPU_HOST_THREADS, default 1 = none)
    std::unique_ptr<HostPool> pool;
    size_t par_calls = 16384;  // batches from this size on use the pool (NFGPU_PAR_CALLS: tests)
    // queued SetRecordInt / SetRecordFloat calls (obj: object index until nfk_execute resolves it;
    // rrc = rec << 16 | row << 8 | col) and their folding scratch
    // op 0 SetRecord*, 1 AddRow (row 0xFF: -1; aux = its values' index in rvals, or 0xFFFFFFFF),
    // 2 Remove, 3 ClearRecord
    struct RSOp { uint32_t obj, rrc; uint64_t bits; uint32_t op, aux; };
    std::vector<RSOp> rsq;
    std::vector<uint64_t> rvals;  // AddRow values, NFK_MAX_REC_COLS words each
    std::unordered_map<uint64_t, std::vector<uint32_t>> rq_index;  // (object << 3 | record) -> its queued calls
    std::unordered_map<uint64_t, uint64_t> ucache;  // (object << 3 | record) -> used mask read this window
    std::vector<uint64_t> rowpairs;  // (slot << 3 | record) with row operations this window (nfk_execute)
    void* rl_buf = nullptr;          // rs_has / rl_cnt / rl_ev
    size_t rl_cap = 0;
    std::vector<uint64_t> rpk, rpk_t;
    std::vector<uint32_t> rs_slot_h, rs_rrc_h, rs_first_h, rss_slot_h, rss_g0_h;
    void* rs_buf = nullptr;   // rs_old / rs_new
    size_t rs_cap = 0;
    void* rss_buf = nullptr;  // rss_ev / rss_msg / rss_pos / rss_pmsg
    size_t rss_cap = 0;
    // the device fold of the schedule calls (hf_buf: keys, counts, pre / post entries, added flags);
    // the last pass's post entries (hf_post, count at *hf_npost) stay for nfk_read_added
    void* hf_buf = nullptr;
    size_t hf_cap = 0;
    bool hf_pending = false;
    size_t hf_max = 0;         // post entries' room (2 per call)
    const uint32_t* hf_npost = nullptr;
    const uint32_t* hf_pslot = nullptr;
    const uint32_t* hf_pkind = nullptr;
    const uint32_t* hf_pop = nullptr;
    const uint8_t* hf_added = nullptr;
    void* xs_buf = nullptr;  // x_old / x_new (/ x_old_h / x_new_h)
    size_t xs_cap = 0;
    struct HOp { int32_t code; uint32_t slot, kind; float interval; int32_t count; int64_t time; };
    std::vector<HOp> hops;

    // pinned upload arena + device staging
    void* pin = nullptr;
    size_t pin_cap = 0;
    hipEvent_t pin_done = nullptr;
    bool pin_pending = false;
    void* stage = nullptr;
    size_t stage_cap = 0;

    // k_tick specialised to this world's schema (nfgpu_jit.hpp); null: the generic instantiations
    hipFunction_t jit_fn = nullptr;
    hipFunction_t jit_chain_fn = nullptr;  // k_chain_u on the same policy
    int jit_waves = 0, jit_u = 0;
    bool jit_lb = false;  // the specialisation keeps k_tick's in-kernel ranks (a world of <= kLbMaxTiles tiles)
    std::string jit_msg = "not compiled";

    int32_t ticks = 0;
    uint32_t last_tcap = 0;  // Dev::msg_tcap of the last launched frame
    uint32_t last_rtcap = 0; // Dev::msg_rtcap of the last launched frame (0: records not fused)
    uint32_t lb_epoch = 0;       // k_tick's own ranks: the last launch's epoch (Dev::lb_epoch)
    bool scan_pending = false;  // the last frame's dense ranks (k_scan_tiles) are built on first read
    Dev scan_dev;               // ... with that frame's Dev
    int64_t last_rec_msgs = 0;  // record-tile messages of the last summarised frame (capacity hint)
    // the last frame ran k_fanout: its error word is copied to err_pin (event err_done) and
    // checked before anything reads or replaces that frame's fan-out (check_fanout)
    bool fan_unchecked = false;
    unsigned* err_pin = nullptr;
    // pinned landing area of the frame's control block and byte tallies (read_ctrl / read_ctrl_tallies:
    // asynchronous copies behind the frame and one stream synchronisation, not two synchronous copies)
    char* ctrl_pin = nullptr;
    hipEvent_t err_done = nullptr;
    int32_t max_np = 0;    // most players in one scene group (an upper bound between full re-layouts)
    // per-Set chains of the watched properties (nfk_watch_props, k_chain): the watch mask, the log
    // of the last nfk_execute (ChainEnt records, its count on the device) and whether that frame ran it
    // (k_chain stages it per tile: chain_tcap records per tile, chain_cnt_d the tiles' counts; the
    // read-back's device scratch and pinned copy are the chain's own, so nfk_read_frame's stay valid)
    uint64_t chain_watch[2] = {0, 0};
    ChainEnt* chain_d = nullptr;
    uint32_t* chain_cnt_d = nullptr;
    size_t chain_cap = 0;  // records
    uint32_t chain_tcap = 0;
    int32_t chain_tiles = 0;
    bool chain_ran = false;
    void* chain_scr = nullptr;
    size_t chain_scap = 0;
    char* chain_pin = nullptr;
    size_t chain_pcap = 0;

    bool profiling = false;
    std::vector<PendingTiming> pend;
    std::vector<hipEvent_t> evpool;
    double kt_ms[KT_N] = {};
    int64_t kt_n[KT_N] = {};
    int64_t kt_bytes[KT_N] = {};
    uint64_t last_bytes[3] = {0, 0, 0};
};

// the device error bits in the host-mapped words (dev_error: one word per bit)
inline unsigned err_host_bits(const World* w) {
    unsigned e = 0;
    for (int i = 0; i < kErrHostWords; i++) e |= ((volatile const unsigned*)w->err_host)[i] ? 1u << i : 0u;
    return e;
}
inline void clear_err_host(World* w) {
    for (int i = 0; i < kErrHostWords; i++) ((volatile unsigned*)w->err_host)[i] = 0;
}

constexpr uint32_t kNoKind = 0xFFFFFFFFu;  // HOp::kind of a RemoveSchedule(self, name) with no device program
// a queued SetProperty of a property no program writes: a standalone event (see nfk_execute)
inline void count_standalone(World* w, uint32_t pid) {
    if (w->tab.w_slot[pid] == kNoU) {
        w->sa_calls++;
        w->sa_pids[pid >> 6] |= 1ull << (pid & 63);
    }
}
static_assert(sizeof(World::HOp) == sizeof(HCall) && offsetof(World::HOp, time) == offsetof(HCall, time),
              "k_hkeys / k_hfold read the queued schedule calls as uploaded");
static_assert(sizeof(World::XOp) == sizeof(XCall) && offsetof(World::XOp, bits) == offsetof(XCall, bits),
              "k_xkeys reads the queued SetProperty calls as uploaded");

// word of property pid (its data half for an object property) in an entity row
inline int64_t prop_word(const World* w, int32_t pid) {
    return pid < w->n_if ? pid : w->n_if + 2 * (int64_t)(pid - w->n_if);
}

// Every failure of nfk_execute after the window's membership changes are applied drops the
// window's remaining queued calls (SetProperty / SetObject, SetRecord, schedule calls) with it: the
// membership part cannot be undone, so none of the window's calls is applied out of its order in
// a later frame.  (A failure before that keeps every queue.)
int drop_window(World* w, int r) {
    w->xq_n = 0;
    w->xops.clear();
    w->xops_h.clear();
    w->sa_calls = 0;
    w->sa_pids[0] = w->sa_pids[1] = 0;
    w->hops.clear();
    w->rsq.clear();
    w->rvals.clear();
    w->rq_index.clear();
    w->ucache.clear();
    w->dcache.clear();
    w->ov_last.clear();
    w->ov_prev.clear();
    return r;
}

int alloc_track(World* w, void** p, size_t bytes) {
    *p = nullptr;
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess) return fail(NFK_ERR_HIP, std::string("hipMalloc ") + std::to_string(bytes) + ": " + hipGetErrorString(e));
    w->allocs.push_back(*p);
    return NFK_OK;
}
#define ALLOC(ptr, bytes)                                                    \
    do {                                                                     \
        void* _p;                                                            \
        int _r = alloc_track(w, &_p, (size_t)(bytes));                       \
        if (_r) return _r;                                                   \
        ptr = reinterpret_cast<decltype(ptr)>(_p);                           \
    } while (0)

hipEvent_t get_event(World* w) {
    if (!w->evpool.empty()) {
        hipEvent_t e = w->evpool.back();
        w->evpool.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int drain_timings(World* w) {
    for (auto& p : w->pend) {
        HIPCHK(hipEventSynchronize(p.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        w->kt_ms[p.kind] += ms;
        w->kt_n[p.kind] += 1;
        w->evpool.push_back(p.a);
        w->evpool.push_back(p.b);
    }
    w->pend.clear();
    return NFK_OK;
}

struct TimeScope {
    World* w;
    int kind;
    hipEvent_t a = nullptr, b = nullptr;
    TimeScope(World* ww, int k) : w(ww), kind(k) {
        if (w->profiling) {
            a = get_event(w);
            b = get_event(w);
            if (a) (void)hipEventRecord(a, w->stream);
        }
    }
    ~TimeScope() {
        if (w->profiling && a && b) {
            (void)hipEventRecord(b, w->stream);
            w->pend.push_back({kind, a, b, 0});
        }
    }
};

// reserve a pinned host arena (waits for the previous upload to finish reading it)
int pin_reserve(World* w, size_t bytes) {
    if (w->pin_pending) {
        HIPCHK(hipEventSynchronize(w->pin_done));
        w->pin_pending = false;
    }
    if (bytes > w->pin_cap) {
        if (w->pin) HIPCHK(hipHostFree(w->pin));
        w->pin = nullptr;
        size_t cap = std::max(bytes, w->pin_cap * 2);
        w->pin_cap = 0;  // (until the new buffer exists)
        HIPCHK(hipHostMalloc(&w->pin, cap, hipHostMallocDefault));
        w->pin_cap = cap;
    }
    if (bytes > w->stage_cap) {
        // kernels of earlier frames may still read the old staging buffer
        HIPCHK(hipStreamSynchronize(w->stream));
        if (w->stage) HIPCHK(hipFree(w->stage));
        w->stage = nullptr;
        size_t cap = std::max(bytes, w->stage_cap * 2);
        w->stage_cap = 0;  // (until the new buffer exists)
        HIPCHK(hipMalloc(&w->stage, cap));
        w->stage_cap = cap;
    }
    return NFK_OK;
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

int lookup(World* w, int64_t h, int64_t d, int32_t* obj) {
    *obj = w->obj_of.find(h, d);
    if (*obj < 0) return fail(NFK_ERR_NOTFOUND, "no object " + std::to_string(h) + "-" + std::to_string(d));
    return NFK_OK;
}

// accumulated algorithmic-byte tallies of k_tick, k_records, k_fanout
constexpr size_t kTallyBytes = (size_t)3 * kTallyN * 8 * 8;  // (the tallies' 64-byte spread slots)
constexpr size_t kCtrlPinTally = (sizeof(Ctrl) + 255) & ~(size_t)255;
constexpr size_t kCtrlPinBytes = kCtrlPinTally + kTallyBytes;
int read_tallies(World* w, uint64_t out[3]) {
    std::vector<unsigned long long> t((size_t)3 * kTallyN * 8);
    HIPCHK(hipMemcpy(t.data(), w->d.tally, t.size() * 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < 3; k++) {
        out[k] = 0;
        for (int i = 0; i < kTallyN; i++) out[k] += t[((size_t)k * kTallyN + i) * 8];
    }
    return NFK_OK;
}

// dense scratch for readback, at least `bytes`
int dense_reserve(World* w, size_t bytes) {
    if (bytes <= w->dense_cap) return NFK_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (w->dense) HIPCHK(hipFree(w->dense));
    w->dense = nullptr;
    HIPCHK(hipMalloc(&w->dense, bytes));
    w->dense_cap = bytes;
    return NFK_OK;
}

// tile-staged src -> host array in global order (n entries)
template <typename T>
int gather_tiles(World* w, const T* src, const uint32_t* base, int n_tiles, int tcap, size_t n, T* host) {
    if (n == 0 || n_tiles == 0) return NFK_OK;
    int r = dense_reserve(w, n * sizeof(T));
    if (r) return r;
    const unsigned nb = (unsigned)std::min(n_tiles, 4096);
    hipLaunchKernelGGL(k_compact<T>, dim3(nb), dim3(kTPB), 0, w->stream, src, (T*)w->dense, base, n_tiles, tcap);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(host, w->dense, n * sizeof(T), hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    return NFK_OK;
}
#define GATHER(...)                    \
    do {                               \
        int _r = gather_tiles(__VA_ARGS__); \
        if (_r) return _r;             \
    } while (0)

// ---------------- membership layout ----------------
// Slots are grouped in scene-group segments in (scene, group) order.  Inside a segment the live
// entities sit in NFGUID order, followed by slack slots (fan_desc = kDeadDesc) that absorb
// arrivals without moving other segments.  NFCSceneGroupInfo keeps its member maps as
// std::map<NFGUID, ...>, so slot order is both the reference's dirty-sync order and
// GetBroadCastObject's recipient order (AOI:572, KM:1270-1294).
bool guid_less(const World* w, int32_t a, int32_t b) {
    const World::Guid x = w->guid[a], y = w->guid[b];
    return x.h != y.h ? x.h < y.h : x.d < y.d;
}

// (scene, group) as one word whose unsigned order is the pair's signed order
uint64_t seg_key_of(int32_t scene, int32_t group) {
    return ((uint64_t)((uint32_t)scene ^ 0x80000000u) << 32) | ((uint32_t)group ^ 0x80000000u);
}

// the segment of (scene, group), or -1
int32_t find_seg(const World* w, int32_t scene, int32_t group) {
    const uint64_t k = seg_key_of(scene, group);
    const auto it = std::lower_bound(w->seg_key.begin(), w->seg_key.end(), k);
    return it != w->seg_key.end() && *it == k ? (int32_t)(it - w->seg_key.begin()) : -1;
}

void index_segs(World* w) {
    w->seg_key.resize(w->segs.size());
    for (size_t g = 0; g < w->segs.size(); g++) w->seg_key[g] = seg_key_of(w->segs[g].scene, w->segs[g].group);
}

int32_t seg_slack(int32_t slack, int32_t len) {
    return slack <= 0 ? 0 : std::max<int32_t>(2, (int32_t)(((int64_t)len * slack + 255) / 256));
}

// segments of every live object with `slack` slots per 256; returns the slot total
int64_t plan_segments(World* w, int32_t slack, std::vector<World::Seg>& segs) {
    std::vector<int32_t> objs;
    for (int32_t o = 0; o < w->n_obj; o++)
        if (w->alive[o]) objs.push_back(o);
    std::sort(objs.begin(), objs.end(), [w](int32_t a, int32_t b) {
        if (w->scene[a] != w->scene[b]) return w->scene[a] < w->scene[b];
        if (w->group[a] != w->group[b]) return w->group[a] < w->group[b];
        return guid_less(w, a, b);
    });
    segs.clear();
    int64_t base = 0;
    for (size_t i = 0; i < objs.size();) {
        size_t j = i;
        const int32_t o = objs[i];
        while (j < objs.size() && w->scene[objs[j]] == w->scene[o] && w->group[objs[j]] == w->group[o]) j++;
        World::Seg g;
        g.scene = w->scene[o];
        g.group = w->group[o];
        g.base = (int32_t)std::min<int64_t>(base, INT32_MAX);
        g.objs.assign(objs.begin() + i, objs.begin() + j);
        g.keys.resize(g.objs.size());
        for (size_t k = 0; k < g.objs.size(); k++) g.keys[k] = w->guid[g.objs[k]];
        g.cap = (int32_t)g.objs.size() + seg_slack(slack, (int32_t)g.objs.size());
        base += g.cap;
        segs.push_back(std::move(g));
        i = j;
    }
    return base;
}

// per-slot metadata of one segment: slot -> object, fan-out descriptor, and the player run
// pl_slot[base, base + players) in NFGUID order (NFCSceneGroupInfo::mxPlayerList)
struct MetaLists {
    std::vector<int32_t> slot, obj, pl;
    std::vector<uint64_t> desc;
};

int seg_meta(World* w, World::Seg& g, MetaLists& m) {
    int32_t np = 0;
    for (int32_t o : g.objs) np += w->isplayer[o] ? 1 : 0;
    if (np > 0x3FFF) return fail(NFK_ERR_ARG, "more than 16383 players in one scene group");
    g.np = np;
    w->max_np = std::max(w->max_np, np);
    const size_t at = m.slot.size();
    int32_t rank = 0;
    for (int32_t i = 0; i < g.cap; i++) {
        m.slot.push_back(g.base + i);
        m.pl.push_back(0);
        if (i < (int32_t)g.objs.size()) {
            const int32_t o = g.objs[i];
            const bool pl = w->isplayer[o];
            m.obj.push_back(o);
            m.desc.push_back((uint64_t)(uint32_t)g.base | ((uint64_t)np << 32) |
                             ((uint64_t)(pl ? rank + 1 : 0) << 46) | ((uint64_t)w->cls[o] << 60));
            if (pl) m.pl[at + rank++] = g.base + i;
        } else {
            m.obj.push_back(-1);
            m.desc.push_back(kDeadDesc);
        }
    }
    return NFK_OK;
}

void set_tiles(Dev& d, int32_t n_slots) {
    d.N = n_slots;
    d.n_tiles = (n_slots + kTile - 1) / kTile;
    d.n_rtiles = (n_slots + kRTile - 1) / kRTile;
}

// grow a device buffer (contents dropped; callers only grow between uses)
int dev_reserve(World* w, void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return NFK_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    const size_t c = std::max(bytes, *cap + *cap / 2);
    *cap = 0;  // (until the new buffer exists)
    HIPCHK(hipMalloc(p, c));
    *cap = c;
    return NFK_OK;
}

// stable LSD radix sort of packed words key << shift | index on the key's low `key_bits` bits
// (11-bit digits, a digit that every key shares is skipped): one array, 8 bytes per element and
// pass instead of a key and a value array
void radix_sort_packed(std::vector<uint64_t>& a, std::vector<uint64_t>& t, int shift, int key_bits) {
    const size_t n = a.size();
    if (n < 2) return;
    t.resize(n);
    uint32_t cnt[2048];
    for (int sh = shift; sh < shift + key_bits; sh += 11) {
        memset(cnt, 0, sizeof cnt);
        for (size_t i = 0; i < n; i++) cnt[(a[i] >> sh) & 2047]++;
        if (cnt[(a[0] >> sh) & 2047] == n) continue;
        uint32_t acc = 0;
        for (int b = 0; b < 2048; b++) {
            const uint32_t c = cnt[b];
            cnt[b] = acc;
            acc += c;
        }
        for (size_t i = 0; i < n; i++) t[cnt[(a[i] >> sh) & 2047]++] = a[i];
        a.swap(t);
    }
}
int bits_for(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 1; }


// look_pin / look_dev (the device lookups' pinned and device staging) hold at least `bytes`
int look_reserve(World* w, size_t bytes) {
    if (bytes > w->look_pin_cap) {
        if (w->look_pin) HIPCHK(hipHostFree(w->look_pin));
        w->look_pin = nullptr;
        w->look_pin_cap = 0;
        HIPCHK(hipHostMalloc((void**)&w->look_pin, bytes + bytes / 2, hipHostMallocDefault));
        w->look_pin_cap = bytes + bytes / 2;
    }
    if (bytes > w->look_dev_cap) {
        if (w->look_dev) HIPCHK(hipFree(w->look_dev));
        w->look_dev = nullptr;
        w->look_dev_cap = 0;
        HIPCHK(hipMalloc(&w->look_dev, bytes + bytes / 2));
        w->look_dev_cap = bytes + bytes / 2;
    }
    return NFK_OK;
}

// Brings the device mirror of obj_of up to date on look_stream (the whole table after a rebuild,
// else the entries written since the last batch) and reserves the staging: the mirror's patch takes
// [0, *used) of look_pin / look_dev, the caller's batch (batch_bytes) follows.
int guid_mirror_update(World* w, size_t batch_bytes, size_t* used) {
    if (!w->look_stream) HIPCHK(hipStreamCreateWithFlags(&w->look_stream, hipStreamNonBlocking));
    using E = GuidMap::E;
    static_assert(sizeof(E) == sizeof(GuidEntry) && offsetof(E, v) == offsetof(GuidEntry, v), "mirror layout");
    const size_t cap = w->obj_of.capacity();
    const size_t tbytes = cap * sizeof(E);
    bool full = w->obj_of.take_rebuilt() || !w->guid_synced || w->guid_dmask != cap - 1;
    size_t np = full ? 0 : w->guid_log.size();
    if (np > cap / 8) {  // (many writes since: the whole table is the smaller upload)
        full = true;
        np = 0;
    }
    const size_t o_pi = 0, o_pe = align16(np * 4), u = align16(o_pe + np * sizeof(E));
    if (int r = look_reserve(w, u + batch_bytes)) return r;
    char* P = w->look_pin;
    char* D = (char*)w->look_dev;
    if (full) {
        if (tbytes > w->guid_dcap) {
            if (w->guid_d) HIPCHK(hipFree(w->guid_d));
            w->guid_d = nullptr;
            w->guid_dcap = 0;
            HIPCHK(hipMalloc(&w->guid_d, tbytes));
            w->guid_dcap = tbytes;
        }
        HIPCHK(hipMemcpyAsync(w->guid_d, w->obj_of.entries(), tbytes, hipMemcpyHostToDevice, w->look_stream));
        w->guid_dmask = cap - 1;
        w->guid_synced = true;
    } else if (np) {
        const E* t = w->obj_of.entries();
        uint32_t* pi = (uint32_t*)(P + o_pi);
        E* pe = (E*)(P + o_pe);
        for (size_t i = 0; i < np; i++) {  // (an entry logged twice is written twice with its final value)
            pi[i] = w->guid_log[i];
            pe[i] = t[w->guid_log[i]];
        }
        HIPCHK(hipMemcpyAsync(D, P, u, hipMemcpyHostToDevice, w->look_stream));
        hipLaunchKernelGGL(k_guid_patch, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, w->look_stream,
                           (GuidEntry*)w->guid_d, (const uint32_t*)(D + o_pi), (const GuidEntry*)(D + o_pe), (int32_t)np);
        HIPCHK(hipGetLastError());
    }
    w->guid_log.clear();
    *used = u;
    return NFK_OK;
}

// n lookups of a large batch on the device mirror of obj_of: one H2D copy of the GUIDs,
// k_guid_find, one D2H copy of the object indices
static bool trace_calls() {
    static const bool t = getenv("NFGPU_TRACE_CALLS") != nullptr;  // call batches' host phases to stderr
    return t;
}
static double ms_since(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
}

int find_many_dev(World* w, int32_t n, const int64_t* gh, const int64_t* gd, int32_t* out) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const size_t cap = w->obj_of.capacity();
    if (cap == 0 || n <= 0) {
        for (int32_t i = 0; i < n; i++) out[i] = -1;
        return NFK_OK;
    }
    const size_t o_q = 0, o_r = align16((size_t)n * 16), tot = align16(o_r + (size_t)n * 4);
    size_t u = 0;
    if (int r = guid_mirror_update(w, tot, &u)) return r;
    char* P = w->look_pin + u;
    char* D = (char*)w->look_dev + u;
    memcpy(P + o_q, gh, (size_t)n * 8);
    memcpy(P + o_q + (size_t)n * 8, gd, (size_t)n * 8);
    const auto t1 = clk::now();
    HIPCHK(hipMemcpyAsync(D, P, o_r, hipMemcpyHostToDevice, w->look_stream));
    hipLaunchKernelGGL(k_guid_find, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, w->look_stream,
                       (const GuidEntry*)w->guid_d, (uint64_t)(cap - 1), (const int64_t*)(D + o_q), n,
                       (int32_t*)(D + o_r));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(P + o_r, D + o_r, (size_t)n * 4, hipMemcpyDeviceToHost, w->look_stream));
    const auto t2 = clk::now();
    HIPCHK(hipStreamSynchronize(w->look_stream));
    const auto t3 = clk::now();
    memcpy(out, P + o_r, (size_t)n * 4);
    if (trace_calls())
        fprintf(stderr, "find_many_dev n=%d: mirror+stage %.3f ms, enqueue %.3f ms, wait %.3f ms, copy-out %.3f ms\n", n,
                ms_since(t0, t1), ms_since(t1, t2), ms_since(t2, t3), ms_since(t3, clk::now()));
    return NFK_OK;
}

// the window's device queue of SetProperty calls (xq[xq_b]) holds at least `recs` records; grown
// on look_stream with its first xq_n records copied (the frame that last read the buffer is done:
// look_stream waited for xq_ev at the window's first device batch)
int xq_reserve(World* w, size_t recs) {
    const int b = w->xq_b;
    if (recs <= w->xq_cap[b]) return NFK_OK;
    const size_t c = std::max<size_t>({recs, w->xq_cap[b] + w->xq_cap[b] / 2, 65536});
    void* nb = nullptr;
    HIPCHK(hipMalloc(&nb, c * sizeof(World::XOp)));
    if (w->xq_n) HIPCHK(hipMemcpyAsync(nb, w->xq[b], w->xq_n * sizeof(World::XOp), hipMemcpyDeviceToDevice, w->look_stream));
    HIPCHK(hipStreamSynchronize(w->look_stream));
    if (w->xq[b]) HIPCHK(hipFree(w->xq[b]));
    w->xq[b] = nb;
    w->xq_cap[b] = c;
    return NFK_OK;
}

// the same at nfk_execute, on the world's stream (the host calls queued after the last device batch
// are appended there): a new buffer gets the device queue's calls, the old one is freed after
int xq_reserve_exec(World* w, size_t recs) {
    const int b = w->xq_b;
    if (recs <= w->xq_cap[b]) return NFK_OK;
    const size_t c = std::max<size_t>({recs, w->xq_cap[b] + w->xq_cap[b] / 2, 65536});
    void* nb = nullptr;
    HIPCHK(hipMalloc(&nb, c * sizeof(World::XOp)));
    HIPCHK(hipMemcpyAsync(nb, w->xq[b], w->xq_n * sizeof(World::XOp), hipMemcpyDeviceToDevice, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    HIPCHK(hipFree(w->xq[b]));
    w->xq[b] = nb;
    w->xq_cap[b] = c;
    return NFK_OK;
}

// A large batch of SetProperty* calls queued on the device (worlds without object properties):
// the lookups run on the device mirror and each call is written straight into the window's device
// queue (k_guid_queue), so the host touches the batch once, to stage it.  The host calls queued
// since the last device batch go in front of it (call order); a GUID that is no object rejects the
// whole batch, as nfk_set_props does.
int set_props_dev(World* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, const uint64_t* bits) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    // the ids checked and the standalone calls counted without a branch per call (a batch's
    // properties follow no order a branch predictor learns: 3.4 ns per call with the branches on
    // the GPU boxes' hosts): one bit per property without a writable slot
    uint64_t nos[2] = {0, 0};
    for (int p = 0; p < w->n_if; p++)
        if (w->tab.w_slot[p] == kNoU) nos[p >> 6] |= 1ull << (p & 63);
    const uint32_t nif = (uint32_t)w->n_if;
    uint32_t bad = 0;
    int64_t sa = 0;
    uint64_t u0 = 0, u1 = 0;
    for (int32_t i = 0; i < n; i++) {
        const uint32_t p = (uint32_t)pid[i];
        bad |= (uint32_t)(p >= nif);
        const uint64_t bit = 1ull << (p & 63);
        const uint64_t hi = 0 - (uint64_t)((p >> 6) & 1);  // all ones for ids 64..127
        sa += (((nos[0] & ~hi) | (nos[1] & hi)) & bit) != 0;
        u0 |= bit & ~hi;
        u1 |= bit & hi;
    }
    if (bad)
        for (int32_t i = 0; i < n; i++)
            if (pid[i] < 0 || pid[i] >= w->n_if)
                return fail(NFK_ERR_ARG, pid[i] >= w->n_if && pid[i] < w->n_prop ? "object property: use nfk_set_objects"
                                                                                  : "bad property id");
    const uint64_t sp[2] = {u0 & nos[0], u1 & nos[1]};
    const auto t1 = clk::now();
    if (!w->look_stream) HIPCHK(hipStreamCreateWithFlags(&w->look_stream, hipStreamNonBlocking));
    const int b = w->xq_b;
    if (w->xq_n == 0 && w->xq_ev_set[b]) HIPCHK(hipStreamWaitEvent(w->look_stream, w->xq_ev[b], 0));
    const size_t tail = w->xops.size();
    if (int r = xq_reserve(w, w->xq_n + tail + (size_t)n)) return r;
    const size_t o_t = 0, o_b = align16(tail * sizeof(World::XOp)), o_p = align16(o_b + (size_t)n * 24),
                 o_m = align16(o_p + (size_t)n * 4), tot = o_m + 16;
    size_t u = 0;
    if (int r = guid_mirror_update(w, tot, &u)) return r;
    char* P = w->look_pin + u;
    char* D = (char*)w->look_dev + u;
    if (tail) memcpy(P + o_t, w->xops.data(), tail * sizeof(World::XOp));
    memcpy(P + o_b, gh, (size_t)n * 8);
    memcpy(P + o_b + (size_t)n * 8, gd, (size_t)n * 8);
    memcpy(P + o_b + (size_t)n * 16, bits, (size_t)n * 8);
    memcpy(P + o_p, pid, (size_t)n * 4);
    *(int32_t*)(P + o_m) = INT32_MAX;
    const auto t2 = clk::now();
    HIPCHK(hipMemcpyAsync(D, P, tot, hipMemcpyHostToDevice, w->look_stream));
    World::XOp* q = (World::XOp*)w->xq[b] + w->xq_n;
    if (tail) HIPCHK(hipMemcpyAsync(q, D + o_t, tail * sizeof(World::XOp), hipMemcpyDeviceToDevice, w->look_stream));
    hipLaunchKernelGGL(k_guid_queue, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, w->look_stream,
                       (const GuidEntry*)w->guid_d, (uint64_t)(w->obj_of.capacity() - 1), (const int64_t*)(D + o_b),
                       (const int32_t*)(D + o_p), n, (XCall*)(q + tail), (int32_t*)(D + o_m));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(P + o_m, D + o_m, 4, hipMemcpyDeviceToHost, w->look_stream));
    const auto t3 = clk::now();
    HIPCHK(hipStreamSynchronize(w->look_stream));
    if (trace_calls())
        fprintf(stderr, "set_props_dev n=%d: validate %.3f ms, mirror+reserve+stage %.3f ms, enqueue %.3f ms, wait %.3f ms\n",
                n, ms_since(t0, t1), ms_since(t1, t2), ms_since(t2, t3), ms_since(t3, clk::now()));
    const int32_t miss = *(const int32_t*)(P + o_m);
    if (miss >= 0 && miss < n)  // NFCKernelModule logs "There is no object" and returns false (KM:331)
        return fail(NFK_ERR_NOTFOUND, "no object " + std::to_string(gh[miss]) + "-" + std::to_string(gd[miss]));
    w->xq_n += tail + (size_t)n;
    w->xops.clear();
    w->ov_last.clear();  // (the overlay index is rebuilt from the whole queue at the next read)
    w->ov_prev.clear();
    w->sa_calls += sa;
    w->sa_pids[0] |= sp[0];
    w->sa_pids[1] |= sp[1];
    return NFK_OK;
}

// the window's device queue back in the host xops, in front of the calls queued after it (a read
// of queued values — GetProperty* — needs them all on the host)
int pull_device_queue(World* w) {
    if (!w->xq_n) return NFK_OK;
    std::vector<World::XOp> dq(w->xq_n);
    HIPCHK(hipMemcpy(dq.data(), w->xq[w->xq_b], w->xq_n * sizeof(World::XOp), hipMemcpyDeviceToHost));
    w->xops.insert(w->xops.begin(), dq.begin(), dq.end());
    w->xq_n = 0;
    w->ov_last.clear();
    w->ov_prev.clear();
    return NFK_OK;
}

// A batch's lookups: on the device from dev_look_min calls on, else GuidMap::find_many (split
// over the host pool for a large batch when the pool has workers)
int find_many_par(World* w, int32_t n, const int64_t* gh, const int64_t* gd, int32_t* out) {
    if (w->dev_look_min && (size_t)n >= w->dev_look_min) return find_many_dev(w, n, gh, gd, out);
    if (w->guid_log.size() > w->obj_of.capacity() / 8) {  // (the mirror is rewritten at its next use)
        w->guid_log.clear();
        w->guid_synced = false;
    }
    if ((size_t)n < w->par_calls || w->pool->threads() < 2) {
        w->obj_of.find_many(n, gh, gd, out);
        return NFK_OK;
    }
    const int P = w->pool->threads();
    w->pool->run(P, [&](int c) {
        const int32_t a = (int32_t)((int64_t)n * c / P), b = (int32_t)((int64_t)n * (c + 1) / P);
        w->obj_of.find_many(b - a, gh + a, gd + a, out + a);
    });
    return NFK_OK;
}


// replace a tracked device allocation by a bigger one (contents dropped)
int regrow(World* w, void** p, size_t bytes) {
    if (*p) {
        HIPCHK(hipFree(*p));
        w->allocs.erase(std::remove(w->allocs.begin(), w->allocs.end(), *p), w->allocs.end());
        *p = nullptr;
    }
    return alloc_track(w, p, bytes);
}

// the property-event tiles with room for `per_tile` events each (a frame with many standalone
// SetProperty groups in one tile); the previous frame's events are dropped
int grow_event_tiles(World* w, int64_t per_tile) {
    Dev& d = w->d;
    const int64_t tcap = (per_tile + kTile - 1) / kTile * kTile;
    if (tcap > 0xFFFF) return fail(NFK_ERR_CAPACITY, "more than 65535 property events in one 256-slot tile");
    HIPCHK(hipStreamSynchronize(w->stream));
    const size_t n = (size_t)(d.cap / kTile) * (size_t)tcap;
    int r;
    if ((r = regrow(w, (void**)&d.ev_slot, n * 4)) || (r = regrow(w, (void**)&d.ev_pid, n * 4)) ||
        (r = regrow(w, (void**)&d.ev_old, n * 8)) || (r = regrow(w, (void**)&d.ev_new, n * 8)) ||
        (r = regrow(w, (void**)&d.ev_moff, n * 4)) ||
        (d.n_obj && ((r = regrow(w, (void**)&d.ev_old_h, n * 8)) || (r = regrow(w, (void**)&d.ev_new_h, n * 8))))) {
        d.ev_tcap = 0;
        return r;
    }
    d.ev_tcap = (int32_t)tcap;
    w->scan_pending = false;
    return NFK_OK;
}

// The programs' working set: program destinations -> writable U slots [0, n_w) and the operands
// programs only read -> slots [n_w, n_u), each group in property-id order; the tables name
// read-only operand r as 0x80 | r.  Fills the kinds' U-slot tables (opu, umask, opx, w_slot);
// false when the set does not fit k_tick's register slots (k_tick_touch runs instead).
// the record-event tiles grown for a frame whose SetRecord groups add events beside the record
// programs' (contents dropped: called before the frame writes them)
int grow_rec_tiles(World* w, int64_t per_tile) {
    Dev& d = w->d;
    const int64_t tcap = (per_tile + 63) / 64 * 64;
    if (tcap > INT32_MAX / 2) return fail(NFK_ERR_CAPACITY, "too many record events in one record tile");
    HIPCHK(hipStreamSynchronize(w->stream));
    const size_t n = (size_t)(d.cap / kRTile) * (size_t)tcap;
    int r;
    if ((r = regrow(w, (void**)&d.re_rrc, n * 4)) ||
        (r = regrow(w, (void**)&d.re_old, n * 8)) || (r = regrow(w, (void**)&d.re_new, n * 8)) ||
        (r = regrow(w, (void**)&d.re_moff, n * 4))) {
        d.re_tcap = 0;
        return r;
    }
    d.re_tcap = (int32_t)tcap;
    w->scan_pending = false;
    return NFK_OK;
}

// the property ops (a program's Get + Set on a property column; record ops run in k_records)
static bool prop_op(int code) {
    return code == NFK_OP_IADD_CLAMP || code == NFK_OP_FLERP || code == NFK_OP_FAFFINE || code == NFK_OP_ISET ||
           code == NFK_OP_FSET;
}

bool build_u_tables(Tables& tab, int NK, std::vector<int>& wp, std::vector<int>& rp) {
    bool u_ok = false;
    {
        std::vector<int> W, R;
        for (int k = 0; k < NK; k++)
            for (int i = 0; i < tab.nops[k]; i++) {
                const nfk_op& op = tab.ops[k][i];
                if (prop_op(op.code)) W.push_back(op.dst);
            }
        std::sort(W.begin(), W.end());
        W.erase(std::unique(W.begin(), W.end()), W.end());
        auto is_w = [&](int64_t p) { return std::binary_search(W.begin(), W.end(), (int)p); };
        for (int k = 0; k < NK; k++)
            for (int i = 0; i < tab.nops[k]; i++) {
                const nfk_op& op = tab.ops[k][i];
                if (op.code == NFK_OP_IADD_CLAMP) {
                    if ((op.flags & NFK_A_PROP) && !is_w(op.a)) R.push_back((int)op.a);
                    if ((op.flags & NFK_LO_PROP) && !is_w(op.b)) R.push_back((int)op.b);
                    if ((op.flags & NFK_HI_PROP) && !is_w(op.c)) R.push_back((int)op.c);
                } else if (op.code == NFK_OP_FLERP && !is_w(op.a)) {
                    R.push_back((int)op.a);
                } else if ((op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) && (op.flags & NFK_A_PROP) && !is_w(op.a)) {
                    R.push_back((int)op.a);
                }
                if ((op.flags & NFK_GUARD) && !is_w(op.guard & 0xFFFF)) R.push_back((int)(op.guard & 0xFFFF));
                if ((op.flags & NFK_GUARD) && (op.guard & NFK_GUARD_PROP) && !is_w(op.guard >> 19))
                    R.push_back((int)(op.guard >> 19));
            }
        std::sort(R.begin(), R.end());
        R.erase(std::unique(R.begin(), R.end()), R.end());
        u_ok = (int)W.size() <= kMaxW && (int)(W.size() + R.size()) <= kMaxU;
        wp.assign(W.begin(), W.end());
        rp.assign(R.begin(), R.end());
        memset(tab.w_slot, kNoU, sizeof tab.w_slot);
        for (size_t i = 0; i < W.size() && i < (size_t)kMaxW; i++) tab.w_slot[W[i]] = (uint8_t)i;
        auto slot = [&](int64_t p) -> uint8_t {
            auto it = std::lower_bound(W.begin(), W.end(), (int)p);
            if (it != W.end() && *it == p) return (uint8_t)(it - W.begin());
            it = std::lower_bound(R.begin(), R.end(), (int)p);
            return (uint8_t)(0x80 | (it - R.begin()));
        };
        for (int k = 0; k < NK && u_ok; k++) {
            tab.umask[k] = 0;
            for (int i = 0; i < tab.nops[k]; i++) {
                const nfk_op& op = tab.ops[k][i];
                uint8_t* u = tab.opu[k][i];
                u[0] = u[1] = u[2] = u[3] = kNoU;
                if (op.code == NFK_OP_IADD_CLAMP) {
                    u[0] = slot(op.dst);
                    if (op.flags & NFK_A_PROP) u[1] = slot(op.a);
                    if (op.flags & NFK_LO_PROP) u[2] = slot(op.b);
                    if (op.flags & NFK_HI_PROP) u[3] = slot(op.c);
                } else if (op.code == NFK_OP_FLERP) {
                    u[0] = slot(op.dst);
                    u[1] = slot(op.a);
                } else if (op.code == NFK_OP_FAFFINE) {
                    u[0] = slot(op.dst);
                } else if (op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) {
                    u[0] = slot(op.dst);
                    if (op.flags & NFK_A_PROP) u[1] = slot(op.a);
                }
                tab.opg[k][i] = (op.flags & NFK_GUARD) ? slot(op.guard & 0xFFFF) : kNoU;
                tab.opg2[k][i] = ((op.flags & NFK_GUARD) && (op.guard & NFK_GUARD_PROP)) ? slot(op.guard >> 19) : kNoU;
                for (int q = 0; q < 6; q++) {  // writable bits | read-only bits << 16
                    const uint8_t uq = q < 4 ? u[q] : q == 4 ? tab.opg[k][i] : tab.opg2[k][i];
                    if (uq != kNoU) tab.umask[k] |= (uq & 0x80) ? 1u << (16 + (uq & 0x7F)) : 1u << uq;
                }
                OpX& x = tab.opx[k][i];
                x.cfd = (uint32_t)op.code | ((uint32_t)op.flags << 8) | ((uint32_t)op.dst << 16);
                x.slots = (uint32_t)u[0] | ((uint32_t)u[1] << 8) | ((uint32_t)u[2] << 16) | ((uint32_t)u[3] << 24);
                x.a = op.a;
                x.b = op.b;
                x.c = op.c;
                x.gd = (op.flags & NFK_GUARD) ? 0x80000000u | (((op.guard >> 16) & 3u) << 8) | tab.opg[k][i] : 0u;
                if (tab.opg2[k][i] != kNoU) x.gd |= 0x40000000u | ((uint32_t)tab.opg2[k][i] << 16);
                else if (op.flags & NFK_GUARD) x.gd |= ((op.guard >> 19) & 0x1FFFu) << 16;  // NFK_GUARD_K
            }
        }
    }
    return u_ok;
}

// Dev::u_* from the working set: slot properties, event order and fan-out classes of the
// writable slots (all read by k_tick as scalars); columns only once the world has property memory
void fill_u_dev(Dev& d, const Tables& tab, const std::vector<int>& wp, const std::vector<int>& rp, bool u_ok) {
    const int n_w = (int)wp.size(), n_r = (int)rp.size();
    for (int j = 0; j < kMaxU; j++) d.u_pid[j] = -1;
    d.n_w = d.n_u = 0;
    if (!u_ok) return;
    for (int i = 0; i < n_w; i++) d.u_pid[i] = wp[i];
    for (int i = 0; i < n_r; i++) d.u_pid[n_w + i] = rp[i];
    d.n_w = n_w;
    d.n_u = n_w + n_r;
    for (int i = 0; i < kMaxW; i++) d.u_order[i] = i < n_w ? i : 0;  // (wp is in property-id order)
    for (int j = 0; j < kMaxU; j++) {
        const int p = d.u_pid[j];
        d.u_col[j] = (p < 0 || !d.pmem) ? nullptr : d.pmem + tab.p_off[p];
        d.u_str[j] = p < 0 ? 0 : tab.p_str[p];
    }
    for (int j = 0; j < kMaxW; j++) {
        d.u_lower[j] = 0;
        for (int i = 0; i < n_w && j < n_w; i++)
            if (d.u_pid[i] < d.u_pid[j]) d.u_lower[j] |= 1u << i;
    }
    for (int c = 0; c < NFK_MAX_CLASSES; c++) {
        uint32_t pub = 0, priv = 0;
        for (int j = 0; j < n_w && c != 15; j++) {  // (class 15 marks a free slot)
            const uint8_t f = tab.pflags[c][d.u_pid[j]];
            if (f & NFK_PUBLIC) pub |= 1u << j;
            else if ((f & NFK_PRIVATE) && !(f & NFK_UPLOAD)) priv |= 1u << j;
        }
        d.u_cmask[c] = pub | (priv << 16);
    }
}

void set_working_set(World* w) { fill_u_dev(w->d, w->tab, w->u_wp, w->u_rp, w->u_ok); }

// waves per SIMD k_tick's register budget aims at, by the working set's size
int tick_waves(int n_u, uint32_t ablate) {
    if (ablate & kAblWaves6) return 6;
    if (n_u <= 8) return kWavesU8;
    if (n_u <= 12) return (ablate & kAblWaves8) ? 8 : kWavesU12;
    return 6;
}

// the non-temporal hints the specialised k_tick is built with (A/B: NFGPU_JIT_NT): the schedule
// records / descriptor loads and the fan-out's LDS-window recipient stores stream past the caches
// (config[1]: 90 vs 115 us with none, 102 with the fan-out stores alone; event-array stores
// non-temporal run 160 us; profiles/r07a_ntab.txt).  Not the lane-group recipient stores
// (kNtFanGroupStore: config[3] 377 vs 415 us, config[4] 94 vs 107 us; profiles/r08i_*)
constexpr uint32_t kJitNtDefault = kNtSchedLoad | kNtFanStore;

// Specialised k_tick kernels built in this process, by (device, variant, policy source): a
// schema compiles once however many worlds use it.
std::mutex g_jit_mu;
std::map<std::string, std::pair<hipFunction_t, hipFunction_t>> g_jit;  // (k_tick, k_chain_u)

void build_jit(World* w) {
    w->jit_fn = nullptr;
    w->jit_chain_fn = nullptr;
    const char* env = getenv("NFGPU_JIT");
    if (env && env[0] == '0') {
        w->jit_msg = "disabled (NFGPU_JIT=0)";
        return;
    }
    if (!w->u_ok) {
        w->jit_msg = "working set does not fit k_tick (k_tick_touch runs)";
        return;
    }
    const int u = std::max(w->d.n_u, 1);
    // The specialised kernel gets the register budget of 5 waves per SIMD (round 4: no spills, and
    // the fan-out's LDS window grows with the budget): config[1] 82.7-83.7 vs 83.7-84.1 us at 6
    // (12 VGPRs spilled), 97 at 7, 122 at 8; config[3] 342-344 vs 347-348 us
    // (profiles/r11j_jit_waves_ab.txt; round 2's r02t_ab_waves.txt chose 6 over 7).
    int waves = (w->d.ablate & (kAblWaves6 | kAblWaves8 | kAblWaves5)) ? tick_waves(w->d.n_u, w->d.ablate) : kWavesJit;
    if (const char* ew = getenv("NFGPU_JIT_WAVES")) waves = std::max(1, std::min(8, atoi(ew)));
    const char* es = getenv("NFGPU_JIT_SPEC");
    const bool spec = es && es[0] == '1';  // every program operand loaded with the schedule records
    // non-temporal hints (kNt* bits of nfgpu_tick.hpp); NFGPU_JIT_NT overrides the default
    uint32_t nt = kJitNtDefault;
    if (const char* en = getenv("NFGPU_JIT_NT")) nt = (uint32_t)strtoul(en, nullptr, 0);
    // a world committed with more than kLbMaxTiles tiles does not rank in k_tick: that code is compiled
    // out of its specialisation (NFGPU_JIT_LB=1 keeps it, for A/B).  By the slots in use, not the
    // capacity: the drop-in reserves 1M slots whatever the world (Tutorial3's 10k objects rank in k_tick
    // and skip k_scan_tiles); a world that grows past the bound later ranks by k_scan_tiles (Dev::lb_rank
    // is decided per frame), one that shrinks below it keeps k_scan_tiles with this code compiled out
    bool lb = ((int64_t)std::max(w->d.N, 1) + kTile - 1) / kTile <= kLbMaxTiles;
    if (const char* el = getenv("NFGPU_JIT_LB")) lb = el[0] == '1';
    const std::string src = jit_schema_source(w->tab, w->d, spec, nt, lb);
    int dev = 0;
    (void)hipGetDevice(&dev);
    const std::string key = std::to_string(dev) + "|" + std::to_string(waves) + "|" + std::to_string(u) + "|" + src;
    std::lock_guard<std::mutex> lk(g_jit_mu);
    auto it = g_jit.find(key);
    if (it == g_jit.end()) {
        JitBuild b = jit_compile(src, waves, u);
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr, cfn = nullptr;
        if (!b.ok || hipModuleLoadData(&mod, b.code.data()) != hipSuccess ||
            hipModuleGetFunction(&fn, mod, b.lowered.c_str()) != hipSuccess ||
            hipModuleGetFunction(&cfn, mod, b.lowered_chain.c_str()) != hipSuccess) {
            w->jit_msg = "hipRTC build failed: " + b.log.substr(0, 2000);
            return;
        }
        it = g_jit.emplace(key, std::make_pair(fn, cfn)).first;
    }
    w->jit_fn = it->second.first;
    w->jit_chain_fn = it->second.second;
    w->jit_lb = lb;
    w->jit_waves = waves;
    w->jit_u = u;
    w->jit_msg = jit_kernel_name(waves, u);
}

// w->mhost -> w->mlist, asynchronously on the world's stream (through a pinned double buffer:
// a buffer is refilled only once the copy from it two uploads ago has completed)
int upload_mhost(World* w) {
    int r = dev_reserve(w, &w->mlist, &w->mlist_cap, w->mhost.size() + 16);
    if (r) return r;
    const int s = w->mpin_slot;
    w->mpin_slot ^= 1;
    if (w->mpin_pending[s]) {
        HIPCHK(hipEventSynchronize(w->mpin_done[s]));
        w->mpin_pending[s] = false;
    }
    if (w->mhost.size() > w->mpin_cap[s]) {
        if (w->mpin[s]) HIPCHK(hipHostFree(w->mpin[s]));
        w->mpin[s] = nullptr;
        const size_t c = std::max(w->mhost.size(), 2 * w->mpin_cap[s]);
        w->mpin_cap[s] = 0;  // (until the new buffer exists)
        HIPCHK(hipHostMalloc((void**)&w->mpin[s], c, hipHostMallocDefault));
        w->mpin_cap[s] = c;
    }
    if (w->mhost.empty()) return NFK_OK;
    memcpy(w->mpin[s], w->mhost.data(), w->mhost.size());
    HIPCHK(hipMemcpyAsync(w->mlist, w->mpin[s], w->mhost.size(), hipMemcpyHostToDevice, w->stream));
    HIPCHK(hipEventRecord(w->mpin_done[s], w->stream));
    w->mpin_pending[s] = true;
    return NFK_OK;
}

template <typename T>
size_t stage_list(World* w, const std::vector<T>& v) {
    const size_t off = align16(w->mhost.size());
    w->mhost.resize(off + v.size() * sizeof(T));
    if (!v.empty()) memcpy(w->mhost.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

unsigned grid_for(size_t work) { return (unsigned)std::max<size_t>(1, std::min<size_t>((work + kTPB - 1) / kTPB, 8192)); }

// per affected segment: its new member list, the old ranks its leavers had and its joiners
// with their new ranks (ins, sorted by rank)
struct EdInfo {
    World::Seg seg;
    std::vector<int32_t> rem, join;
    std::vector<std::pair<int32_t, int32_t>> ins;  // (new rank, object)
};

// A window's membership changes, planned on the host (plan_membership: the new member lists and
// the device's edit / move plans; it changes nothing of the world) and then applied
// (commit_membership: uploads and launches, then the host maps while the device rewrites the
// slots).  nfk_execute plans while the previous frame still runs on the GPU and waits for that
// frame before the commit, which rewrites slots the previous frame's fan-out recovery
// (regrow_fanout) reads.
struct MemPlan {
    bool active = false, full = false;
    int32_t max_np0 = 0;
    std::vector<int32_t> aff, epos;
    // einfo[0, n_einfo): this plan's affected segments; the entries (and their lists' buffers)
    // are kept from plan to plan, so a window's edits allocate nothing once they have been seen
    std::vector<EdInfo> einfo;
    size_t n_einfo = 0;
    std::vector<SegEdit> edits;
    std::vector<int32_t> ins_rank, ins_obj, rem_rank;
    std::vector<uint64_t> ins_meta;
    std::vector<int64_t> ins_src;
    std::vector<SegMove> moves;
    std::vector<World::Seg> nsegs;  // full: the new segment table
    std::vector<int32_t> nsrc;      // full: nsegs[i] is untouched segment nsrc[i] (members kept), or -1
    int32_t mv_rows_dev = 0, mv_list_dev = 0, ed_rows = 0, ed_list = 0;
    std::chrono::steady_clock::time_point t_host, t_edit, t_lists;
    std::chrono::steady_clock::time_point t_leave, t_join;  // (trace) the edit phase's parts
};

// Apply this window's membership changes (SwitchScene across groups, DestroyObject, exports,
// imports) before the frame: only the scene-group segments that changed are rewritten (the
// entities behind the first change shift by one slot each); a new (scene, group) or a segment
// whose slack ran out rebuilds the whole layout.
int plan_membership(World* w, MemPlan& p) {
    p.active = false;
    if (w->touched.empty()) return NFK_OK;
    using clk = std::chrono::steady_clock;
    p.t_host = clk::now();
    p.full = false;
    p.aff.clear();
    p.n_einfo = 0;
    p.edits.clear();
    p.ins_rank.clear();
    p.ins_obj.clear();
    p.rem_rank.clear();
    p.ins_meta.clear();
    p.ins_src.clear();
    p.moves.clear();
    p.mv_rows_dev = p.mv_list_dev = p.ed_rows = p.ed_list = 0;
    p.nsegs.clear();
    p.nsrc.clear();
    Dev& d = w->d;
    const auto cmp = [w](int32_t a, int32_t b) { return guid_less(w, a, b); };
    // The new member lists are built on copies of the affected segments; nothing of the world
    // changes before every check has passed (a failure leaves the window's calls queued).
    bool& full = p.full;
    std::vector<int32_t>& aff = p.aff;  // affected segments, in first-touch order
    auto seg_at = [&](int32_t slot) {
        int32_t lo = 0, hi = (int32_t)w->segs.size() - 1;
        while (lo < hi) {
            const int32_t mid = (lo + hi + 1) / 2;
            if (w->segs[mid].base <= slot) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    std::vector<int32_t>& epos = p.epos;
    epos.assign(w->segs.size(), -1);
    std::vector<EdInfo>& einfo = p.einfo;
    einfo.reserve(2 * w->touched.size() + 1);
    auto ed = [&](int32_t g) -> EdInfo& {
        if (epos[g] < 0) {
            if (p.n_einfo == einfo.size()) einfo.emplace_back();
            EdInfo& x = einfo[p.n_einfo];
            x.rem.clear();
            x.join.clear();
            x.ins.clear();
            x.seg.objs.clear();
            x.seg.keys.clear();
            epos[g] = (int32_t)p.n_einfo++;
            aff.push_back(g);
        }
        return einfo[epos[g]];
    };
    for (int32_t o : w->touched) {
        const int32_t s = w->slot_of_obj[o];
        if (s < 0) continue;
        const int32_t gi = seg_at(s);
        ed(gi).rem.push_back(s - w->segs[gi].base);  // members occupy [base, base + n) in NFGUID order
    }
    p.t_leave = clk::now();
    for (int32_t o : w->touched) {
        if (!w->alive[o]) continue;
        const int32_t gi = find_seg(w, w->scene[o], w->group[o]);
        if (gi < 0) {
            full = true;
            continue;
        }
        ed(gi).join.push_back(o);
    }
    p.t_join = clk::now();
    // each new member list in one pass: the old list without its leavers (known by rank, no
    // NFGUID comparison), the joiners (sorted) spliced in at their binary-searched places
    for (int32_t g : aff) {
        EdInfo& x = einfo[epos[g]];
        const World::Seg& old = w->segs[g];
        x.seg.scene = old.scene;
        x.seg.group = old.group;
        x.seg.base = old.base;
        x.seg.cap = old.cap;
        x.seg.np = old.np;
        std::sort(x.rem.begin(), x.rem.end());
        std::sort(x.join.begin(), x.join.end(), cmp);
        std::vector<int32_t>& v = x.seg.objs;
        std::vector<World::Guid>& kv = x.seg.keys;
        v.reserve(old.objs.size() - x.rem.size() + x.join.size());
        kv.reserve(v.capacity());
        // (a joiner's place is searched in the old list, leavers included: they are still in
        // NFGUID order, and one that rejoins compares equal to itself and is skipped below)
        size_t r = 0, at = 0;
        auto copy_to = [&](size_t p) {  // old ranks [at, p) without the leavers, as runs (memcpy-speed copies)
            while (at < p) {
                if (r < x.rem.size() && x.rem[r] == (int32_t)at) {
                    r++;
                    at++;
                    continue;
                }
                const size_t e = (r < x.rem.size() && (size_t)x.rem[r] < p) ? (size_t)x.rem[r] : p;
                v.insert(v.end(), old.objs.begin() + (std::ptrdiff_t)at, old.objs.begin() + (std::ptrdiff_t)e);
                kv.insert(kv.end(), old.keys.begin() + (std::ptrdiff_t)at, old.keys.begin() + (std::ptrdiff_t)e);
                at = e;
            }
        };
        const auto key_less = [](const World::Guid& a, const World::Guid& b) { return a.h != b.h ? a.h < b.h : a.d < b.d; };
        for (int32_t o : x.join) {
            const World::Guid go = w->guid[o];
            copy_to((size_t)(std::lower_bound(old.keys.begin() + at, old.keys.end(), go, key_less) - old.keys.begin()));
            x.ins.push_back({(int32_t)v.size(), o});
            v.push_back(o);
            kv.push_back(go);
        }
        copy_to(old.objs.size());
        if ((int32_t)v.size() > old.cap) full = true;
    }
    // edited and new segments: their slot lists are generated on the device (k_seg_edit) from the
    // removed ranks and the inserted objects at their new ranks
    std::vector<SegEdit>& edits = p.edits;
    std::vector<int32_t>&ins_rank = p.ins_rank, &ins_obj = p.ins_obj, &rem_rank = p.rem_rank;
    std::vector<uint64_t>& ins_meta = p.ins_meta;
    std::vector<int64_t>& ins_src = p.ins_src;
    int32_t &ed_rows = p.ed_rows, &ed_list = p.ed_list;
    // ob: the old segment (-1: a new (scene, group) pair; its members are all inserted)
    auto add_edit = [&](World::Seg& g, int32_t ob_seg, const std::vector<std::pair<int32_t, int32_t>>* ins,
                        const std::vector<int32_t>* rem, bool all) -> int {
        SegEdit e{};
        const World::Seg* old = ob_seg >= 0 ? &w->segs[ob_seg] : nullptr;
        e.ob = old ? old->base : -1;
        e.nb = g.base;
        e.on = old ? (int32_t)old->objs.size() : 0;
        e.nn = (int32_t)g.objs.size();
        e.nc = g.cap;
        int32_t np = old ? old->np : 0;
        e.io = (int32_t)ins_rank.size();
        if (ins) {  // (new rank, object), in rank order
            for (const auto& x : *ins) {
                const int32_t o = x.second;
                np += w->isplayer[o] ? 1 : 0;
                ins_rank.push_back(x.first);
                ins_obj.push_back(o);
                ins_meta.push_back(((uint64_t)w->cls[o] << 60) | (w->isplayer[o] ? 1u : 0u));
                ins_src.push_back(w->src_row[o] >= 0 ? -1 - w->src_row[o] : (int64_t)w->slot_of_obj[o]);
            }
        }
        e.ni = (int32_t)ins_rank.size() - e.io;
        e.ro = (int32_t)rem_rank.size();
        if (rem) {
            const size_t r0 = rem_rank.size();
            for (int32_t rk : *rem) {
                rem_rank.push_back(rk);
                np -= w->isplayer[old->objs[rk]] ? 1 : 0;
            }
            std::sort(rem_rank.begin() + r0, rem_rank.end());
        }
        e.nr = (int32_t)rem_rank.size() - e.ro;
        if (np > 0x3FFF) return fail(NFK_ERR_ARG, "more than 16383 players in one scene group");
        e.np = np;
        e.all = all ? 1 : 0;
        g.np = np;
        w->max_np = std::max(w->max_np, np);
        edits.push_back(e);
        return NFK_OK;
    };
    std::vector<World::Seg>& nsegs = p.nsegs;
    std::vector<int32_t>& nsrc = p.nsrc;
    std::vector<int32_t> nold;   // full: nsegs[i] is edited segment nold[i], or -1 (untouched / new)
    std::vector<SegMove>& moves = p.moves;  // full: untouched segments whose slot range changes
    int32_t &mv_rows_dev = p.mv_rows_dev, &mv_list_dev = p.mv_list_dev;
    const int32_t max_np0 = p.max_np0 = w->max_np;
    p.t_edit = clk::now();
    if (full) {
        // The (scene, group)-ordered segment table is rebuilt from the member lists: untouched
        // segments keep theirs, edited ones take their edit copies, the objects of new (scene,
        // group) pairs form new NFGUID-sorted segments, empty segments are dropped, and every
        // segment gets a fresh base and slack.  Nothing of the world is sorted — the result is
        // the layout a sort of every live object by (scene, group, NFGUID) would give.  The slot
        // lists of edited and new segments are built here; those of the untouched segments (the
        // bulk of the world) are generated on the device from their old and new ranges.
        std::map<std::pair<int32_t, int32_t>, std::vector<int32_t>> fresh;
        for (int32_t o : w->touched)
            if (w->alive[o] && find_seg(w, w->scene[o], w->group[o]) < 0)
                fresh[{w->scene[o], w->group[o]}].push_back(o);
        for (auto& f : fresh) std::sort(f.second.begin(), f.second.end(), cmp);
        auto fit = fresh.begin();
        auto push_fresh = [&]() {
            World::Seg g;
            g.scene = fit->first.first;
            g.group = fit->first.second;
            g.objs = std::move(fit->second);
            g.keys.resize(g.objs.size());
            for (size_t k = 0; k < g.objs.size(); k++) g.keys[k] = w->guid[g.objs[k]];
            nsegs.push_back(std::move(g));
            nsrc.push_back(-1);
            nold.push_back(-1);
            ++fit;
        };
        for (int32_t gi = 0; gi < (int32_t)w->segs.size(); gi++) {
            const World::Seg& old = w->segs[gi];
            const std::pair<int32_t, int32_t> key{old.scene, old.group};
            while (fit != fresh.end() && fit->first < key) push_fresh();
            const bool edited = epos[gi] >= 0;
            if ((edited ? einfo[epos[gi]].seg.objs : old.objs).empty()) continue;
            World::Seg g;
            g.scene = old.scene;
            g.group = old.group;
            if (edited) {
                g.objs = std::move(einfo[epos[gi]].seg.objs);
                g.keys = std::move(einfo[epos[gi]].seg.keys);
            }
            nsegs.push_back(std::move(g));
            nsrc.push_back(edited ? -1 : gi);
            nold.push_back(edited ? gi : -1);
        }
        while (fit != fresh.end()) push_fresh();
        auto members = [&](size_t i) -> const std::vector<int32_t>& {
            return nsrc[i] >= 0 ? w->segs[nsrc[i]].objs : nsegs[i].objs;
        };
        auto assign = [&](int32_t sl) {
            int64_t base = 0;
            for (size_t i = 0; i < nsegs.size(); i++) {
                const int32_t n = (int32_t)members(i).size();
                nsegs[i].base = (int32_t)std::min<int64_t>(base, INT32_MAX);
                nsegs[i].cap = n + seg_slack(sl, n);
                base += nsegs[i].cap;
            }
            return base;
        };
        int64_t total = assign(w->slack);
        if (total > d.cap) total = assign(0);
        if (total > d.cap) return fail(NFK_ERR_CAPACITY, "entity capacity exceeded (nothing of the window applied)");
        w->max_np = 0;  // recomputed over every segment below
        for (size_t i = 0; i < nsegs.size(); i++) {
            World::Seg& g = nsegs[i];
            if (nsrc[i] >= 0) {
                const World::Seg& old = w->segs[nsrc[i]];
                g.np = old.np;
                w->max_np = std::max(w->max_np, g.np);
                if (old.base == g.base && old.cap == g.cap) continue;  // stays where it is
                moves.push_back({old.base, g.base, (int32_t)old.objs.size(), g.cap, old.np, mv_rows_dev, mv_list_dev, 0});
                mv_rows_dev += (int32_t)old.objs.size();
                mv_list_dev += g.cap;
                continue;
            }
            int r;
            if (nold[i] >= 0) {
                const EdInfo& x = einfo[epos[nold[i]]];
                r = add_edit(g, nold[i], &x.ins, &x.rem, true);
            } else {  // a new (scene, group) pair: every member joins, at its rank
                std::vector<std::pair<int32_t, int32_t>> all_in(g.objs.size());
                for (size_t k = 0; k < g.objs.size(); k++) all_in[k] = {(int32_t)k, g.objs[k]};
                r = add_edit(g, -1, &all_in, nullptr, true);
            }
            if (r) {
                w->max_np = max_np0;
                return r;
            }
        }
    } else {
        for (int32_t gi : aff) {
            EdInfo& x = einfo[epos[gi]];
            int r = add_edit(x.seg, gi, &x.ins, &x.rem, false);
            if (r) {
                w->max_np = max_np0;
                return r;
            }
        }
    }
    for (SegEdit& e : edits) {  // their lists follow the untouched segments' (device-generated too)
        e.po = mv_rows_dev + ed_rows;
        e.lo = mv_list_dev + ed_list;
        ed_rows += e.nn;
        ed_list += e.nc;
    }

    p.t_lists = clk::now();
    p.active = true;
    return NFK_OK;
}

// the device phase of a planned window (after the previous frame has been waited for)
int commit_membership(World* w, MemPlan& p) {
    if (!p.active) return NFK_OK;
    p.active = false;
    w->obj_slot_dirty = true;  // (k_obj_slots before the next device fold)
    using clk = std::chrono::steady_clock;
    const auto t_dev = clk::now();
    Dev& d = w->d;
    const bool full = p.full;
    const std::vector<SegEdit>& edits = p.edits;
    const std::vector<int32_t>&ins_rank = p.ins_rank, &ins_obj = p.ins_obj, &rem_rank = p.rem_rank;
    const std::vector<uint64_t>& ins_meta = p.ins_meta;
    const std::vector<int64_t>& ins_src = p.ins_src;
    const std::vector<SegMove>& moves = p.moves;
    const int32_t mv_rows_dev = p.mv_rows_dev, mv_list_dev = p.mv_list_dev, ed_rows = p.ed_rows, ed_list = p.ed_list;
    std::vector<int32_t> pack_src, un_dst;  // (host-built lists: none since k_seg_edit)
    std::vector<int64_t> un_src;
    MetaLists m;
    // device: pack movers (old slots), then unpack into the new layout, then the metadata.  The
    // untouched segments' lists (full re-layout) are generated first, from the old metadata.
    const int32_t rw = w->row_words;
    w->mhost.clear();
    const size_t o_ps = stage_list(w, pack_src), o_ud = stage_list(w, un_dst), o_us = stage_list(w, un_src);
    const size_t o_ms = stage_list(w, m.slot), o_mo = stage_list(w, m.obj), o_md = stage_list(w, m.desc);
    const size_t o_mp = stage_list(w, m.pl), o_mv = stage_list(w, moves);
    const size_t o_ed = stage_list(w, edits), o_ir = stage_list(w, ins_rank), o_io = stage_list(w, ins_obj);
    const size_t o_im = stage_list(w, ins_meta), o_is = stage_list(w, ins_src), o_rr = stage_list(w, rem_rank);
    const size_t hp = pack_src.size();
    const size_t nd = (size_t)mv_list_dev + ed_list, npk = (size_t)mv_rows_dev + ed_rows;
    int r = dev_reserve(w, (void**)&w->mv_rows, &w->mv_cap, std::max<size_t>(hp + npk, 1) * rw * 8);
    if (r) return r;
    // device-generated lists (untouched segments that move, then edited / new segments):
    // pack_src | un_dst | un_src | m_slot | m_obj | m_desc | m_pl
    const size_t g_ps = 0, g_ud = align16(g_ps + npk * 4), g_us = align16(g_ud + nd * 4), g_ms = align16(g_us + nd * 8),
                 g_mo = align16(g_ms + nd * 4), g_md = align16(g_mo + nd * 4), g_mp = align16(g_md + nd * 8),
                 g_end = align16(g_mp + nd * 4);
    if (nd) {
        r = dev_reserve(w, (void**)&w->glist, &w->glist_cap, g_end);
        if (r) return r;
    }
    r = upload_mhost(w);
    if (r) return r;
    {
        TimeScope ts(w, KT_MEM);
        char* L = (char*)w->mlist;
        char* G = (char*)w->glist;
        if (!moves.empty())
            hipLaunchKernelGGL(k_seg_lists, dim3((unsigned)std::min<size_t>(moves.size(), 8192)), dim3(kTPB), 0,
                               w->stream, (const SegMove*)(L + o_mv), (int32_t)moves.size(),
                               (const int32_t*)w->slot_obj_d, (const uint64_t*)w->fan_desc_w,
                               (const int32_t*)w->pl_slot_w, (int32_t*)(G + g_ps), (int32_t*)(G + g_ud),
                               (int64_t*)(G + g_us), (int32_t*)(G + g_ms), (int32_t*)(G + g_mo), (uint64_t*)(G + g_md),
                               (int32_t*)(G + g_mp));
        if (!edits.empty())
            hipLaunchKernelGGL(k_seg_edit, dim3((unsigned)std::min<size_t>(edits.size(), 8192)), dim3(kTPB), 0,
                               w->stream, (const SegEdit*)(L + o_ed), (int32_t)edits.size(), (const int32_t*)(L + o_ir),
                               (const int32_t*)(L + o_io), (const uint64_t*)(L + o_im), (const int64_t*)(L + o_is),
                               (const int32_t*)(L + o_rr), (const int32_t*)w->slot_obj_d, (const uint64_t*)w->fan_desc_w,
                               (int32_t*)(G + g_ps), (int32_t*)(G + g_ud), (int64_t*)(G + g_us), (int32_t*)(G + g_ms),
                               (int32_t*)(G + g_mo), (uint64_t*)(G + g_md), (int32_t*)(G + g_mp));
        if (hp)
            hipLaunchKernelGGL(k_pack, dim3(grid_for(hp * rw)), dim3(kTPB), 0, w->stream, d,
                               (const int32_t*)(L + o_ps), (int32_t)hp, rw, w->mv_rows);
        if (npk)
            hipLaunchKernelGGL(k_pack, dim3(grid_for(npk * rw)), dim3(kTPB), 0, w->stream, d,
                               (const int32_t*)(G + g_ps), (int32_t)npk, rw, w->mv_rows + hp * rw);
        if (!un_dst.empty())
            hipLaunchKernelGGL(k_unpack, dim3(grid_for(un_dst.size() * rw)), dim3(kTPB), 0, w->stream, d,
                               (const int32_t*)(L + o_ud), (const int64_t*)(L + o_us), (int32_t)un_dst.size(), rw,
                               (const uint64_t*)w->mv_rows, (const uint64_t*)w->ins_rows);
        if (nd)
            hipLaunchKernelGGL(k_unpack, dim3(grid_for(nd * rw)), dim3(kTPB), 0, w->stream, d,
                               (const int32_t*)(G + g_ud), (const int64_t*)(G + g_us), (int32_t)nd, rw,
                               (const uint64_t*)(w->mv_rows + hp * rw), (const uint64_t*)w->ins_rows);
        if (!m.slot.empty())
            hipLaunchKernelGGL(k_meta, dim3(grid_for(m.slot.size())), dim3(kTPB), 0, w->stream,
                               (const int32_t*)(L + o_ms), (const int32_t*)(L + o_mo), (const uint64_t*)(L + o_md),
                               (const int32_t*)(L + o_mp), (int32_t)m.slot.size(), w->slot_obj_d, w->fan_desc_w,
                               w->pl_slot_w);
        if (nd)
            hipLaunchKernelGGL(k_meta, dim3(grid_for(nd)), dim3(kTPB), 0, w->stream, (const int32_t*)(G + g_ms),
                               (const int32_t*)(G + g_mo), (const uint64_t*)(G + g_md), (const int32_t*)(G + g_mp),
                               (int32_t)nd, w->slot_obj_d, w->fan_desc_w, w->pl_slot_w);
        HIPCHK(hipGetLastError());
    }
    const auto t_launched = clk::now();
    const size_t n_touched = w->touched.size();
    // host maps (while the device rewrites the slots)
    std::vector<int32_t>& aff = p.aff;
    const std::vector<int32_t>& epos = p.epos;
    std::vector<EdInfo>& einfo = p.einfo;
    std::vector<World::Seg>& nsegs = p.nsegs;
    const std::vector<int32_t>& nsrc = p.nsrc;
    if (full) {
        w->n_relayout_full++;
        std::vector<int32_t> seg_base0(nsegs.size(), -1), seg_cap0(nsegs.size(), -1);
        for (size_t i = 0; i < nsegs.size(); i++)
            if (nsrc[i] >= 0) {
                seg_base0[i] = w->segs[nsrc[i]].base;
                seg_cap0[i] = w->segs[nsrc[i]].cap;
                nsegs[i].objs = std::move(w->segs[nsrc[i]].objs);
                nsegs[i].keys = std::move(w->segs[nsrc[i]].keys);
            }
        w->segs = std::move(nsegs);
        index_segs(w);
        int64_t total = 0;
        for (const auto& g : w->segs) total = (int64_t)g.base + g.cap;
        // slots past the new end held entities before; every slot below it belongs to a segment
        for (int64_t sl = total; sl < std::min<int64_t>(d.N, (int64_t)w->obj_of_slot.size()); sl++)
            w->obj_of_slot[sl] = -1;
        set_tiles(d, (int32_t)total);
        // the host maps change for the segments whose slots or members changed
        aff.clear();
        for (size_t g = 0; g < w->segs.size(); g++)
            if (nsrc[g] < 0 || w->segs[g].base != seg_base0[g] || w->segs[g].cap != seg_cap0[g]) aff.push_back((int32_t)g);
    } else {
        w->n_relayout_seg++;
        for (int32_t gi : aff) {  // (the old list's buffer goes back to the plan, for the next window)
            std::swap(w->segs[gi].objs, einfo[epos[gi]].seg.objs);
            std::swap(w->segs[gi].keys, einfo[epos[gi]].seg.keys);
            w->segs[gi].np = einfo[epos[gi]].seg.np;
        }
    }
    // the ranks whose slot <-> object pairs change: [first leaver / joiner, the longer of the two
    // lists), or only up to the last leaver / joiner when as many join as leave (the members
    // behind it keep their ranks)
    std::vector<int32_t> mlo(aff.size(), 0), mhi(aff.size());
    for (size_t k = 0; k < aff.size(); k++) {
        mhi[k] = w->segs[aff[k]].cap;
        if (full) continue;
        const EdInfo& x = einfo[epos[aff[k]]];
        const int32_t nn = (int32_t)w->segs[aff[k]].objs.size(), no = nn - (int32_t)x.ins.size() + (int32_t)x.rem.size();
        int32_t lo = INT32_MAX, last = -1;
        if (!x.rem.empty()) lo = x.rem.front(), last = x.rem.back();
        if (!x.ins.empty()) lo = std::min(lo, x.ins.front().first), last = std::max(last, x.ins.back().first);
        mlo[k] = std::min(lo, mhi[k]);
        mhi[k] = nn != no ? std::max(nn, no) : last + 1;
    }
    for (int32_t o : w->touched)
        if (!w->alive[o]) w->slot_of_obj[o] = -1;
    // slot <-> object of the changed segments (disjoint slots and objects per segment: split over
    // threads when large)
    auto maps = [w, &aff, &mlo, &mhi](size_t a, size_t b) {
        for (size_t k = a; k < b; k++) {
            const World::Seg& g = w->segs[aff[k]];
            for (int32_t i = mlo[k]; i < mhi[k]; i++) {
                const int32_t ns = g.base + i;
                const int32_t o = i < (int32_t)g.objs.size() ? g.objs[i] : -1;
                w->obj_of_slot[ns] = o;
                if (o >= 0) w->slot_of_obj[o] = ns;
            }
        }
    };
    {
        int64_t work = 0;
        for (size_t k = 0; k < aff.size(); k++) work += mhi[k] - mlo[k];
        const int nt = work >= (1 << 17) ? (int)std::min<size_t>(8, aff.size()) : 1;
        if (nt <= 1) {
            maps(0, aff.size());
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; t++) th.emplace_back(maps, aff.size() * t / nt, aff.size() * (t + 1) / nt);
            for (auto& x : th) x.join();
        }
    }
    for (int32_t o : w->touched) {
        w->m_flag[o] = 0;
        w->src_row[o] = -1;
    }
    w->touched.clear();
    w->ins_n = 0;
    const auto t_end = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    (full ? w->ms_relayout_full : w->ms_relayout_seg) += ms(p.t_host, p.t_lists) + ms(t_dev, t_end);
    if (getenv("NFGPU_TRACE_MEMBERSHIP"))
        fprintf(stderr, "apply_membership %s: %zu touched, edit %.3f ms (leavers %.3f, joiners %.3f, member lists %.3f), "
                "lists %.3f ms (%zu edited segments, %zu moves; "
                "before the previous frame is waited for), upload+launch %.3f ms, host maps %.3f ms\n",
                full ? "full" : "seg", n_touched, ms(p.t_host, p.t_edit), ms(p.t_host, p.t_leave), ms(p.t_leave, p.t_join),
                ms(p.t_join, p.t_edit), ms(p.t_edit, p.t_lists), edits.size(),
                moves.size(), ms(t_dev, t_launched), ms(t_launched, t_end));
    return NFK_OK;
}

// a new object index (creation order in this world)
int32_t add_object(World* w, int64_t gh, int64_t gd, int32_t scene, int32_t group, uint8_t cls, uint8_t pl) {
    const int32_t o = w->n_obj++;
    w->obj_of.insert(gh, gd, o);
    w->gh.push_back(gh);
    w->guid.push_back({gh, gd});
    w->gd.push_back(gd);
    w->scene.push_back(scene);
    w->group.push_back(group);
    w->cls.push_back(cls);
    w->isplayer.push_back(pl ? 1 : 0);
    w->alive.push_back(1);
    w->src_row.push_back(-1);
    w->m_flag.push_back(0);
    w->slot_of_obj.push_back(-1);
    return o;
}

void touch(World* w, int32_t o) {
    if (!w->m_flag[o]) {
        w->m_flag[o] = 1;
        w->touched.push_back(o);
    }
}

}  // namespace

extern "C" {

static int check_fanout(World* w);

const char* nfk_last_error(void) { return g_err.c_str(); }

int nfk_create(const nfk_config* cfg, void** out) {
    if (!cfg || !out) return fail(NFK_ERR_ARG, "null argument");
    if (cfg->capacity <= 0 || cfg->n_int < 0 || cfg->n_int > NFK_MAX_INT_PROPS || cfg->n_flt < 0 ||
        cfg->n_flt > NFK_MAX_FLT_PROPS || cfg->n_class <= 0 || cfg->n_class > NFK_MAX_CLASSES - 1 ||
        cfg->n_kind < 0 || cfg->n_kind > NFK_MAX_KINDS || cfg->n_rec < 0 || cfg->n_rec > NFK_MAX_RECORDS ||
        cfg->n_obj < 0 || cfg->n_obj > NFK_MAX_OBJ_PROPS || cfg->n_int + cfg->n_flt + cfg->n_obj > NFK_MAX_PROPS)
        return fail(NFK_ERR_ARG, "config out of range");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return fail(NFK_ERR_HIP, "no HIP device available");
    World* w = new World();
    {
        // host threads for large call batches (the caller and nt - 1 workers).  Default 1: on the
        // GPU boxes the workers made the host work slower, not faster (schedule-call fold 0.85 vs
        // 0.31 ms, the SetProperty fold 3-6 vs 0.67 ms before it moved to the device;
        // profiles/r08b_hostprof*.log)
        int nt = 1;
        if (const char* e = getenv("NFGPU_HOST_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
        w->pool.reset(new HostPool(nt - 1));
        if (const char* e = getenv("NFGPU_PAR_CALLS")) w->par_calls = (size_t)std::max(1, atoi(e));
        if (const char* e = getenv("NFGPU_DEV_LOOKUP")) w->dev_look_min = (size_t)std::max(0, atoi(e));
        w->obj_of.set_log(&w->guid_log);
    }
    w->cfg = *cfg;
    w->n_if = cfg->n_int + cfg->n_flt;
    w->n_prop = w->n_if + cfg->n_obj;
    w->n_pw = w->n_if + 2 * cfg->n_obj;
    w->slack = cfg->slack_per_256 == 0 ? 16 : std::max(cfg->slack_per_256, 0);
    if (cfg->stream) {
        w->stream = (hipStream_t)cfg->stream;
    } else {
        if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) {
            delete w;
            return fail(NFK_ERR_HIP, "hipStreamCreate failed");
        }
        w->own_stream = true;
    }
    if (hipEventCreateWithFlags(&w->pin_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->mpin_done[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->mpin_done[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->err_done, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&w->err_pin, 64, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&w->ctrl_pin, kCtrlPinBytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&w->err_host, 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&w->err_host_d, w->err_host, 0) != hipSuccess) {
        delete w;
        return fail(NFK_ERR_HIP, "hipEventCreate failed");
    }
    clear_err_host(w);
    w->init_props.resize(w->n_prop);
    w->init_rcells.resize(cfg->n_rec);
    w->init_rused.resize(cfg->n_rec);
    w->rec_defined.assign(cfg->n_rec, false);
    *out = w;
    return NFK_OK;
}

int nfk_destroy(void* world) {
    World* w = (World*)world;
    if (!w) return NFK_OK;
    (void)hipStreamSynchronize(w->stream);
    for (void* p : w->allocs) (void)hipFree(p);
    if (w->pin) (void)hipHostFree(w->pin);
    if (w->stage) (void)hipFree(w->stage);
    if (w->dense) (void)hipFree(w->dense);
    if (w->fr_dev) (void)hipFree(w->fr_dev);
    if (w->fr_pin) (void)hipHostFree(w->fr_pin);
    if (w->fr_scr) (void)hipFree(w->fr_scr);
    if (w->rank_d) (void)hipFree(w->rank_d);
    if (w->ins_rows) (void)hipFree(w->ins_rows);
    if (w->mv_rows) (void)hipFree(w->mv_rows);
    if (w->mlist) (void)hipFree(w->mlist);
    if (w->glist) (void)hipFree(w->glist);
    if (w->xs_buf) (void)hipFree(w->xs_buf);
    if (w->xf_buf) (void)hipFree(w->xf_buf);
    if (w->tile_work_d) (void)hipFree(w->tile_work_d);
    for (int b = 0; b < 2; b++) {
        if (w->xq[b]) (void)hipFree(w->xq[b]);
        if (w->xq_ev[b]) (void)hipEventDestroy(w->xq_ev[b]);
    }
    if (w->obj_slot_d) (void)hipFree(w->obj_slot_d);
    if (w->rs_buf) (void)hipFree(w->rs_buf);
    if (w->rss_buf) (void)hipFree(w->rss_buf);
    if (w->rl_buf) (void)hipFree(w->rl_buf);
    if (w->look_stream) (void)hipStreamSynchronize(w->look_stream);
    if (w->guid_d) (void)hipFree(w->guid_d);
    if (w->look_dev) (void)hipFree(w->look_dev);
    if (w->look_pin) (void)hipHostFree(w->look_pin);
    if (w->look_stream) (void)hipStreamDestroy(w->look_stream);
    if (w->gat) (void)hipFree(w->gat);
    if (w->moff_tmp) (void)hipFree(w->moff_tmp);
    if (w->hf_buf) (void)hipFree(w->hf_buf);
    if (w->chain_d) (void)hipFree(w->chain_d);
    if (w->chain_cnt_d) (void)hipFree(w->chain_cnt_d);
    if (w->chain_scr) (void)hipFree(w->chain_scr);
    if (w->chain_pin) (void)hipHostFree(w->chain_pin);
    for (auto& p : w->pend) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : w->evpool) (void)hipEventDestroy(e);
    if (w->pin_done) (void)hipEventDestroy(w->pin_done);
    if (w->err_done) (void)hipEventDestroy(w->err_done);
    if (w->err_pin) (void)hipHostFree(w->err_pin);
    if (w->ctrl_pin) (void)hipHostFree(w->ctrl_pin);
    if (w->err_host) (void)hipHostFree(w->err_host);
    for (int i = 0; i < 2; i++) {
        if (w->mpin_done[i]) (void)hipEventDestroy(w->mpin_done[i]);
        if (w->mpin[i]) (void)hipHostFree(w->mpin[i]);
    }
    if (w->xpin_done) (void)hipEventDestroy(w->xpin_done);
    if (w->xpin) (void)hipHostFree(w->xpin);
    if (w->own_stream) (void)hipStreamDestroy(w->stream);
    delete w;
    return NFK_OK;
}

int nfk_set_prop_flags(void* world, int32_t c, const uint8_t* flags) {
    World* w = (World*)world;
    if (!w || !flags || c < 0 || c >= w->cfg.n_class) return fail(NFK_ERR_ARG, "bad class");
    for (int p = 0; p < w->n_prop; p++) w->tab.pflags[c][p] = flags[p];
    return NFK_OK;
}

int nfk_define_record(void* world, int32_t rec, int32_t rows, int32_t cols, const uint8_t* col_types,
                      const uint8_t* flags_per_class) {
    World* w = (World*)world;
    if (!w || rec < 0 || rec >= w->cfg.n_rec || rows <= 0 || rows > NFK_MAX_REC_ROWS || cols <= 0 ||
        cols > NFK_MAX_REC_COLS || !flags_per_class)
        return fail(NFK_ERR_ARG, "bad record definition");
    if (w->committed) return fail(NFK_ERR_STATE, "schema is fixed after commit");
    w->tab.rec_rows[rec] = rows;
    w->tab.rec_cols[rec] = cols;
    for (int c = 0; c < w->cfg.n_class; c++) w->tab.rflags[c][rec] = flags_per_class[c];
    for (int c = 0; c < cols; c++) {
        if (col_types && col_types[c] > 1) return fail(NFK_ERR_ARG, "record column type must be 0 (int64) or 1 (f64)");
        w->rec_ctype[rec][c] = col_types ? col_types[c] : 0;
    }
    w->rec_defined[rec] = true;
    return NFK_OK;
}

int nfk_define_kind(void* world, int32_t kind, const nfk_op* ops, int32_t n_ops) {
    World* w = (World*)world;
    if (!w || kind < 0 || kind >= w->cfg.n_kind || n_ops < 0 || n_ops > NFK_MAX_OPS || (n_ops && !ops))
        return fail(NFK_ERR_ARG, "bad kind definition");
    if (w->committed) return fail(NFK_ERR_STATE, "schema is fixed after commit");
    for (int i = 0; i < n_ops; i++) {
        const nfk_op& op = ops[i];
        const int np = w->n_if, ni = w->cfg.n_int;  // (object properties are no program operands)
        auto isint = [&](int64_t p) { return p >= 0 && p < ni; };
        auto isflt = [&](int64_t p) { return p >= ni && p < np; };
        if (op.flags & NFK_GUARD) {
            const bool rec = op.code == NFK_OP_RIADD_CLAMP || op.code == NFK_OP_RFAFFINE;
            // (NFK_GUARD_PROP: compared to the int property guard >> 19; otherwise to the constant
            // NFK_GUARD_KVAL(guard) in bits 19..31, any value)
            const bool vs = (op.guard & NFK_GUARD_PROP) != 0;
            if (rec || op.code == NFK_OP_NOP || !isint(op.guard & 0xFFFF) || (vs && !isint(op.guard >> 19)))
                return fail(NFK_ERR_ARG, "NFK_GUARD: a property op guarded by an int property");
        } else if (op.guard) {
            return fail(NFK_ERR_ARG, "nfk_op.guard without NFK_GUARD");
        }
        switch (op.code) {
        case NFK_OP_IADD_CLAMP:
            if (!isint(op.dst) || ((op.flags & NFK_A_PROP) && !isint(op.a)) ||
                ((op.flags & NFK_LO_PROP) && !isint(op.b)) || ((op.flags & NFK_HI_PROP) && !isint(op.c)))
                return fail(NFK_ERR_ARG, "IADD_CLAMP operands must be int properties");
            break;
        case NFK_OP_FLERP:
            if (!isflt(op.dst) || !isflt(op.a)) return fail(NFK_ERR_ARG, "FLERP operands must be float properties");
            break;
        case NFK_OP_FAFFINE:
            if (!isflt(op.dst)) return fail(NFK_ERR_ARG, "FAFFINE dst must be a float property");
            break;
        case NFK_OP_ISET:
            if (!isint(op.dst) || ((op.flags & NFK_A_PROP) && !isint(op.a)))
                return fail(NFK_ERR_ARG, "ISET operands must be int properties");
            break;
        case NFK_OP_FSET:
            if (!isflt(op.dst) || ((op.flags & NFK_A_PROP) && !isflt(op.a)))
                return fail(NFK_ERR_ARG, "FSET operands must be float properties");
            break;
        case NFK_OP_RIADD_CLAMP:
        case NFK_OP_RFAFFINE: {
            int r = op.dst >> 8, col = op.dst & 255;
            if (r >= w->cfg.n_rec || !w->rec_defined[r] || col >= w->tab.rec_cols[r])
                return fail(NFK_ERR_ARG, "record op on undefined record/col");
            // NFCRecord::SetInt / SetFloat refuse a cell of the other type (RC:189, RC:250): such
            // an op could never change a cell, so it is rejected with the kind
            if (w->rec_ctype[r][col] != (op.code == NFK_OP_RFAFFINE ? 1 : 0))
                return fail(NFK_ERR_ARG, "record op type does not match the column type");
            break;
        }
        case NFK_OP_NOP:
            break;
        default:
            return fail(NFK_ERR_ARG, "unknown op code");
        }
        w->tab.ops[kind][i] = op;
    }
    w->tab.nops[kind] = n_ops;
    w->kind_defined[kind] = true;
    return NFK_OK;
}

int nfk_create_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* scene,
                       const int32_t* group, const uint8_t* cls, const uint8_t* isplayer) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !scene || !group || !cls || !isplayer)))
        return fail(NFK_ERR_ARG, "null argument");
    if (w->committed) return fail(NFK_ERR_STATE, "after commit, create objects with nfk_import_objects / nfk_spawn_objects");
    if ((int64_t)w->n_obj + n > w->cfg.capacity) return fail(NFK_ERR_CAPACITY, "entity capacity exceeded");
    for (int32_t i = 0; i < n; i++) {
        if (cls[i] >= w->cfg.n_class) return fail(NFK_ERR_ARG, "class id out of range");
        if (group[i] < 0) return fail(NFK_ERR_ARG, "negative group");
        if (w->obj_of.count(gh[i], gd[i])) return fail(NFK_ERR_ARG, "The object has Exists");  // KM:131
    }
    for (int32_t i = 0; i < n; i++) add_object(w, gh[i], gd[i], scene[i], group[i], cls[i], isplayer[i]);
    return NFK_OK;
}

int nfk_load_prop(void* world, int32_t pid, const uint64_t* bits) {
    World* w = (World*)world;
    if (!w || pid < 0 || pid >= w->n_if || !bits) return fail(NFK_ERR_ARG, "bad property (object properties: nfk_load_object)");
    if (w->committed) return fail(NFK_ERR_STATE, "load before commit");
    w->init_props[pid].assign(bits, bits + w->n_obj);
    return NFK_OK;
}

int nfk_load_object(void* world, int32_t pid, const int64_t* head, const int64_t* data) {
    World* w = (World*)world;
    if (!w || pid < w->n_if || pid >= w->n_prop || !head || !data) return fail(NFK_ERR_ARG, "bad object property");
    if (w->committed) return fail(NFK_ERR_STATE, "load before commit");
    std::vector<uint64_t>& v = w->init_props[pid];  // (data, head) per object
    v.resize((size_t)2 * w->n_obj);
    for (int32_t o = 0; o < w->n_obj; o++) {
        v[2 * (size_t)o] = (uint64_t)data[o];
        v[2 * (size_t)o + 1] = (uint64_t)head[o];
    }
    return NFK_OK;
}

int nfk_load_record(void* world, int32_t rec, const uint64_t* cells, const uint64_t* used) {
    World* w = (World*)world;
    if (!w || rec < 0 || rec >= w->cfg.n_rec || !w->rec_defined[rec] || !cells || !used)
        return fail(NFK_ERR_ARG, "bad record");
    if (w->committed) return fail(NFK_ERR_STATE, "load before commit");
    size_t per = (size_t)w->tab.rec_rows[rec] * w->tab.rec_cols[rec];
    w->init_rcells[rec].assign(cells, cells + per * w->n_obj);
    w->init_rused[rec].assign(used, used + w->n_obj);
    return NFK_OK;
}

int nfk_commit(void* world) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (w->committed) return fail(NFK_ERR_STATE, "already committed");
    const int32_t cfg_cap = w->cfg.capacity;
    int32_t cap = 0;
    const int NI = w->cfg.n_int, NF = w->cfg.n_flt, NK = w->cfg.n_kind, NR = w->cfg.n_rec;
    for (int r = 0; r < NR; r++)
        if (!w->rec_defined[r]) return fail(NFK_ERR_ARG, "record " + std::to_string(r) + " not defined");

    // record ops: compiled list sorted by (rec, col); distinct (rec, col) required
    int nro = 0;
    for (int k = 0; k < NK; k++)
        for (int i = 0; i < w->tab.nops[k]; i++) {
            const nfk_op& op = w->tab.ops[k][i];
            if (op.code == NFK_OP_RIADD_CLAMP || op.code == NFK_OP_RFAFFINE) {
                if (nro == NFK_MAX_REC_OPS) return fail(NFK_ERR_ARG, "at most NFK_MAX_REC_OPS record ops across all kinds");
                RecOp ro{k, op.dst >> 8, op.dst & 255, op.code, op.a, op.b, op.c};
                w->tab.recops[nro++] = ro;
                w->tab.kind_has_recop |= 1u << k;
            } else if (prop_op(op.code)) {
                w->dst_union_mask[op.dst >> 6] |= 1ull << (op.dst & 63);
            }
        }
    std::sort(w->tab.recops, w->tab.recops + nro, [](const RecOp& a, const RecOp& b) {
        return a.rec != b.rec ? a.rec < b.rec : a.col < b.col;
    });
    for (int i = 1; i < nro; i++)
        if (w->tab.recops[i].rec == w->tab.recops[i - 1].rec && w->tab.recops[i].col == w->tab.recops[i - 1].col)
            return fail(NFK_ERR_ARG, "two record ops on the same (record, col)");
    w->tab.n_recops = nro;
    // the programs' working set (k_tick): program destinations -> writable U slots, read-only
    // operands after them (build_u_tables)
    w->u_ok = build_u_tables(w->tab, NK, w->u_wp, w->u_rp);
    w->n_dst_union = __builtin_popcountll(w->dst_union_mask[0]) + __builtin_popcountll(w->dst_union_mask[1]);
    if (w->n_dst_union > NFK_MAX_TOUCH)
        return fail(NFK_ERR_TOUCH, "programs write more than NFK_MAX_TOUCH distinct properties");

    // property columns (Tables::p_off / p_str): one plain column per property.  Two interleaved
    // layouts are kept as timing variants (NFGPU_ABLATE): kAblGroupColumns, the properties one
    // heartbeat program touches interleaved (one line per entity for a sparse kind), and
    // kAblSigGroups, properties with the same access signature interleaved.  Plain columns measured
    // fastest on config[1] (profiles/r01zo_ablate.log: 99.8 us vs 110.7 grouped, 104.8 by
    // signature): a dense kind's strided 8-byte accesses cost twice the L2 requests per load and
    // its write-backs cover half lines, while a sparse kind's extra lines are few.
    std::vector<std::vector<int>> pgroups;
    const char* ab_env = getenv("NFGPU_ABLATE");
    const uint32_t ab_layout = ab_env ? (uint32_t)strtoul(ab_env, nullptr, 0) : 0u;
    if (!(ab_layout & kAblGroupColumns)) {
        // plain columns, or groups of properties with the same access signature (the set of
        // (kind, read / write) that touch them): every access covers a group
        const int NP = w->n_if;
        std::vector<std::vector<int>> sig(NP);
        for (int k = 0; k < NK && (ab_layout & kAblSigGroups); k++)
            for (int i = 0; i < w->tab.nops[k]; i++) {
                const nfk_op& op = w->tab.ops[k][i];
                auto add = [&](int p, int rw) { if (p >= 0 && p < NP) sig[p].push_back(2 * k + rw); };
                if (op.code == NFK_OP_IADD_CLAMP) {
                    add(op.dst, 1);
                    if (op.flags & NFK_A_PROP) add((int)op.a, 0);
                    if (op.flags & NFK_LO_PROP) add((int)op.b, 0);
                    if (op.flags & NFK_HI_PROP) add((int)op.c, 0);
                } else if (op.code == NFK_OP_FLERP) {
                    add(op.dst, 1);
                    add((int)op.a, 0);
                } else if (op.code == NFK_OP_FAFFINE) {
                    add(op.dst, 1);
                } else if (op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) {
                    add(op.dst, 1);
                    if (op.flags & NFK_A_PROP) add((int)op.a, 0);
                }
                if (op.flags & NFK_GUARD) add((int)(op.guard & 0xFFFF), 0);
                if ((op.flags & NFK_GUARD) && (op.guard & NFK_GUARD_PROP)) add((int)(op.guard >> 19), 0);
            }
        std::map<std::vector<int>, int> gi;
        for (int p = 0; p < NP; p++) {
            auto& g = sig[p];
            std::sort(g.begin(), g.end());
            g.erase(std::unique(g.begin(), g.end()), g.end());
            auto it = g.empty() ? gi.end() : gi.find(g);
            if (it != gi.end() && pgroups[it->second].size() < 8) {
                pgroups[it->second].push_back(p);
            } else {
                if (!g.empty()) gi[g] = (int)pgroups.size();
                pgroups.push_back({p});
            }
        }
    } else {
        const int NP = w->n_if;
        constexpr int kGroupMax = 8;
        std::vector<int> par(NP), sz(NP, 1);
        for (int p = 0; p < NP; p++) par[p] = p;
        std::function<int(int)> find = [&](int x) { return par[x] == x ? x : par[x] = find(par[x]); };
        // (NFGPU_GROUP_SKIP: a mask of kinds whose properties are not grouped, for A/B)
        const uint32_t skip = getenv("NFGPU_GROUP_SKIP") ? (uint32_t)strtoul(getenv("NFGPU_GROUP_SKIP"), nullptr, 0) : 0u;
        for (int k = 0; k < NK; k++) {
            std::vector<int> ps;
            for (int i = 0; i < w->tab.nops[k] && !((skip >> k) & 1); i++) {
                const nfk_op& op = w->tab.ops[k][i];
                if (op.code == NFK_OP_IADD_CLAMP) {
                    ps.push_back(op.dst);
                    if (op.flags & NFK_A_PROP) ps.push_back((int)op.a);
                    if (op.flags & NFK_LO_PROP) ps.push_back((int)op.b);
                    if (op.flags & NFK_HI_PROP) ps.push_back((int)op.c);
                } else if (op.code == NFK_OP_FLERP) {
                    ps.push_back(op.dst);
                    ps.push_back((int)op.a);
                } else if (op.code == NFK_OP_FAFFINE) {
                    ps.push_back(op.dst);
                } else if (op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) {
                    ps.push_back(op.dst);
                    if (op.flags & NFK_A_PROP) ps.push_back((int)op.a);
                }
                if (op.flags & NFK_GUARD) ps.push_back((int)(op.guard & 0xFFFF));
                if ((op.flags & NFK_GUARD) && (op.guard & NFK_GUARD_PROP)) ps.push_back((int)(op.guard >> 19));
            }
            for (size_t i = 1; i < ps.size(); i++) {
                const int a = find(ps[0]), b = find(ps[i]);
                if (a != b && sz[a] + sz[b] <= kGroupMax) {
                    par[b] = a;
                    sz[a] += sz[b];
                }
            }
        }
        std::vector<int> gi(NP, -1);
        for (int p = 0; p < NP; p++) {
            const int r = find(p);
            if (gi[r] < 0) {
                gi[r] = (int)pgroups.size();
                pgroups.emplace_back();
            }
            pgroups[gi[r]].push_back(p);
        }
    }

    // membership layout: scene-group segments, NFGUID order inside (see plan_membership)
    const int64_t n_slots = plan_segments(w, w->slack, w->segs);
    index_segs(w);
    MetaLists meta;
    w->max_np = 0;
    for (auto& g : w->segs) {
        int r = seg_meta(w, g, meta);
        if (r) return r;
    }
    {
        // slot capacity: the population plus slack, and at least the configured capacity plus slack
        const int64_t want = std::max<int64_t>(n_slots, (int64_t)cfg_cap + (int64_t)cfg_cap * w->slack / 256);
        const int64_t c = (want + kTile - 1) / kTile * kTile;
        if (c > INT32_MAX / 2) return fail(NFK_ERR_CAPACITY, "slot capacity too large");
        cap = (int32_t)c;
    }
    w->obj_of_slot.assign(cap, -1);
    for (size_t i = 0; i < meta.slot.size(); i++) {
        w->obj_of_slot[meta.slot[i]] = meta.obj[i];
        if (meta.obj[i] >= 0) w->slot_of_obj[meta.obj[i]] = meta.slot[i];
    }
    w->row_words = w->n_pw + 4 * NK;
    for (int r = 0; r < NR; r++) w->row_words += w->tab.rec_rows[r] * w->tab.rec_cols[r] + 1;

    // device allocation
    Dev& d = w->d;
    d.cap = cap;
    set_tiles(d, (int32_t)n_slots);
    d.n_int = NI;
    d.n_flt = NF;
    d.n_if = NI + NF;
    d.n_obj = w->cfg.n_obj;
    d.err_host = w->err_host_d;
    d.n_kind = NK;
    d.n_rec = NR;
    d.n_class = w->cfg.n_class;
    // the record pipeline (fired masks, k_records, record tiles) runs in a world with record
    // programs or with records that SetRecord* calls can change
    bool any_rec = false;
    for (int r = 0; r < NR; r++) any_rec = any_rec || w->rec_defined[r];
    d.has_recops = nro > 0 || any_rec;
    memcpy(w->tab.rec_ctype, w->rec_ctype, sizeof(w->tab.rec_ctype));
    ALLOC(w->tab_d, sizeof(Tables));
    ALLOC(d.tally, (size_t)3 * kTallyN * 8 * 8);
    ALLOC(w->ctrl, sizeof(Ctrl));
    const int64_t cpad = (ab_layout & kAblNoPad) ? 0 : kColPad / 8;  // column pad in values
    d.s_kstr = cap + (int32_t)((ab_layout & kAblNoPad) ? 0 : kColPad / (int64_t)sizeof(SchedHot));
    ALLOC(d.pmem, ((size_t)cap + cpad) * (size_t)std::max(w->n_pw, 1) * 8);
    {
        int64_t off = 0;
        for (const auto& g : pgroups) {
            for (size_t i = 0; i < g.size(); i++) {
                w->tab.p_off[g[i]] = off + (int64_t)i;
                w->tab.p_str[g[i]] = (int32_t)g.size();
            }
            off += (int64_t)g.size() * cap + cpad;
        }
        // an object property is one 16-byte column: (data, head) of slot e at p_off + 2e
        for (int p = w->n_if; p < w->n_prop; p++) {
            w->tab.p_off[p] = off;
            w->tab.p_str[p] = 2;
            off += 2 * (int64_t)cap + cpad;
        }
    }
    set_working_set(w);
    ALLOC(d.s_hot, (size_t)std::max(NK, 1) * d.s_kstr * sizeof(SchedHot));
    ALLOC(d.s_cold, (size_t)std::max(NK, 1) * d.s_kstr * sizeof(SchedCold));
    ALLOC(d.e_flags, cap);
    ALLOC(d.ext_head, (size_t)cap * 4);
    ALLOC(d.rs_head, (size_t)cap * 4);
    ALLOC(d.fired_mask, (size_t)cap * 4);
    size_t rec_events_per_ent = 0;
    for (int i = 0; i < nro; i++) rec_events_per_ent += w->tab.rec_rows[w->tab.recops[i].rec];
    for (int r = 0; r < NR; r++) {
        ALLOC(d.rcells[r], (size_t)cap * w->tab.rec_rows[r] * w->tab.rec_cols[r] * 8);
        ALLOC(d.rused[r], (size_t)cap * 8);
    }
    ALLOC(w->pl_slot_w, (size_t)cap * 4);
    ALLOC(w->slot_obj_d, (size_t)cap * 4);
    ALLOC(w->fan_desc_w, (size_t)cap * 8);
    d.fan_desc = w->fan_desc_w;
    {
        const char* ab = getenv("NFGPU_ABLATE");
        d.ablate = ab ? (uint32_t)strtoul(ab, nullptr, 0) : 0u;
    }
    d.pl_slot = w->pl_slot_w;
    // output staging sized for every tile of the slot capacity
    d.ev_tcap = kTile * std::max(w->n_dst_union, 1);  // grows for frames with standalone SetProperty groups
    d.fi_tcap = kTile * std::max(NK, 1);
    d.re_tcap = (int32_t)(kRTile * std::max<size_t>(rec_events_per_ent, 1));
    const size_t nt = cap / kTile, nrt = cap / kRTile;
    const size_t ev_n = nt * d.ev_tcap, fi_n = nt * d.fi_tcap, re_n = d.has_recops ? nrt * d.re_tcap : 1;
    ALLOC(d.t_ev, nt * 4);
    ALLOC(d.t_fi, nt * 4);
    ALLOC(d.t_re, nrt * 4);
    ALLOC(d.t_msg, (nt + nrt) * 4);
    ALLOC(d.ev_base, (nt + 1) * 4);
    ALLOC(d.fi_base, (nt + 1) * 4);
    ALLOC(d.re_base, (nrt + 1) * 4);
    ALLOC(d.msg_base, (nt + nrt + 1) * 4);
    ALLOC(d.lb_st, std::min<size_t>(nt, kLbMaxTiles) * 4 * 8);
    ALLOC(d.lb_cnt, 64);
    d.msg_cap = w->cfg.msg_capacity > 0 ? w->cfg.msg_capacity : (int64_t)cap * 32;
    if (d.msg_cap > 0xFFFFFFFFll) return fail(NFK_ERR_ARG, "msg_capacity must fit 32-bit offsets");
    ALLOC(d.ev_slot, ev_n * 4);
    ALLOC(d.ev_pid, ev_n * 4);
    ALLOC(d.ev_old, ev_n * 8);
    ALLOC(d.ev_new, ev_n * 8);
    ALLOC(d.ev_moff, ev_n * 4);
    if (w->cfg.n_obj) {
        ALLOC(d.ev_old_h, ev_n * 8);
        ALLOC(d.ev_new_h, ev_n * 8);
    }
    ALLOC(d.fi_slot, fi_n * 4);
    ALLOC(d.fi_kind, fi_n * 4);
    ALLOC(d.fi_remain, fi_n * 4);
    ALLOC(d.re_rrc, re_n * 4);
    ALLOC(d.re_old, re_n * 8);
    ALLOC(d.re_new, re_n * 8);
    ALLOC(d.re_moff, re_n * 4);
    ALLOC(d.msg_rcpt, d.msg_cap * 4);
    d.tab = w->tab_d;
    d.ctrl = w->ctrl;
    // record ops with their record's arrays and op span (k_records reads them as scalars)
    d.n_rops = nro;
    d.rop_kinds = w->tab.kind_has_recop;
    for (int i = 0; i < nro; i++) {
        const RecOp& ro = w->tab.recops[i];
        RecOpX& x = d.rops[i];
        x.cells = d.rcells[ro.rec];
        x.used = d.rused[ro.rec];
        x.a = ro.a;
        x.b = ro.b;
        x.c = ro.c;
        x.kind = ro.kind;
        x.rec = ro.rec;
        x.col = ro.col;
        x.code = ro.code;
        x.rows = w->tab.rec_rows[ro.rec];
        x.cols = w->tab.rec_cols[ro.rec];
        int f = i, l = i;
        while (f > 0 && w->tab.recops[f - 1].rec == ro.rec) f--;
        while (l + 1 < nro && w->tab.recops[l + 1].rec == ro.rec) l++;
        x.gfirst = f;
        x.glast = l;
    }

    // uploads (synchronous: commit is control plane)
    HIPCHK(hipMemcpy(w->tab_d, &w->tab, sizeof(Tables), hipMemcpyHostToDevice));
    HIPCHK(hipMemset(w->ctrl, 0, sizeof(Ctrl)));
    HIPCHK(hipMemset(d.tally, 0, (size_t)3 * kTallyN * 8 * 8));
    for (const auto& g : pgroups) {
        const size_t gs = g.size();
        std::vector<uint64_t> blk((size_t)cap * gs, 0);
        for (size_t i = 0; i < gs; i++)
            if (!w->init_props[g[i]].empty())
                for (int32_t s = 0; s < d.N; s++)
                    if (w->obj_of_slot[s] >= 0) blk[(size_t)s * gs + i] = w->init_props[g[i]][w->obj_of_slot[s]];
        HIPCHK(hipMemcpy(d.pmem + w->tab.p_off[g[0]], blk.data(), blk.size() * 8, hipMemcpyHostToDevice));
    }
    for (int p = w->n_if; p < w->n_prop; p++) {
        std::vector<uint64_t> blk((size_t)cap * 2, 0);
        if (!w->init_props[p].empty())
            for (int32_t s = 0; s < d.N; s++)
                if (w->obj_of_slot[s] >= 0) {
                    blk[(size_t)s * 2] = w->init_props[p][(size_t)w->obj_of_slot[s] * 2];
                    blk[(size_t)s * 2 + 1] = w->init_props[p][(size_t)w->obj_of_slot[s] * 2 + 1];
                }
        HIPCHK(hipMemcpy(d.pmem + w->tab.p_off[p], blk.data(), blk.size() * 8, hipMemcpyHostToDevice));
    }
    for (int r = 0; r < NR; r++) {
        size_t per = (size_t)w->tab.rec_rows[r] * w->tab.rec_cols[r];
        std::vector<uint64_t> cells(per * cap, 0), used(cap, 0);
        if (!w->init_rcells[r].empty())
            for (int32_t s = 0; s < d.N; s++) {
                int32_t o = w->obj_of_slot[s];
                if (o < 0) continue;
                used[s] = w->init_rused[r][o];
                // each column's vector in packed row order (rec_pos)
                const int rows = w->tab.rec_rows[r], cols = w->tab.rec_cols[r];
                const uint64_t rowm = rec_rowm(rows);
                const uint64_t* src = &w->init_rcells[r][(size_t)o * per];
                uint64_t* dst = &cells[(size_t)s * per];
                for (int c = 0; c < cols; c++)
                    for (int q = 0; q < rows; q++) dst[(size_t)c * rows + rec_pos(used[s], rowm, q)] = src[(size_t)c * rows + q];
            }
        HIPCHK(hipMemcpy(d.rcells[r], cells.data(), cells.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d.rused[r], used.data(), used.size() * 8, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemset(d.s_hot, 0, (size_t)std::max(NK, 1) * d.s_kstr * sizeof(SchedHot)));
    HIPCHK(hipMemset(d.s_cold, 0, (size_t)std::max(NK, 1) * d.s_kstr * sizeof(SchedCold)));
    {
        std::vector<uint64_t> fd(cap, kDeadDesc);
        std::vector<int32_t> pls(cap, 0), so(cap, -1);
        for (size_t i = 0; i < meta.slot.size(); i++) {
            fd[meta.slot[i]] = meta.desc[i];
            pls[meta.slot[i]] = meta.pl[i];
            so[meta.slot[i]] = meta.obj[i];
        }
        HIPCHK(hipMemcpy(w->fan_desc_w, fd.data(), (size_t)cap * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(w->pl_slot_w, pls.data(), (size_t)cap * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(w->slot_obj_d, so.data(), (size_t)cap * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMemset(d.e_flags, 0, cap));
    HIPCHK(hipMemset(d.ext_head, 0, (size_t)cap * 4));
    HIPCHK(hipMemset(d.rs_head, 0, (size_t)cap * 4));
    HIPCHK(hipMemset(d.fired_mask, 0, (size_t)cap * 4));
    HIPCHK(hipMemset(d.t_ev, 0, nt * 4));
    HIPCHK(hipMemset(d.t_fi, 0, nt * 4));
    HIPCHK(hipMemset(d.t_re, 0, nrt * 4));
    HIPCHK(hipMemset(d.t_msg, 0, (nt + nrt) * 4));
    HIPCHK(hipMemset(d.ev_base, 0, (nt + 1) * 4));
    HIPCHK(hipMemset(d.fi_base, 0, (nt + 1) * 4));
    HIPCHK(hipMemset(d.re_base, 0, (nrt + 1) * 4));
    HIPCHK(hipMemset(d.msg_base, 0, (nt + nrt + 1) * 4));
    HIPCHK(hipMemset(d.lb_st, 0, std::min<size_t>(nt, kLbMaxTiles) * 4 * 8));
    HIPCHK(hipMemset(d.lb_cnt, 0, 64));
    w->lb_epoch = 0;
    // creation-time values are now on the device
    for (auto& v : w->init_props) std::vector<uint64_t>().swap(v);
    for (auto& v : w->init_rcells) std::vector<uint64_t>().swap(v);
    build_jit(w);  // k_tick for this schema (hipRTC); the generic kernel stays when it cannot be built
    // room for objects created or imported after commit (every arrival takes a new object index):
    // the per-object vectors and the arrivals' row buffer grow in the background of a frame only
    // after a quarter of the world has arrived, not on the first SwitchScene into this shard
    {
        const size_t room = (size_t)w->n_obj + (size_t)w->n_obj / 4 + 4096;
        w->gh.reserve(room);
        w->gd.reserve(room);
        w->guid.reserve(room);
        w->scene.reserve(room);
        w->group.reserve(room);
        w->cls.reserve(room);
        w->isplayer.reserve(room);
        w->slot_of_obj.reserve(room);
        w->alive.reserve(room);
        w->src_row.reserve(room);
        w->m_flag.reserve(room);
        if (!w->ins_rows) {
            const size_t c = 1024;
            HIPCHK(hipMalloc((void**)&w->ins_rows, c * (size_t)w->row_words * 8));
            w->ins_cap = c;
        }
    }
    w->committed = true;
    return NFK_OK;
}

// the SetProperty* calls of a batch, their objects resolved (obj[i] < 0: no such object; gh / gd
// name it in the error when given): every call is checked before any is queued
static int queue_sets(World* w, int32_t n, const int32_t* obj, const int32_t* pid, const uint64_t* bits,
                      const int64_t* gh, const int64_t* gd) {
    for (int32_t i = 0; i < n; i++) {
        if (obj[i] < 0)  // NFCKernelModule logs "There is no object" and returns false (KM:331)
            return fail(NFK_ERR_NOTFOUND, gh ? "no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i])
                                             : "no object index " + std::to_string(obj[i]));
        if (pid[i] < 0 || pid[i] >= w->n_if)
            return fail(NFK_ERR_ARG, pid[i] >= w->n_if && pid[i] < w->n_prop ? "object property: use nfk_set_objects"
                                                                              : "bad property id");
    }
    const size_t at = w->xops.size();
    w->xops.resize(at + (size_t)n);
    World::XOp* x = w->xops.data() + at;
    for (int32_t i = 0; i < n; i++) {
        x[i] = World::XOp{(uint32_t)obj[i], (uint32_t)pid[i], bits[i]};
        count_standalone(w, (uint32_t)pid[i]);
    }
    if (w->cfg.n_obj) w->xops_h.resize(w->xops.size(), 0);
    return NFK_OK;
}

// object indices as the caller holds them (nfk's creation order, the outputs' ev_obj / fi_obj):
// -1 for one that is not a live object of this world
static const int32_t* live_objects(World* w, int32_t n, const int32_t* obj) {
    w->look.resize(n);
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = obj[i];
        w->look[i] = (o >= 0 && o < w->n_obj && w->alive[o]) ? o : -1;
    }
    return w->look.data();
}

int nfk_set_props(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid,
                  const uint64_t* bits) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !pid || !bits))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    // a large batch in a world without object properties: looked up and queued on the device
    if (w->dev_look_min && (size_t)n >= w->dev_look_min && w->cfg.n_obj == 0) return set_props_dev(w, n, gh, gd, pid, bits);
    w->look.resize(n);  // one GUID lookup per call
    if (int rl = find_many_par(w, n, gh, gd, w->look.data())) return rl;
    return queue_sets(w, n, w->look.data(), pid, bits, gh, gd);
}

int nfk_set_props_obj(void* world, int32_t n, const int32_t* obj, const int32_t* pid, const uint64_t* bits) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!obj || !pid || !bits))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    return queue_sets(w, n, live_objects(w, n, obj), pid, bits, nullptr, nullptr);
}

int nfk_set_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid,
                    const int64_t* vh, const int64_t* vd) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !pid || !vh || !vd))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    w->look.resize(n);
    if (int rl = find_many_par(w, n, gh, gd, w->look.data())) return rl;
    for (int32_t i = 0; i < n; i++) {
        if (w->look[i] < 0)  // "There is no object" (KM:370)
            return fail(NFK_ERR_NOTFOUND, "no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        if (pid[i] < w->n_if || pid[i] >= w->n_prop) return fail(NFK_ERR_ARG, "not an object property");
    }
    // one queue with the int / f64 Sets: the call order across properties is kept
    w->xops_h.resize(w->xops.size(), 0);
    for (int32_t i = 0; i < n; i++) {
        w->xops.push_back(World::XOp{(uint32_t)w->look[i], (uint32_t)pid[i], (uint64_t)vd[i]});
        w->xops_h.push_back((uint64_t)vh[i]);
        count_standalone(w, (uint32_t)pid[i]);
    }
    return NFK_OK;
}

int nfk_set_records(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec,
                    const int32_t* row, const int32_t* col, const uint8_t* is_float, const uint64_t* bits) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !rec || !row || !col || !bits))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    // every call is checked before any is queued; one GUID lookup per call
    w->look.resize(n);
    if (int rl = find_many_par(w, n, gh, gd, w->look.data())) return rl;
    for (int32_t i = 0; i < n; i++) {
        if (w->look[i] < 0)  // NFCKernelModule logs "There is no object" and returns false (KM:505)
            return fail(NFK_ERR_NOTFOUND, "no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        const int32_t r = rec[i];
        if (r < 0 || r >= w->cfg.n_rec || !w->rec_defined[r] || row[i] < 0 || row[i] >= w->tab.rec_rows[r] ||
            col[i] < 0 || col[i] >= w->tab.rec_cols[r])
            return fail(NFK_ERR_ARG, "record cell out of range");
    }
    w->rsq.reserve(w->rsq.size() + n);
    for (int32_t i = 0; i < n; i++) {
        // NFCRecord::SetInt / SetFloat on a column of the other type write nothing (RC:189 / RC:250)
        if (is_float && (is_float[i] != 0) != (w->rec_ctype[rec[i]][col[i]] != 0)) continue;
        w->rq_index[((uint64_t)w->look[i] << 3) | (uint32_t)rec[i]].push_back((uint32_t)w->rsq.size());
        w->rsq.push_back(World::RSOp{(uint32_t)w->look[i], ((uint32_t)rec[i] << 16) | ((uint32_t)row[i] << 8) | (uint32_t)col[i],
                                     bits[i], 0u, 0u});
    }
    return NFK_OK;
}

int nfk_record_rows(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, const int32_t* op,
                    const int32_t* row, const uint64_t* values) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !rec || !op || !row))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    w->look.resize(n);
    if (int rl = find_many_par(w, n, gh, gd, w->look.data())) return rl;
    for (int32_t i = 0; i < n; i++) {
        if (w->look[i] < 0)  // FindRecord: "There is no object" (KM:487)
            return fail(NFK_ERR_NOTFOUND, "no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        const int32_t r = rec[i];
        if (r < 0 || r >= w->cfg.n_rec || !w->rec_defined[r] || op[i] < 1 || op[i] > 3)
            return fail(NFK_ERR_ARG, "bad record or row operation");
        if ((op[i] == 1 && (row[i] < -1 || row[i] >= w->tab.rec_rows[r])) ||
            (op[i] == 2 && (row[i] < 0 || row[i] >= w->tab.rec_rows[r])))
            return fail(NFK_ERR_ARG, "row out of range");
    }
    for (int32_t i = 0; i < n; i++) {
        uint32_t aux = 0;
        const uint32_t rr = op[i] == 3 ? 0u : (row[i] < 0 ? 0xFFu : (uint32_t)row[i]);
        if (op[i] == 1) {
            aux = 0xFFFFFFFFu;
            if (values) {
                aux = (uint32_t)(w->rvals.size() / NFK_MAX_REC_COLS);
                w->rvals.insert(w->rvals.end(), values + (size_t)i * NFK_MAX_REC_COLS,
                                values + (size_t)(i + 1) * NFK_MAX_REC_COLS);
            }
        }
        w->rq_index[((uint64_t)w->look[i] << 3) | (uint32_t)rec[i]].push_back((uint32_t)w->rsq.size());
        w->rsq.push_back(World::RSOp{(uint32_t)w->look[i], ((uint32_t)rec[i] << 16) | (rr << 8), 0ull, (uint32_t)op[i], aux});
    }
    return NFK_OK;
}

// device address of object o's used-row mask of record r (its import row in this window, or its slot)
static int used_addr(World* w, int32_t o, int32_t r, const uint64_t** used) {
    const int rows = w->tab.rec_rows[r], cols = w->tab.rec_cols[r];
    if (w->src_row[o] >= 0) {
        int64_t off = w->n_pw + 4 * w->cfg.n_kind;
        for (int x = 0; x < r; x++) off += (int64_t)w->tab.rec_rows[x] * w->tab.rec_cols[x] + 1;
        *used = w->ins_rows + (size_t)w->src_row[o] * w->row_words + off + (size_t)rows * cols;
    } else if (w->slot_of_obj[o] >= 0) {
        *used = w->d.rused[r] + w->slot_of_obj[o];
    } else {
        return fail(NFK_ERR_STATE, "object without a slot");
    }
    return NFK_OK;
}

// 8-byte device words at absolute addresses (waits for the world's stream)
static int read_abs(World* w, const std::vector<uint64_t>& addr, uint64_t* got) {
    if (addr.empty()) return NFK_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (addr.size() <= 4) {
        for (size_t q = 0; q < addr.size(); q++)
            HIPCHK(hipMemcpy(&got[q], (const void*)(uintptr_t)addr[q], 8, hipMemcpyDeviceToHost));
        return NFK_OK;
    }
    int r = dev_reserve(w, (void**)&w->gat, &w->gat_cap, addr.size() * 16);
    if (r) return r;
    HIPCHK(hipMemcpy(w->gat, addr.data(), addr.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gather_abs, dim3((unsigned)((addr.size() + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream,
                       (const uint64_t*)w->gat, (int32_t)addr.size(), w->gat + addr.size());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(got, w->gat + addr.size(), addr.size() * 8, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    return NFK_OK;
}

// the queued row operations of (object o, record r) replayed on a used-row mask
static uint64_t replay_rows(const World* w, int32_t o, int32_t r, uint64_t u) {
    auto it = w->rq_index.find(((uint64_t)o << 3) | (uint32_t)r);
    if (it == w->rq_index.end()) return u;
    const int rows = w->tab.rec_rows[r];
    for (uint32_t k : it->second) {
        const World::RSOp& x = w->rsq[k];
        const int xr = (int)((x.rrc >> 8) & 0xFF);
        if (x.op == 1) {
            if (xr == 0xFF) {
                const uint64_t fr = ~u & (rows >= 64 ? ~0ull : ((1ull << rows) - 1));
                if (fr) u |= fr & (~fr + 1);
            } else {
                u |= 1ull << xr;
            }
        } else if (x.op == 2) {
            u &= ~(1ull << xr);
        } else if (x.op == 3) {
            u = 0;
        }
    }
    return u;
}

int nfk_get_used_rows(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec, uint64_t* masks) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !rec || !masks))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    std::vector<int32_t> obj(n);
    if (int rl = find_many_par(w, n, gh, gd, obj.data())) return rl;
    std::vector<uint64_t> addr;
    std::vector<int32_t> miss;
    for (int32_t i = 0; i < n; i++) {
        if (obj[i] < 0) return fail(NFK_ERR_NOTFOUND, "There is no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        if (rec[i] < 0 || rec[i] >= w->cfg.n_rec || !w->rec_defined[rec[i]]) return fail(NFK_ERR_ARG, "bad record");
        auto it = w->ucache.find(((uint64_t)obj[i] << 3) | (uint32_t)rec[i]);
        if (it != w->ucache.end()) {
            masks[i] = it->second;
            continue;
        }
        const uint64_t* u;
        int r = used_addr(w, obj[i], rec[i], &u);
        if (r) return r;
        addr.push_back((uint64_t)(uintptr_t)u);
        miss.push_back(i);
    }
    std::vector<uint64_t> got(addr.size());
    int r = read_abs(w, addr, got.data());
    if (r) return r;
    for (size_t q = 0; q < miss.size(); q++) {
        masks[miss[q]] = got[q];
        w->ucache[((uint64_t)obj[miss[q]] << 3) | (uint32_t)rec[miss[q]]] = got[q];
    }
    for (int32_t i = 0; i < n; i++) masks[i] = replay_rows(w, obj[i], rec[i], masks[i]);
    return NFK_OK;
}

int nfk_get_records(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* rec,
                    const int32_t* row, const int32_t* col, uint64_t* bits) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !rec || !row || !col || !bits))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    std::vector<int32_t> obj(n);
    if (int rl = find_many_par(w, n, gh, gd, obj.data())) return rl;
    for (int32_t i = 0; i < n; i++) {
        if (obj[i] < 0) return fail(NFK_ERR_NOTFOUND, "There is no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        const int32_t r = rec[i];
        if (r < 0 || r >= w->cfg.n_rec || !w->rec_defined[r] || row[i] < 0 || row[i] >= w->tab.rec_rows[r] ||
            col[i] < 0 || col[i] >= w->tab.rec_cols[r])
            return fail(NFK_ERR_ARG, "record cell out of range");
    }
    // every query's used-row mask (this window's cache, else one gather), then the cells of the
    // rows the device holds as used in a second: a cell's place in its vector follows from the
    // mask (rec_pos); a row the device holds unused reads 0 unless a queued AddRow writes it
    std::vector<uint64_t> um(n), cv(n, 0);
    {
        std::vector<uint64_t> addr;
        std::vector<int32_t> miss;
        for (int32_t i = 0; i < n; i++) {
            auto it = w->ucache.find(((uint64_t)obj[i] << 3) | (uint32_t)rec[i]);
            if (it != w->ucache.end()) {
                um[i] = it->second;
                continue;
            }
            const uint64_t* u;
            if (int r = used_addr(w, obj[i], rec[i], &u)) return r;
            addr.push_back((uint64_t)(uintptr_t)u);
            miss.push_back(i);
        }
        std::vector<uint64_t> got(addr.size());
        if (int r = read_abs(w, addr, got.data())) return r;
        for (size_t q = 0; q < miss.size(); q++) {
            um[miss[q]] = got[q];
            w->ucache[((uint64_t)obj[miss[q]] << 3) | (uint32_t)rec[miss[q]]] = got[q];
        }
    }
    {
        std::vector<uint64_t> addr;
        std::vector<int32_t> at;
        for (int32_t i = 0; i < n; i++) {
            const int32_t o = obj[i], r = rec[i], rows = w->tab.rec_rows[r], cols = w->tab.rec_cols[r];
            if (!((um[i] >> row[i]) & 1)) continue;
            const size_t place = (size_t)col[i] * rows + rec_pos(um[i], rec_rowm(rows), row[i]);
            const uint64_t* cell;
            if (w->src_row[o] >= 0) {  // entered in this window: its row of the import buffer
                int64_t off = w->n_pw + 4 * w->cfg.n_kind;
                for (int x = 0; x < r; x++) off += (int64_t)w->tab.rec_rows[x] * w->tab.rec_cols[x] + 1;
                cell = w->ins_rows + (size_t)w->src_row[o] * w->row_words + off + place;
            } else if (w->slot_of_obj[o] >= 0) {
                cell = w->d.rcells[r] + (size_t)w->slot_of_obj[o] * cols * rows + place;
            } else {
                return fail(NFK_ERR_STATE, "object without a slot");
            }
            addr.push_back((uint64_t)(uintptr_t)cell);
            at.push_back(i);
        }
        std::vector<uint64_t> got(addr.size());
        if (int r = read_abs(w, addr, got.data())) return r;
        for (size_t q = 0; q < at.size(); q++) cv[at[q]] = got[q];
    }
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = obj[i], r = rec[i], rows = w->tab.rec_rows[r];
        uint64_t u = um[i], c = cv[i];
        // this window's queued calls on the record replayed in call order: SetRecord* through
        // RC:182 / RC:243 on the row's used state at that call, AddRow / Remove / ClearRecord on the
        // used-row mask (RC:111, RC:1086, RC:1109)
        auto it = w->rq_index.find(((uint64_t)o << 3) | (uint32_t)r);
        if (it != w->rq_index.end())
            for (uint32_t k : it->second) {
                const World::RSOp& x = w->rsq[k];
                const int xr = (int)((x.rrc >> 8) & 0xFF), xc = (int)(x.rrc & 0xFF);
                if (x.op == 0) {
                    if (xr != row[i] || xc != col[i] || !((u >> xr) & 1)) continue;
                    const uint64_t b = x.bits;
                    if (w->rec_ctype[r][col[i]]) {
                        double bd, cd;
                        memcpy(&bd, &b, 8);
                        memcpy(&cd, &c, 8);
                        const double df = bd - cd;
                        if (!(df < 0.001 && df > -0.001)) c = b;
                    } else {
                        c = b;
                    }
                } else if (x.op == 1) {
                    int rr = xr;
                    if (xr == 0xFF) {
                        const uint64_t fr = ~u & (rows >= 64 ? ~0ull : ((1ull << rows) - 1));
                        if (!fr) continue;
                        rr = __builtin_ctzll(fr);
                    }
                    u |= 1ull << rr;
                    if (rr == row[i]) c = x.aux == 0xFFFFFFFFu ? 0ull : w->rvals[(size_t)x.aux * NFK_MAX_REC_COLS + col[i]];
                } else if (x.op == 2) {
                    u &= ~(1ull << xr);
                } else {
                    u = 0;
                }
            }
        // NFCRecord::GetInt / GetFloat of an unused row (RC:623): 0
        bits[i] = ((u >> row[i]) & 1) ? c : 0;
    }
    return NFK_OK;
}

int nfk_add_schedules(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* kind,
                      const float* interval, const int32_t* count, const int64_t* now_ms) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !kind || !interval || !count || !now_ms)))
        return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    std::vector<int32_t> obj(n);
    for (int32_t i = 0; i < n; i++) {
        int r = lookup(w, gh[i], gd[i], &obj[i]);
        if (r) return r;
        if (kind[i] < 0 || kind[i] >= w->cfg.n_kind || !w->kind_defined[kind[i]])
            return fail(NFK_ERR_ARG, "undefined heartbeat kind");
    }
    for (int32_t i = 0; i < n; i++)
        w->hops.push_back({1, (uint32_t)obj[i], (uint32_t)kind[i], interval[i], count[i], now_ms[i]});
    return NFK_OK;
}

int nfk_remove_schedule(void* world, int64_t gh, int64_t gd, int32_t kind) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    int32_t obj;
    int r = lookup(w, gh, gd, &obj);
    if (r) return r;
    if (kind < -1 || kind >= w->cfg.n_kind) return fail(NFK_ERR_ARG, "bad kind");
    w->hops.push_back({2, (uint32_t)obj, kind < 0 ? kNoKind : (uint32_t)kind, 0.f, 0, 0});
    return NFK_OK;
}

int nfk_remove_all_schedules(void* world, int64_t gh, int64_t gd) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    int32_t obj;
    int r = lookup(w, gh, gd, &obj);
    if (r) return r;
    w->hops.push_back({3, (uint32_t)obj, 0u, 0.f, 0, 0});
    return NFK_OK;
}

// a batch of schedule calls, their objects resolved (see queue_sets)
static int queue_schedule_calls(World* w, int32_t n, const int32_t* op, const int32_t* obj, const int32_t* kind,
                                const float* interval, const int32_t* count, const int64_t* now_ms, const int64_t* gh,
                                const int64_t* gd) {
    // appended and checked in one pass without a branch per check (the ops of a batch come in no
    // predictable order); a batch with a bad call is taken back out and walked again for the first
    // one's error
    const int32_t nk = w->cfg.n_kind;
    const size_t base = w->hops.size();
    if (w->hops.capacity() < base + (size_t)n)  // (geometric: single calls append one by one)
        w->hops.reserve(std::max(base + (size_t)n, 2 * w->hops.capacity()));
    uint32_t bad = 0;
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = op[i], k = kind[i];
        const bool add = o == 1;
        const bool kin = (uint32_t)k < (uint32_t)nk;
        const bool def = w->kind_defined[kin ? k : 0] && kin;
        bad |= (uint32_t)(obj[i] < 0) | (uint32_t)((uint32_t)(o - 1) > 2u) | (uint32_t)(add && !def) |
               (uint32_t)(o == 2 && (k < -1 || k >= nk));
        w->hops.push_back({o, (uint32_t)obj[i], o == 3 ? 0u : (k < 0 ? kNoKind : (uint32_t)k), add ? interval[i] : 0.f,
                           add ? count[i] : 0, add ? now_ms[i] : 0});
    }
    if (bad) {
        w->hops.resize(base);
        for (int32_t i = 0; i < n; i++) {
            if (obj[i] < 0)
                return fail(NFK_ERR_NOTFOUND, gh ? "no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i])
                                                 : "no object index " + std::to_string(obj[i]));
            if (op[i] < 1 || op[i] > 3) return fail(NFK_ERR_ARG, "schedule call op must be 1, 2 or 3");
            if (op[i] == 1 && (kind[i] < 0 || kind[i] >= w->cfg.n_kind || !w->kind_defined[kind[i]]))
                return fail(NFK_ERR_ARG, "undefined heartbeat kind");
            if (op[i] == 2 && (kind[i] < -1 || kind[i] >= w->cfg.n_kind)) return fail(NFK_ERR_ARG, "bad kind");
        }
        return fail(NFK_ERR_ARG, "bad schedule call");
    }
    return NFK_OK;
}

int nfk_schedule_calls(void* world, int32_t n, const int32_t* op, const int64_t* gh, const int64_t* gd,
                       const int32_t* kind, const float* interval, const int32_t* count, const int64_t* now_ms) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!op || !gh || !gd || !kind || !interval || !count || !now_ms)))
        return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    w->look.resize(n);
    const auto t0 = std::chrono::steady_clock::now();
    if (int rl = find_many_par(w, n, gh, gd, w->look.data())) return rl;
    const auto t1 = std::chrono::steady_clock::now();
    const int r = queue_schedule_calls(w, n, op, w->look.data(), kind, interval, count, now_ms, gh, gd);
    if (trace_calls())
        fprintf(stderr, "schedule_calls n=%d: lookups %.3f ms, queue %.3f ms\n", n, ms_since(t0, t1),
                ms_since(t1, std::chrono::steady_clock::now()));
    return r;
}

int nfk_schedule_calls_obj(void* world, int32_t n, const int32_t* op, const int32_t* obj, const int32_t* kind,
                           const float* interval, const int32_t* count, const int64_t* now_ms) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!op || !obj || !kind || !interval || !count || !now_ms)))
        return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    return queue_schedule_calls(w, n, op, live_objects(w, n, obj), kind, interval, count, now_ms, nullptr, nullptr);
}

// The world's values of property words after the last frame (waits for the world's stream): src
// entries are pmem word offsets, or (1 << 63 | word index in ins_rows) for an object that entered
// in this window; at most 8 single-element reads, else one gather kernel
static int read_words(World* w, const std::vector<uint64_t>& src, uint64_t* got) {
    if (src.empty()) return NFK_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (src.size() <= 8) {
        for (size_t q = 0; q < src.size(); q++) {
            const uint64_t* a = (src[q] >> 63) ? w->ins_rows + (src[q] & ~(1ull << 63)) : w->d.pmem + src[q];
            HIPCHK(hipMemcpy(&got[q], a, 8, hipMemcpyDeviceToHost));
        }
        return NFK_OK;
    }
    int r = dev_reserve(w, (void**)&w->gat, &w->gat_cap, src.size() * 16);
    if (r) return r;
    HIPCHK(hipMemcpy(w->gat, src.data(), src.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gather_words, dim3((unsigned)((src.size() + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream,
                       (const uint64_t*)w->gat, (int32_t)src.size(), (const uint64_t*)w->d.pmem,
                       (const uint64_t*)w->ins_rows, w->gat + src.size());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(got, w->gat + src.size(), src.size() * 8, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    return NFK_OK;
}

// where property word `half` (0 data, 1 head) of pid of object o is read from (see read_words)
static int word_src(World* w, int32_t o, int32_t pid, int half, uint64_t* src) {
    const int32_t sl = w->slot_of_obj[o];
    if (w->src_row[o] >= 0)  // entered in this window: its row of the import buffer
        *src = (1ull << 63) | ((uint64_t)w->src_row[o] * w->row_words + (uint64_t)(prop_word(w, pid) + half));
    else if (sl >= 0)
        *src = (uint64_t)(w->tab.p_off[pid] + (int64_t)sl * w->tab.p_str[pid] + half);
    else
        return fail(NFK_ERR_STATE, "object without a slot");
    return NFK_OK;
}

// index the queued Set calls by (object, property) (ov_last / ov_prev chains, call order)
static int index_queued_sets(World* w) {
    if (int r = pull_device_queue(w)) return r;
    for (size_t i = w->ov_prev.size(); i < w->xops.size(); i++) {
        const uint64_t key = ((uint64_t)w->xops[i].slot << 7) | w->xops[i].pid;
        auto it = w->ov_last.find(key);
        w->ov_prev.push_back(it == w->ov_last.end() ? 0xFFFFFFFFu : it->second);
        w->ov_last[key] = (uint32_t)i;
    }
    return NFK_OK;
}

int nfk_get_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, int64_t* vh,
                    int64_t* vd) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !pid || !vh || !vd))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    std::vector<int32_t> obj(n);
    if (int rl = find_many_par(w, n, gh, gd, obj.data())) return rl;
    std::vector<uint64_t> src(2 * (size_t)n), got(2 * (size_t)n);
    for (int32_t i = 0; i < n; i++) {
        if (obj[i] < 0) return fail(NFK_ERR_NOTFOUND, "There is no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        if (pid[i] < w->n_if || pid[i] >= w->n_prop) return fail(NFK_ERR_ARG, "not an object property");
        for (int h = 0; h < 2; h++) {
            int r = word_src(w, obj[i], pid[i], h, &src[2 * (size_t)i + h]);
            if (r) return r;
        }
    }
    int r = read_words(w, src, got.data());
    if (r) return r;
    // this window's queued SetObject calls on top: NFCProperty::SetObject keeps the last value
    if (int r = index_queued_sets(w)) return r;
    for (int32_t i = 0; i < n; i++) {
        vd[i] = (int64_t)got[2 * (size_t)i];
        vh[i] = (int64_t)got[2 * (size_t)i + 1];
        auto it = w->ov_last.find(((uint64_t)obj[i] << 7) | (uint32_t)pid[i]);
        if (it == w->ov_last.end()) continue;
        vd[i] = (int64_t)w->xops[it->second].bits;
        vh[i] = (int64_t)w->xops_h[it->second];
    }
    return NFK_OK;
}

int nfk_get_props(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* pid, uint64_t* bits) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !pid || !bits))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    std::vector<int32_t> obj(n);
    if (int rl = find_many_par(w, n, gh, gd, obj.data())) return rl;
    for (int32_t i = 0; i < n; i++) {
        if (obj[i] < 0) return fail(NFK_ERR_NOTFOUND, "There is no object " + std::to_string(gh[i]) + "-" + std::to_string(gd[i]));
        if (pid[i] < 0 || pid[i] >= w->n_if) return fail(NFK_ERR_ARG, "bad property id (object properties: nfk_get_objects)");
    }
    // 1. the world's values after the last frame (a per-window cache of device reads)
    std::vector<uint64_t> src;
    std::vector<int32_t> miss;
    for (int32_t i = 0; i < n; i++) {
        const uint64_t key = ((uint64_t)obj[i] << 7) | (uint32_t)pid[i];
        auto it = w->dcache.find(key);
        if (it != w->dcache.end()) {
            bits[i] = it->second;
            continue;
        }
        uint64_t a;
        int r = word_src(w, obj[i], pid[i], 0, &a);
        if (r) return r;
        src.push_back(a);
        miss.push_back(i);
    }
    if (!miss.empty()) {
        std::vector<uint64_t> got(miss.size());
        int r = read_words(w, src, got.data());
        if (r) return r;
        for (size_t q = 0; q < miss.size(); q++) {
            const int32_t i = miss[q];
            bits[i] = got[q];
            w->dcache[((uint64_t)obj[i] << 7) | (uint32_t)pid[i]] = got[q];
        }
    }
    // 2. this window's queued writes of the property on top, in call order (PR:254 / PR:295)
    if (int r = index_queued_sets(w)) return r;
    std::vector<uint32_t> chain;
    for (int32_t i = 0; i < n; i++) {
        auto it = w->ov_last.find(((uint64_t)obj[i] << 7) | (uint32_t)pid[i]);
        if (it == w->ov_last.end()) continue;
        chain.clear();
        for (uint32_t x = it->second; x != 0xFFFFFFFFu; x = w->ov_prev[x]) chain.push_back(x);
        uint64_t v = bits[i];
        for (size_t c = chain.size(); c-- > 0;) {
            const uint64_t b = w->xops[chain[c]].bits;
            if (pid[i] < w->cfg.n_int) {
                v = b;
            } else {
                double bd, vd;
                memcpy(&bd, &b, 8);
                memcpy(&vd, &v, 8);
                if (!(fabs(bd - vd) <= 1e-15)) v = b;
            }
        }
        bits[i] = v;
    }
    return NFK_OK;
}

int nfk_exist_schedule(void* world, int64_t gh, int64_t gd, int32_t kind, int32_t* exists) {
    World* w = (World*)world;
    if (!w || !exists) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    if (kind < 0 || kind >= w->cfg.n_kind) return fail(NFK_ERR_ARG, "bad kind");
    *exists = 0;
    const int32_t o = w->obj_of.find(gh, gd);
    if (o < 0) return NFK_OK;  // no schedule map for the object
    for (const auto& h : w->hops)
        if (h.code == 3 && h.slot == (uint32_t)o) return NFK_OK;  // RemoveSchedule(self) erased it
    uint64_t word = 0;
    HIPCHK(hipStreamSynchronize(w->stream));
    if (w->src_row[o] >= 0) {
        HIPCHK(hipMemcpy(&word, w->ins_rows + (size_t)w->src_row[o] * w->row_words + w->n_pw + 4 * kind + 1, 8,
                         hipMemcpyDeviceToHost));
    } else if (w->slot_of_obj[o] >= 0) {
        HIPCHK(hipMemcpy(&word, (const char*)(w->d.s_hot + (size_t)kind * w->d.s_kstr + w->slot_of_obj[o]) + 8, 8,
                         hipMemcpyDeviceToHost));
    }
    *exists = (int32_t)((word >> 32) & kStPresent);
    return NFK_OK;
}

int nfk_watch_props(void* world, int32_t n, const int32_t* pid) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && !pid)) return fail(NFK_ERR_ARG, "null argument");
    uint64_t m[2] = {0, 0};
    for (int32_t i = 0; i < n; i++) {
        if (pid[i] < 0 || pid[i] >= w->n_if) return fail(NFK_ERR_ARG, "nfk_watch_props: not an int / f64 property");
        m[pid[i] >> 6] |= 1ull << (pid[i] & 63);
    }
    w->chain_watch[0] = m[0];
    w->chain_watch[1] = m[1];
    return NFK_OK;
}

static int update_guid_ranks(World* w);

int nfk_read_chain(void* world, int32_t cap, int32_t* n, int32_t* obj, int32_t* kind, int32_t* op, int32_t* pid,
                   uint64_t* old_bits, uint64_t* new_bits) {
    World* w = (World*)world;
    if (!w || !n || cap < 0) return fail(NFK_ERR_ARG, "null argument");
    *n = 0;
    if (!w->chain_ran) return NFK_OK;
    // the tiles' counts -> dense bases (and the total), on the world's stream after the frame
    const int32_t nt = w->chain_tiles;
    const size_t s_db = 0, s_k1 = (((size_t)nt + 1) * 4 + 255) & ~(size_t)255;
    if (s_k1 > w->chain_scap) {
        HIPCHK(hipStreamSynchronize(w->stream));
        if (w->chain_scr) HIPCHK(hipFree(w->chain_scr));
        w->chain_scr = nullptr;
        w->chain_scap = s_k1 + 4096;
        HIPCHK(hipMalloc(&w->chain_scr, w->chain_scap));
    }
    uint32_t* db = (uint32_t*)((char*)w->chain_scr + s_db);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, w->stream, w->chain_cnt_d, db, nt);
    uint32_t cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, db + nt, sizeof(cnt), hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    *n = (int32_t)cnt;
    const uint32_t m = std::min<uint32_t>(cnt, (uint32_t)cap);
    if (!m) return NFK_OK;
    if (!obj || !kind || !op || !pid || !old_bits || !new_bits) return fail(NFK_ERR_ARG, "null argument");
    // walk order: (NFGUID rank of the object, kind, op) keys sorted on the device, the entries
    // gathered in that order as object-index columns, one copy back
    int r = update_guid_ranks(w);
    if (r) return r;
    int key_bits = 8;
    while ((1ll << (key_bits - 8)) < (long long)std::max(w->n_obj, 1)) key_bits++;
    size_t sort_bytes = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                     (uint32_t*)nullptr, cnt, 0, key_bits, w->stream));
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t s_k2 = s_k1 + al((size_t)cnt * 8), s_i1 = s_k2 + al((size_t)cnt * 8), s_i2 = s_i1 + al((size_t)cnt * 4);
    const size_t s_out = s_i2 + al((size_t)cnt * 4), s_tmp = s_out + al((size_t)cnt * 32);
    const size_t need = s_tmp + sort_bytes + 256, pin = (size_t)cnt * 32;
    if (need > w->chain_scap || pin > w->chain_pcap) {
        // (db survives: the scan is redone into the new scratch)
        HIPCHK(hipStreamSynchronize(w->stream));
        if (need > w->chain_scap) {
            HIPCHK(hipFree(w->chain_scr));
            w->chain_scr = nullptr;
            w->chain_scap = need + need / 4 + 4096;
            HIPCHK(hipMalloc(&w->chain_scr, w->chain_scap));
            db = (uint32_t*)((char*)w->chain_scr + s_db);
            hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, w->stream, w->chain_cnt_d, db, nt);
        }
        if (pin > w->chain_pcap) {
            if (w->chain_pin) HIPCHK(hipHostFree(w->chain_pin));
            w->chain_pin = nullptr;
            w->chain_pcap = pin + pin / 4 + 4096;
            HIPCHK(hipHostMalloc((void**)&w->chain_pin, w->chain_pcap, hipHostMallocDefault));
        }
    }
    char* S = (char*)w->chain_scr;
    uint64_t* k1 = (uint64_t*)(S + s_k1);
    uint64_t* k2 = (uint64_t*)(S + s_k2);
    uint32_t* i1 = (uint32_t*)(S + s_i1);
    uint32_t* i2 = (uint32_t*)(S + s_i2);
    const unsigned gt = (unsigned)std::max(1, std::min(nt, 4096));
    hipLaunchKernelGGL(k_chain_keys, dim3(gt), dim3(kTPB), 0, w->stream, (const ChainEnt*)w->chain_d, (const uint32_t*)db, nt,
                       w->chain_tcap, (const int32_t*)w->slot_obj_d, (const int32_t*)w->rank_d, k1, i1);
    size_t sb = sort_bytes;
    if (cnt <= (uint32_t)kSmallPairs)
        hipLaunchKernelGGL(k_sort_small_pairs, dim3((cnt + kTPB - 1) / kTPB), dim3(kTPB), 0, w->stream, (const uint64_t*)k1,
                           k2, (const uint32_t*)i1, i2, (int)cnt);
    else
        HIPCHK(rocprim::radix_sort_pairs(S + s_tmp, sb, k1, k2, i1, i2, cnt, 0, key_bits, w->stream));
    int32_t* oi = (int32_t*)(S + s_out);
    uint64_t* ou = (uint64_t*)(S + s_out + (size_t)cnt * 16);
    hipLaunchKernelGGL(k_chain_gather, dim3((cnt + kTPB - 1) / kTPB), dim3(kTPB), 0, w->stream, (const ChainEnt*)w->chain_d,
                       (const uint32_t*)i2, (int)cnt, (const int32_t*)w->slot_obj_d, oi, ou);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(w->chain_pin, S + s_out, (size_t)cnt * 32, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    const int32_t* hi = (const int32_t*)w->chain_pin;
    const uint64_t* hu = (const uint64_t*)(w->chain_pin + (size_t)cnt * 16);
    memcpy(obj, hi, (size_t)m * 4);
    memcpy(kind, hi + cnt, (size_t)m * 4);
    memcpy(op, hi + 2 * (size_t)cnt, (size_t)m * 4);
    memcpy(pid, hi + 3 * (size_t)cnt, (size_t)m * 4);
    memcpy(old_bits, hu, (size_t)m * 8);
    memcpy(new_bits, hu + cnt, (size_t)m * 8);
    return NFK_OK;
}

int nfk_read_added(void* world, int32_t cap, int32_t* n, int64_t* gh, int64_t* gd, int32_t* kind) {
    World* w = (World*)world;
    if (!w || !n || cap < 0 || (cap && (!gh || !gd || !kind))) return fail(NFK_ERR_ARG, "null argument");
    *n = 0;
    if (!w->hf_pending) return NFK_OK;
    // the last pass's post-scan entries (the device fold's): which AddSchedule created a schedule
    HIPCHK(hipStreamSynchronize(w->stream));
    uint32_t np = 0;
    HIPCHK(hipMemcpy(&np, w->hf_npost, 4, hipMemcpyDeviceToHost));
    np = std::min<uint32_t>(np, (uint32_t)w->hf_max);
    if (np == 0) return NFK_OK;
    std::vector<uint32_t> sl(np), kd(np), op(np);
    std::vector<uint8_t> added(np);
    HIPCHK(hipMemcpy(sl.data(), w->hf_pslot, np * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(kd.data(), w->hf_pkind, np * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(op.data(), w->hf_pop, np * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(added.data(), w->hf_added, np, hipMemcpyDeviceToHost));
    int32_t k = 0;
    for (uint32_t i = 0; i < np; i++) {
        if (!added[i] || !(op[i] & 2u) || sl[i] >= w->obj_of_slot.size()) continue;
        const int32_t o = w->obj_of_slot[sl[i]];
        if (o < 0) continue;
        if (k < cap) {
            gh[k] = w->gh[o];
            gd[k] = w->gd[o];
            kind[k] = (int32_t)kd[i];
        }
        k++;
    }
    *n = k;
    return NFK_OK;
}

int nfk_set_scene_props(void* world, int32_t pid_scene, int32_t pid_group, int32_t pid_x, int32_t pid_y,
                        int32_t pid_z) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    const int NI = w->cfg.n_int;
    auto ok_i = [&](int32_t p) { return p == -1 || (p >= 0 && p < NI); };
    auto ok_f = [&](int32_t p) { return p == -1 || (p >= NI && p < w->n_if); };
    if (!ok_i(pid_scene) || !ok_i(pid_group) || !ok_f(pid_x) || !ok_f(pid_y) || !ok_f(pid_z))
        return fail(NFK_ERR_ARG, "SceneID/GroupID must be int properties, X/Y/Z float properties");
    w->pid_scene = pid_scene;
    w->pid_group = pid_group;
    w->pid_x = pid_x;
    w->pid_y = pid_y;
    w->pid_z = pid_z;
    return NFK_OK;
}

int nfk_switch_scene(void* world, int64_t gh, int64_t gd, int32_t scene, int32_t group, float x, float y, float z) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    int32_t o;
    int r = lookup(w, gh, gd, &o);
    if (r) return r;  // "There is no object" (KM:948)
    if (group < 0) return fail(NFK_ERR_ARG, "negative group");
    // the property writes of KM:931-942, in call order (queued like SetProperty*)
    auto put = [&](int32_t pid, uint64_t bits) {
        if (pid >= 0) {
            w->xops.push_back({(uint32_t)o, (uint32_t)pid, bits});
            count_standalone(w, (uint32_t)pid);
        }
    };
    auto dbits = [](double v) {
        uint64_t u;
        memcpy(&u, &v, 8);
        return u;
    };
    if (scene != w->scene[o]) {
        put(w->pid_group, 0);
        put(w->pid_scene, (uint64_t)(int64_t)scene);
    }
    put(w->pid_x, dbits((double)x));
    put(w->pid_y, dbits((double)y));
    put(w->pid_z, dbits((double)z));
    put(w->pid_group, (uint64_t)(int64_t)group);
    // RemoveObjectFromGroup + AddObjectToGroup (KM:928, 944): a new slot in the target group
    if (scene != w->scene[o] || group != w->group[o]) {
        w->scene[o] = scene;
        w->group[o] = group;
        touch(w, o);
    }
    return NFK_OK;
}

int nfk_destroy_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    for (int32_t i = 0; i < n; i++) {
        int32_t o;
        int r = lookup(w, gh[i], gd[i], &o);
        if (r) return r;
    }
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = w->obj_of.find(gh[i], gd[i]);
        w->obj_of.erase(gh[i], gd[i]);
        w->alive[o] = 0;
        touch(w, o);
    }
    return NFK_OK;
}

int nfk_object_count(void* world, int32_t* n) {
    World* w = (World*)world;
    if (!w || !n) return fail(NFK_ERR_ARG, "null argument");
    *n = w->n_obj;
    return NFK_OK;
}

int nfk_row_words(void* world, int32_t* words) {
    World* w = (World*)world;
    if (!w || !words) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    *words = w->row_words;
    return NFK_OK;
}

int nfk_export_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, uint64_t* rows_dev) {
    World* w = (World*)world;
    if (!w || n < 0 || (n && (!gh || !gd || !rows_dev))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    if (n == 0) return NFK_OK;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::vector<int32_t> src(n), objs(n);
    for (int32_t i = 0; i < n; i++) {
        int r = lookup(w, gh[i], gd[i], &objs[i]);
        if (r) return r;
        if (w->m_flag[objs[i]] || w->slot_of_obj[objs[i]] < 0)
            return fail(NFK_ERR_STATE, "export of an object whose membership already changed in this window");
        src[i] = w->slot_of_obj[objs[i]];
    }
    const auto t1 = clk::now();
    // the slot list from pinned host memory (the last export's k_pack has read its copy)
    if (!w->xpin_done) HIPCHK(hipEventCreateWithFlags(&w->xpin_done, hipEventDisableTiming));
    if (w->xpin_pending) {
        HIPCHK(hipEventSynchronize(w->xpin_done));
        w->xpin_pending = false;
    }
    if ((size_t)n > w->xpin_cap) {
        if (w->xpin) HIPCHK(hipHostFree(w->xpin));
        w->xpin = nullptr;
        const size_t c = std::max<size_t>((size_t)n, 2 * w->xpin_cap);
        w->xpin_cap = 0;  // (until the new buffer exists)
        HIPCHK(hipHostMalloc((void**)&w->xpin, c * sizeof(int32_t), hipHostMallocDefault));
        HIPCHK(hipHostGetDevicePointer((void**)&w->xpin_dev, w->xpin, 0));
        w->xpin_cap = c;
    }
    memcpy(w->xpin, src.data(), (size_t)n * sizeof(int32_t));
    const auto t2 = clk::now();
    hipLaunchKernelGGL(k_pack, dim3(grid_for((size_t)n * w->row_words)), dim3(kTPB), 0, w->stream, w->d,
                       (const int32_t*)w->xpin_dev, n, w->row_words, rows_dev);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(w->xpin_done, w->stream));
    w->xpin_pending = true;
    const auto t3 = clk::now();
    for (int32_t i = 0; i < n; i++) {
        w->obj_of.erase(gh[i], gd[i]);
        w->alive[objs[i]] = 0;
        touch(w, objs[i]);
    }
    if (getenv("NFGPU_TRACE_MEMBERSHIP")) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "nfk_export_objects: %d rows, lookup %.3f ms, upload %.3f ms, launch %.3f ms, unmap %.3f ms\n", n,
                ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, clk::now()));
    }
    return NFK_OK;
}

static int import_common(World* w, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* scene,
                         const int32_t* group, const uint8_t* cls, const uint8_t* isplayer, const void* rows,
                         hipMemcpyKind kind) {
    if (n < 0 || (n && (!gh || !gd || !scene || !group || !cls || !isplayer || !rows)))
        return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first (before it, use nfk_create_objects)");
    if (n == 0) return NFK_OK;
    for (int32_t i = 0; i < n; i++) {
        if (cls[i] >= w->cfg.n_class) return fail(NFK_ERR_ARG, "class id out of range");
        if (group[i] < 0) return fail(NFK_ERR_ARG, "negative group");
        if (w->obj_of.count(gh[i], gd[i])) return fail(NFK_ERR_ARG, "The object has Exists");  // KM:131
        for (int32_t j = 0; j < i; j++)
            if (gh[j] == gh[i] && gd[j] == gd[i]) return fail(NFK_ERR_ARG, "The object has Exists");
    }
    const size_t rb = (size_t)w->row_words * 8;
    if (w->ins_n + n > w->ins_cap) {
        // grow, keeping this window's earlier rows
        const size_t c = std::max(w->ins_n + n, w->ins_cap * 2);
        uint64_t* p = nullptr;
        HIPCHK(hipMalloc((void**)&p, c * rb));
        if (w->ins_n) HIPCHK(hipMemcpyAsync(p, w->ins_rows, w->ins_n * rb, hipMemcpyDeviceToDevice, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        if (w->ins_rows) HIPCHK(hipFree(w->ins_rows));
        w->ins_rows = p;
        w->ins_cap = c;
    }
    HIPCHK(hipMemcpyAsync(w->ins_rows + w->ins_n * w->row_words, rows, (size_t)n * rb, kind, w->stream));
    if (kind == hipMemcpyHostToDevice) HIPCHK(hipStreamSynchronize(w->stream));
    for (int32_t i = 0; i < n; i++) {
        const int32_t o = add_object(w, gh[i], gd[i], scene[i], group[i], cls[i], isplayer[i]);
        w->src_row[o] = (int64_t)(w->ins_n + i);
        touch(w, o);
    }
    w->ins_n += n;
    return NFK_OK;
}

int nfk_import_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* scene,
                       const int32_t* group, const uint8_t* cls, const uint8_t* isplayer, const uint64_t* rows_dev) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    return import_common(w, n, gh, gd, scene, group, cls, isplayer, rows_dev, hipMemcpyDeviceToDevice);
}

int nfk_spawn_objects(void* world, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* scene,
                      const int32_t* group, const uint8_t* cls, const uint8_t* isplayer, const uint64_t* props) {
    World* w = (World*)world;
    if (!w || (n > 0 && !props)) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first (before it, use nfk_create_objects)");
    std::vector<uint64_t> rows((size_t)std::max(n, 0) * w->row_words, 0);
    for (int32_t i = 0; i < n; i++)
        memcpy(&rows[(size_t)i * w->row_words], props + (size_t)i * w->n_pw, (size_t)w->n_pw * 8);
    return import_common(w, n, gh, gd, scene, group, cls, isplayer, rows.data(), hipMemcpyHostToDevice);
}

// one device pass over the window's queued calls; calls_only: nfk_execute_calls (nothing fires,
// k_tick runs only the tiles with SetProperty groups)
static int execute_frame(World* w, int64_t now_ms, bool calls_only) {
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    // a device error of an earlier frame (host-mapped, no device read): that frame's outputs are
    // incomplete, so no further frame runs until nfk_summary_get has reported and cleared it
    if (const unsigned e = err_host_bits(w); e & (kErrFanBound | kErrTouch))
        return fail(NFK_ERR_DEVICE, std::string("device error of an earlier frame: ") +
                                        ((e & kErrFanBound) ? "a tile's fan-out exceeded its bound" : "touch list overflow") +
                                        " (nfk_summary_get reports and clears it)");
    using clk = std::chrono::steady_clock;
    const bool trace = getenv("NFGPU_TRACE_EXEC") != nullptr;  // host phases to stderr
    clk::time_point tp[6];
    tp[0] = clk::now();
    // ---- membership changes of this window ----
    {
        // the window's host plan overlaps the previous frame still on the GPU; its device phase
        // follows the wait for that frame
        if (!w->mplan) w->mplan.reset(new MemPlan());
        MemPlan& mp = *w->mplan;
        int r = plan_membership(w, mp);
        if (r) return r;  // nothing of the window applied; its calls stay queued
        const int rf = check_fanout(w);  // the last frame's fan-out is complete before it is replaced
        r = commit_membership(w, mp);    // (a planned window is applied either way)
        if (rf) return drop_window(w, rf);
        if (r) return drop_window(w, r);
    }
    // test hook: a failure right after the window's membership changes (tests/test_gpu_parity.py)
    if (const char* inj = getenv("NFGPU_INJECT_EXEC_FAIL"); inj && inj[0] == '1')
        return drop_window(w, fail(NFK_ERR_CAPACITY, "injected failure after the membership changes"));
    if (w->cfg.n_obj) w->xops_h.resize(w->xops.size(), 0);
    Dev d = w->d;
    d.now = now_ms;

    tp[1] = clk::now();
    // ---- host-side preparation of queued calls ----
    // Queued calls hold object indices; each resolves to its slot after the window's membership
    // changes (a destroyed / exported object's calls are dropped: "There is no object").  Calls
    // are folded by a stable radix sort of packed words (key << ib | call index), ib = the bits
    // of the largest call index, so the sort moves one array and keeps call order within a key.
    //
    // SetProperty*: (slot, property) groups, each group's calls in call order, folded on the
    // device (k_xkeys, radix sort, k_scan_heads, k_xgroups below): the host hands the calls over as
    // queued.  A tile's events are its slots' program destinations plus its standalone groups
    // (properties no program writes); those are bounded here without the slots: at most one per
    // standalone call, and at most one per slot and standalone property the window sets.
    // (the window's SetProperty calls: xq_n on the device queue, then the host's)
    const size_t n_xdev = w->xq_n, n_xq = n_xdev + w->xops.size(), n_hq = w->hops.size();
    const int64_t max_sa = n_xq ? std::min<int64_t>(w->sa_calls, (int64_t)kTile * (__builtin_popcountll(w->sa_pids[0]) +
                                                                                   __builtin_popcountll(w->sa_pids[1])))
                                : 0;
    // a tile's events: its slots' program destinations plus its standalone Set groups
    {
        const int64_t need_ev = (int64_t)kTile * std::max(w->n_dst_union, 1) + max_sa;
        if (need_ev > w->d.ev_tcap) {
            int r = grow_event_tiles(w, need_ev);
            if (r) return drop_window(w, r);
            d.ev_tcap = w->d.ev_tcap;
            d.ev_slot = w->d.ev_slot; d.ev_pid = w->d.ev_pid; d.ev_old = w->d.ev_old;
            d.ev_new = w->d.ev_new; d.ev_moff = w->d.ev_moff;
            d.ev_old_h = w->d.ev_old_h; d.ev_new_h = w->d.ev_new_h;
        }
    }
    // SetRecordInt / SetRecordFloat: (slot, cell) groups, each group's calls in call order (key
    // slot << 19 | rec << 16 | row << 8 | col).  Record row operations (AddRow / Remove /
    // ClearRecord): one list per (slot, record) that has any, with every call on that pair (its
    // SetRecord calls too, whose groups k_rsets then leaves to k_rrows: rs_rrc bit 31) in call
    // order.  The slots with groups or lists, in slot order, are each run by k_rset_slots; a record
    // tile's extra events are bounded by its groups plus its lists' row events.
    const size_t n_rq = w->rsq.size();
    std::vector<uint32_t>& rs_slot = w->rs_slot_h;
    std::vector<uint32_t>& rs_rrc = w->rs_rrc_h;
    std::vector<uint32_t>& rs_first = w->rs_first_h;
    std::vector<uint32_t>& rss_slot = w->rss_slot_h;
    std::vector<uint32_t>& rss_g0 = w->rss_g0_h;
    rs_slot.clear();
    rs_rrc.clear();
    rs_first.clear();
    rss_slot.clear();
    rss_g0.clear();
    std::vector<uint32_t> rss_l0, rl_slot, rl_rec, rl_c0, rl_ev0, rc_code, rc_aux;
    std::vector<uint64_t> rc_bits;
    std::vector<uint64_t>& rowpairs = w->rowpairs;
    rowpairs.clear();
    std::vector<uint64_t>& rpk = w->rpk;
    rpk.clear();
    const int rib = bits_for(n_rq);
    const uint64_t rim = (1ull << rib) - 1;
    int64_t max_rs_tile = 0;
    size_t n_rev = 0;  // row-event bound of the window
    if (n_rq) {
        for (size_t i = 0; i < n_rq; i++)
            if (w->rsq[i].op) {
                const int32_t sl = w->slot_of_obj[w->rsq[i].obj];
                if (sl >= 0) rowpairs.push_back(((uint64_t)(uint32_t)sl << 3) | (w->rsq[i].rrc >> 16));
            }
        std::sort(rowpairs.begin(), rowpairs.end());
        rowpairs.erase(std::unique(rowpairs.begin(), rowpairs.end()), rowpairs.end());
        auto pair_of = [&](uint32_t sl, uint32_t rec) -> int64_t {
            if (rowpairs.empty()) return -1;
            const uint64_t key = ((uint64_t)sl << 3) | rec;
            auto it = std::lower_bound(rowpairs.begin(), rowpairs.end(), key);
            return (it != rowpairs.end() && *it == key) ? (int64_t)(it - rowpairs.begin()) : -1;
        };
        rpk.resize(n_rq);
        uint64_t kor = 0;
        size_t k = 0;
        for (size_t i = 0; i < n_rq; i++) {
            if (w->rsq[i].op) continue;
            const int32_t sl = w->slot_of_obj[w->rsq[i].obj];
            if (sl < 0) continue;  // destroyed / exported in this window
            const uint64_t key = ((uint64_t)(uint32_t)sl << 19) | w->rsq[i].rrc;
            kor |= key;
            rpk[k++] = (key << rib) | i;
        }
        rpk.resize(k);
        if (bits_for(kor) + rib > 64) return drop_window(w, fail(NFK_ERR_CAPACITY, "too many queued SetRecord calls"));
        radix_sort_packed(rpk, w->rpk_t, rib, bits_for(kor));
        uint64_t prev = ~0ull;
        for (size_t i = 0; i < k; i++) {
            const uint64_t key = rpk[i] >> rib;
            if (key == prev) continue;
            prev = key;
            const uint32_t sl = (uint32_t)(key >> 19), rrc = (uint32_t)(key & 0x7FFFF);
            rs_slot.push_back(sl);
            rs_rrc.push_back(rrc | (pair_of(sl, rrc >> 16) >= 0 ? 0x80000000u : 0u));
            rs_first.push_back((uint32_t)i);
        }
        rs_first.push_back((uint32_t)k);
        // the row-operation lists (one per pair, pair order), their calls in call order
        const size_t npair = rowpairs.size();
        if (npair) {
            std::vector<uint32_t> cnt(npair + 1, 0);
            std::vector<int64_t> call_pair(n_rq, -1);
            for (size_t i = 0; i < n_rq; i++) {
                const int32_t sl = w->slot_of_obj[w->rsq[i].obj];
                if (sl < 0) continue;
                call_pair[i] = pair_of((uint32_t)sl, w->rsq[i].rrc >> 16);
                if (call_pair[i] >= 0) cnt[call_pair[i]]++;
            }
            rl_c0.assign(npair + 1, 0);
            for (size_t q = 0; q < npair; q++) rl_c0[q + 1] = rl_c0[q] + cnt[q];
            rc_code.assign(rl_c0[npair], 0);
            rc_aux.assign(rl_c0[npair], 0);
            rc_bits.assign(rl_c0[npair], 0);
            rl_ev0.assign(npair, 0);
            std::vector<uint32_t> fill(rl_c0.begin(), rl_c0.end() - 1), evb(npair, 0);
            for (size_t i = 0; i < n_rq; i++) {
                if (call_pair[i] < 0) continue;
                const World::RSOp& x = w->rsq[i];
                const int64_t q = call_pair[i];
                const uint32_t at = fill[q]++;
                const uint32_t rec = x.rrc >> 16, row = (x.rrc >> 8) & 0xFF, col = x.rrc & 0xFF;
                rc_code[at] = x.op | (row << 8) | (col << 16);
                rc_bits[at] = x.bits;
                if (x.op == 0) {  // its cell's group (binary search over the sorted groups)
                    const uint64_t key = ((uint64_t)(rowpairs[q] >> 3) << 19) | (x.rrc & 0x7FFFF);
                    size_t lo = 0, hi = rs_slot.size();
                    while (lo < hi) {
                        const size_t m = (lo + hi) / 2;
                        const uint64_t km = ((uint64_t)rs_slot[m] << 19) | (rs_rrc[m] & 0x7FFFF);
                        if (km < key) lo = m + 1;
                        else hi = m;
                    }
                    rc_aux[at] = (uint32_t)lo;
                } else {
                    rc_aux[at] = x.aux;
                    evb[q] += x.op == 3 ? (uint32_t)w->tab.rec_rows[rec] : 1u;
                }
            }
            for (size_t q = 0; q < npair; q++) {
                rl_slot.push_back((uint32_t)(rowpairs[q] >> 3));
                rl_rec.push_back((uint32_t)(rowpairs[q] & 7));
                rl_ev0[q] = (uint32_t)n_rev;
                n_rev += evb[q];
            }
            // the tile bound: per record tile, its groups plus its lists' row-event bounds
            std::vector<std::pair<uint32_t, uint32_t>> per_tile;  // (record tile, events)
            for (size_t g = 0; g < rs_slot.size(); g++) per_tile.push_back({rs_slot[g] / kRTile, 1u});
            for (size_t q = 0; q < npair; q++) per_tile.push_back({rl_slot[q] / kRTile, evb[q]});
            std::sort(per_tile.begin(), per_tile.end());
            for (size_t a = 0; a < per_tile.size();) {
                int64_t t = 0;
                size_t b = a;
                for (; b < per_tile.size() && per_tile[b].first == per_tile[a].first; b++) t += per_tile[b].second;
                max_rs_tile = std::max(max_rs_tile, t);
                a = b;
            }
        } else {
            uint32_t cur_rt = 0xFFFFFFFFu;
            int64_t tile_groups = 0;
            for (size_t g = 0; g < rs_slot.size(); g++) {
                if (rs_slot[g] / kRTile != cur_rt) {
                    cur_rt = rs_slot[g] / kRTile;
                    tile_groups = 0;
                }
                max_rs_tile = std::max(max_rs_tile, ++tile_groups);
            }
        }
        // the slots with record work: groups or lists, in slot order
        for (size_t gi = 0, pi = 0; gi < rs_slot.size() || pi < rl_slot.size();) {
            const uint32_t sl = std::min(gi < rs_slot.size() ? rs_slot[gi] : 0xFFFFFFFFu,
                                         pi < rl_slot.size() ? rl_slot[pi] : 0xFFFFFFFFu);
            rss_slot.push_back(sl);
            rss_g0.push_back((uint32_t)gi);
            rss_l0.push_back((uint32_t)pi);
            while (gi < rs_slot.size() && rs_slot[gi] == sl) gi++;
            while (pi < rl_slot.size() && rl_slot[pi] == sl) pi++;
        }
        // a record tile's events: its slots' record-program cells plus its SetRecord groups
        int64_t cells = 0;
        for (int j = 0; j < d.n_rops; j++) cells += d.rops[j].rows;
        const int64_t need_re = (int64_t)kRTile * std::max<int64_t>(cells, 1) + max_rs_tile;
        if (need_re > w->d.re_tcap) {
            int r = grow_rec_tiles(w, need_re);
            if (r) return drop_window(w, r);
            d.re_tcap = w->d.re_tcap;
            d.re_rrc = w->d.re_rrc; d.re_old = w->d.re_old;
            d.re_new = w->d.re_new; d.re_moff = w->d.re_moff;
        }
    }
    const size_t ngr = rs_slot.size(), nrss = rss_slot.size(), nrc = rpk.size();
    tp[2] = clk::now();
    // schedule calls: pre-scan entries (remove-list key owner, RemoveSchedule(self)) and post-scan
    // (slot, kind) entries (remove, add), folded on the device (k_hkeys, radix sort, k_hfold;
    // nfgpu_kernels.hip states the reference's rules).  Their counts stay on the device: k_pre_hostops
    // and k_post_hostops read them, nfk_read_added reads them back.

    // k_tick runs the programs on the working set fixed at commit (Dev::u_*); a schema whose
    // working set does not fit the register slots runs k_tick_touch
    const bool use_u = w->u_ok && !(d.ablate & kAblPerKind);
    // a calls-only pass runs k_tick on the tiles with SetProperty groups only (k_xgroups marks them)
    d.tile_work = nullptr;
    if (calls_only && use_u && d.n_tiles) {
        int r = dev_reserve(w, (void**)&w->tile_work_d, &w->tile_work_cap, (size_t)d.n_tiles);
        if (r) return drop_window(w, r);
        if (hipMemsetAsync(w->tile_work_d, 0, (size_t)d.n_tiles, w->stream) != hipSuccess)
            return drop_window(w, fail(NFK_ERR_HIP, "hipMemsetAsync (tile_work)"));
        d.tile_work = w->tile_work_d;
    }

    tp[3] = clk::now();
    // ---- uploads through the pinned arena ----
    // (the SetProperty calls as queued: (object, property, bits) and the head halves)
    // (schedule calls: staged as queued; pre / post entries at most 2 per call, counted on the device)
    const size_t ng = n_xq, nhq = n_hq, npre = 2 * n_hq, npost = 2 * n_hq;
    const size_t n_xhost = ng - n_xdev;  // (uploaded; the device queue's calls are there already)
    size_t off_xc = 0;
    size_t off_hc = align16(off_xc + n_xhost * sizeof(World::XOp));
    size_t off_rs = align16(off_hc + nhq * sizeof(World::HOp)), off_rr = align16(off_rs + ngr * 4);
    size_t off_rf = align16(off_rr + ngr * 4), off_rb = align16(off_rf + (ngr + 1) * 4);
    size_t off_ss = align16(off_rb + nrc * 8), off_sg = align16(off_ss + nrss * 4);
    const bool objs = w->cfg.n_obj > 0;
    size_t off_xh = align16(off_sg + nrss * 4);  // head halves of the calls (object properties)
    // record row-operation lists
    const size_t nrl = rl_slot.size(), nrcall = rc_code.size(), nval = w->rvals.size();
    size_t off_l0 = align16(off_xh + (objs ? ng * 8 : 0)), off_ls = align16(off_l0 + (nrl ? nrss * 4 : 0));
    size_t off_lr = align16(off_ls + nrl * 4), off_lc = align16(off_lr + nrl * 4);
    size_t off_le = align16(off_lc + (nrl ? (nrl + 1) * 4 : 0)), off_cc = align16(off_le + nrl * 4);
    size_t off_ca = align16(off_cc + nrcall * 4), off_cb = align16(off_ca + nrcall * 4);
    size_t off_rv = align16(off_cb + nrcall * 8);
    size_t total = align16(off_rv + (nrl ? nval * 8 : 0));
    // device fold scratch: keys, sorted keys, call indices, sorted indices, group starts [ng + 1],
    // the groups (slot, property, first call [ng + 1]), the sorted values (and head halves), then
    // the radix sort's temporary storage
    const int xkey_bits = bits_for((uint64_t)std::max(w->d.cap, 1)) + 8;  // (~0: no slot, sorts last)
    size_t xf_sort = 0;
    const size_t xa = (ng * 8 + 255) & ~(size_t)255, xa4 = ((ng + 1) * 4 + 255) & ~(size_t)255;
    const size_t xo_k1 = 0, xo_k2 = xo_k1 + xa, xo_i1 = xo_k2 + xa, xo_i2 = xo_i1 + xa4, xo_gi = xo_i2 + xa4,
                 xo_xs = xo_gi + xa4, xo_xp = xo_xs + xa4, xo_xf = xo_xp + xa4, xo_xb = xo_xf + xa4,
                 xo_xh = xo_xb + xa, xo_tmp = xo_xh + (objs ? xa : 0);
    if (ng) {
        int r = dev_reserve(w, (void**)&w->xs_buf, &w->xs_cap, ng * (objs ? 32 : 16));
        if (r) return drop_window(w, r);
        HIPCHK(rocprim::radix_sort_pairs(nullptr, xf_sort, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                         (uint32_t*)nullptr, ng, 0, xkey_bits, w->stream));
        r = dev_reserve(w, &w->xf_buf, &w->xf_cap, xo_tmp + xf_sort + 256);
        if (r) return drop_window(w, r);
    }
    // the schedule-call fold's scratch: keys, sorted keys, indices, sorted indices, per-slot counts
    // and their scans, pre entries, post entries (slot, kind, op, interval, count, time), added
    // flags, the sort's temporary storage
    const int hkey_bits = bits_for((uint64_t)std::max(w->d.cap, 1)) + 6;  // (~0: no slot, sorts last)
    size_t hf_sort = 0;
    const size_t hn8 = (nhq * 8 + 255) & ~(size_t)255, hn4 = ((nhq + 1) * 4 + 255) & ~(size_t)255;
    const size_t hm4 = (npost * 4 + 255) & ~(size_t)255, hm8 = (npost * 8 + 255) & ~(size_t)255;
    const size_t ho_k1 = 0, ho_k2 = hn8, ho_i1 = 2 * hn8, ho_i2 = ho_i1 + hn4, ho_cp = ho_i2 + hn4, ho_cq = ho_cp + hn4,
                 ho_op = ho_cq + hn4, ho_oq = ho_op + hn4, ho_ps = ho_oq + hn4, ho_po = ho_ps + hm4,
                 ho_qs = ho_po + hm4, ho_qk = ho_qs + hm4, ho_qo = ho_qk + hm4, ho_qi = ho_qo + hm4, ho_qc = ho_qi + hm4,
                 ho_qt = ho_qc + hm4, ho_ad = ho_qt + hm8, ho_tmp = ho_ad + hm4;
    if (nhq) {
        HIPCHK(rocprim::radix_sort_pairs(nullptr, hf_sort, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                         (uint32_t*)nullptr, nhq, 0, hkey_bits, w->stream));
        size_t scan_b = 0;  // (the per-slot count scans: device-wide, n + 1 counts, the last 0)
        HIPCHK(rocprim::exclusive_scan(nullptr, scan_b, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, nhq + 1,
                                       rocprim::plus<uint32_t>(), w->stream));
        hf_sort = std::max(hf_sort, scan_b);
        int r = dev_reserve(w, &w->hf_buf, &w->hf_cap, ho_tmp + hf_sort + 256);
        if (r) return drop_window(w, r);
    }
    if (ng || nhq) {  // object -> slot after the window's membership changes
        if (w->obj_slot_dirty || (size_t)w->n_obj * 4 > w->obj_slot_cap) {
            int r = dev_reserve(w, (void**)&w->obj_slot_d, &w->obj_slot_cap, ((size_t)w->n_obj + 1) * 4);
            if (r) return drop_window(w, r);
            HIPCHK(hipMemsetAsync(w->obj_slot_d, 0xFF, (size_t)w->n_obj * 4, w->stream));
            if (d.N > 0)
                hipLaunchKernelGGL(k_obj_slots, dim3((unsigned)((d.N + 255) / 256)), dim3(256), 0, w->stream,
                                   (const int32_t*)w->slot_obj_d, (const uint64_t*)w->fan_desc_w, (int32_t)d.N,
                                   w->obj_slot_d);
            HIPCHK(hipGetLastError());
            w->obj_slot_dirty = false;
        }
    }
    if (nrss) {
        int r = dev_reserve(w, (void**)&w->rs_buf, &w->rs_cap, std::max<size_t>(ngr, 1) * 16);
        if (r) return drop_window(w, r);
        r = dev_reserve(w, (void**)&w->rss_buf, &w->rss_cap, nrss * 16);
        if (r) return drop_window(w, r);
        // rs_has [ngr] bytes, then (with lists) rl_cnt [nrl] and rl_ev [row-event bound]
        r = dev_reserve(w, &w->rl_buf, &w->rl_cap, align16(std::max<size_t>(ngr, 1)) + (nrl + n_rev + 1) * 4);
        if (r) return drop_window(w, r);
    }
    if (total > 0 && (ng || nhq || nrss)) {
        int r = pin_reserve(w, total);
        if (r) return drop_window(w, r);
        char* P = (char*)w->pin;
        if (ng) {
            if (n_xhost) memcpy(P + off_xc, w->xops.data(), n_xhost * sizeof(World::XOp));
            if (objs) memcpy(P + off_xh, w->xops_h.data(), ng * 8);
        }
        if (nhq) memcpy(P + off_hc, w->hops.data(), nhq * sizeof(World::HOp));
        if (nrss) {
            memcpy(P + off_rs, rs_slot.data(), ngr * 4);
            memcpy(P + off_rr, rs_rrc.data(), ngr * 4);
            memcpy(P + off_rf, rs_first.data(), (ngr + 1) * 4);
            uint64_t* rb = (uint64_t*)(P + off_rb);
            for (size_t i = 0; i < nrc; i++) rb[i] = w->rsq[rpk[i] & rim].bits;
            memcpy(P + off_ss, rss_slot.data(), nrss * 4);
            memcpy(P + off_sg, rss_g0.data(), nrss * 4);
        }
        if (nrl) {
            memcpy(P + off_l0, rss_l0.data(), nrss * 4);
            memcpy(P + off_ls, rl_slot.data(), nrl * 4);
            memcpy(P + off_lr, rl_rec.data(), nrl * 4);
            memcpy(P + off_lc, rl_c0.data(), (nrl + 1) * 4);
            memcpy(P + off_le, rl_ev0.data(), nrl * 4);
            memcpy(P + off_cc, rc_code.data(), nrcall * 4);
            memcpy(P + off_ca, rc_aux.data(), nrcall * 4);
            memcpy(P + off_cb, rc_bits.data(), nrcall * 8);
            if (nval) memcpy(P + off_rv, w->rvals.data(), nval * 8);
        }
        HIPCHK(hipMemcpyAsync(w->stage, w->pin, total, hipMemcpyHostToDevice, w->stream));
        HIPCHK(hipEventRecord(w->pin_done, w->stream));
        w->pin_pending = true;
    }
    tp[4] = clk::now();
    char* S = (char*)w->stage;
    // the groups as k_xgroups lays them out: n_x = the call count bounds the groups (entries past
    // the frame's groups hold kNoGroupSlot)
    char* XF = (char*)w->xf_buf;
    d.n_x = (int32_t)ng;
    d.x_slot = ng ? (const uint32_t*)(XF + xo_xs) : nullptr;
    d.x_pid = ng ? (const uint32_t*)(XF + xo_xp) : nullptr;
    d.x_first = ng ? (const uint32_t*)(XF + xo_xf) : nullptr;
    d.x_bits = ng ? (const uint64_t*)(XF + xo_xb) : nullptr;
    d.x_old = ng ? (uint64_t*)w->xs_buf : nullptr;
    d.x_new = ng ? (uint64_t*)w->xs_buf + ng : nullptr;
    d.x_bits_h = ng && objs ? (const uint64_t*)(XF + xo_xh) : nullptr;
    d.x_old_h = ng && objs ? (uint64_t*)w->xs_buf + 2 * ng : nullptr;
    d.x_new_h = ng && objs ? (uint64_t*)w->xs_buf + 3 * ng : nullptr;
    d.n_rs = (int32_t)ngr;
    d.n_rss = (int32_t)nrss;
    d.rs_slot = nrss ? (const uint32_t*)(S + off_rs) : nullptr;
    d.rs_rrc = nrss ? (const uint32_t*)(S + off_rr) : nullptr;
    d.rs_first = nrss ? (const uint32_t*)(S + off_rf) : nullptr;
    d.rs_bits = nrss ? (const uint64_t*)(S + off_rb) : nullptr;
    d.rss_slot = nrss ? (const uint32_t*)(S + off_ss) : nullptr;
    d.rss_g0 = nrss ? (const uint32_t*)(S + off_sg) : nullptr;
    d.rs_old = nrss ? (uint64_t*)w->rs_buf : nullptr;
    d.rs_new = nrss ? (uint64_t*)w->rs_buf + ngr : nullptr;
    d.rs_has = nrss ? (uint8_t*)w->rl_buf : nullptr;
    d.rss_ev = nrss ? (uint32_t*)w->rss_buf : nullptr;
    d.rss_msg = nrss ? (uint32_t*)w->rss_buf + nrss : nullptr;
    d.rss_pos = nrss ? (uint32_t*)w->rss_buf + 2 * nrss : nullptr;
    d.rss_pmsg = nrss ? (uint32_t*)w->rss_buf + 3 * nrss : nullptr;
    d.n_rl = (int32_t)nrl;
    d.rss_l0 = nrl ? (const uint32_t*)(S + off_l0) : nullptr;
    d.rl_slot = nrl ? (const uint32_t*)(S + off_ls) : nullptr;
    d.rl_rec = nrl ? (const uint32_t*)(S + off_lr) : nullptr;
    d.rl_c0 = nrl ? (const uint32_t*)(S + off_lc) : nullptr;
    d.rl_ev0 = nrl ? (const uint32_t*)(S + off_le) : nullptr;
    d.rc_code = nrl ? (const uint32_t*)(S + off_cc) : nullptr;
    d.rc_aux = nrl ? (const uint32_t*)(S + off_ca) : nullptr;
    d.rc_bits = nrl ? (const uint64_t*)(S + off_cb) : nullptr;
    d.rvals = nrl ? (const uint64_t*)(S + off_rv) : nullptr;
    d.rl_cnt = nrl ? (uint32_t*)((char*)w->rl_buf + align16(std::max<size_t>(ngr, 1))) : nullptr;
    d.rl_ev = nrl ? d.rl_cnt + nrl : nullptr;
    w->rsq.clear();
    w->rvals.clear();
    w->rq_index.clear();
    w->ucache.clear();
    w->xops.clear();
    w->xq_n = 0;
    w->xops_h.clear();
    w->sa_calls = 0;
    w->sa_pids[0] = w->sa_pids[1] = 0;
    w->hops.clear();
    w->dcache.clear();
    w->ov_last.clear();
    w->ov_prev.clear();

    // (schedule calls queued: e_flags may be set by k_pre_hostops; they are 0 wherever it sets none)
    d.has_pre = nhq > 0;
    char* HF = (char*)w->hf_buf;
    HPost hpost{};
    if (nhq) {
        hpost = HPost{(uint32_t*)(HF + ho_qs), (uint32_t*)(HF + ho_qk), (uint32_t*)(HF + ho_qo), (float*)(HF + ho_qi),
                      (int32_t*)(HF + ho_qc), (int64_t*)(HF + ho_qt)};
        w->hf_pending = true;
        w->hf_max = npost;
        w->hf_npost = (const uint32_t*)(HF + ho_oq) + nhq;
        w->hf_pslot = hpost.slot;
        w->hf_pkind = hpost.kind;
        w->hf_pop = hpost.op;
        w->hf_added = (const uint8_t*)(HF + ho_ad);
    } else {
        w->hf_pending = false;
    }
    if (ng || nhq || nrss) {
        TimeScope ts(w, KT_AUX);
        if (nrss) {
            hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)((nrss + 255) / 256)), dim3(256), 0, w->stream,
                               d.rss_slot, (int32_t)nrss, d.rs_head);
            if (ngr)
                hipLaunchKernelGGL(k_rsets, dim3((unsigned)((ngr + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream, d);
            if (nrl)  // after k_rsets: it clears the has-flags of the lists' groups
                hipLaunchKernelGGL(k_rrows, dim3((unsigned)((nrl + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream, d);
        }
        if (ng) {
            // the device fold: keys (slot << 7 | property) -> stable radix sort -> groups
            const unsigned gx = (unsigned)((ng + 255) / 256);
            // the calls in call order: the device queue's, then the host's appended to it
            const XCall* xc = (const XCall*)(S + off_xc);
            if (n_xdev) {
                if (int r = xq_reserve_exec(w, ng)) return drop_window(w, r);
                World::XOp* q = (World::XOp*)w->xq[w->xq_b];
                if (n_xhost)
                    HIPCHK(hipMemcpyAsync(q + n_xdev, S + off_xc, n_xhost * sizeof(World::XOp), hipMemcpyDeviceToDevice,
                                          w->stream));
                xc = (const XCall*)q;
            }
            uint64_t* k1 = (uint64_t*)(XF + xo_k1);
            uint64_t* k2 = (uint64_t*)(XF + xo_k2);
            uint32_t* i1 = (uint32_t*)(XF + xo_i1);
            uint32_t* i2 = (uint32_t*)(XF + xo_i2);
            uint32_t* gi = (uint32_t*)(XF + xo_gi);
            hipLaunchKernelGGL(k_xkeys, dim3(gx), dim3(256), 0, w->stream, xc, (int32_t)ng,
                               (const int32_t*)w->obj_slot_d, k1, i1, (uint32_t*)d.x_slot);
            size_t sb = xf_sort;
            if (ng <= (size_t)kSmallPairs)  // (a window's few calls: one launch instead of the radix passes)
                hipLaunchKernelGGL(k_sort_small_pairs, dim3((unsigned)((ng + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream,
                                   (const uint64_t*)k1, k2, (const uint32_t*)i1, i2, (int)ng);
            else
                HIPCHK(rocprim::radix_sort_pairs(XF + xo_tmp, sb, k1, k2, i1, i2, ng, 0, xkey_bits, w->stream));
            hipLaunchKernelGGL(k_scan_heads, dim3(1), dim3(1024), 0, w->stream, (const uint64_t*)k2, (int)ng, gi);
            hipLaunchKernelGGL(k_xgroups, dim3(gx), dim3(256), 0, w->stream, (const uint64_t*)k2, (const uint32_t*)i2,
                               (const uint32_t*)gi, xc, objs ? (const uint64_t*)(S + off_xh) : nullptr, (int32_t)ng,
                               (uint32_t*)d.x_slot, (uint32_t*)d.x_pid, (uint32_t*)d.x_first, (uint64_t*)d.x_bits,
                               (uint64_t*)d.x_bits_h, d.ext_head, (uint8_t*)d.tile_work);
            if (n_xdev) {  // the buffer is free again once the fold has read it; the next window takes the other
                const int b = w->xq_b;
                if (!w->xq_ev[b]) HIPCHK(hipEventCreateWithFlags(&w->xq_ev[b], hipEventDisableTiming));
                HIPCHK(hipEventRecord(w->xq_ev[b], w->stream));
                w->xq_ev_set[b] = true;
                w->xq_b ^= 1;
            }
            hipLaunchKernelGGL(k_sets, dim3((unsigned)((ng + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream, d);
        }
        if (nhq) {
            // the device fold of the schedule calls: keys -> stable radix sort -> per-slot counts ->
            // scans -> pre / post entries; then the pre-scan effects
            const unsigned gh_ = (unsigned)((nhq + 255) / 256);
            const HCall* hc = (const HCall*)(S + off_hc);
            uint64_t* k1 = (uint64_t*)(HF + ho_k1);
            uint64_t* k2 = (uint64_t*)(HF + ho_k2);
            uint32_t* i1 = (uint32_t*)(HF + ho_i1);
            uint32_t* i2 = (uint32_t*)(HF + ho_i2);
            uint32_t* cp = (uint32_t*)(HF + ho_cp);
            uint32_t* cq = (uint32_t*)(HF + ho_cq);
            uint32_t* op = (uint32_t*)(HF + ho_op);
            uint32_t* oq = (uint32_t*)(HF + ho_oq);
            uint32_t* ps = (uint32_t*)(HF + ho_ps);
            uint32_t* po = (uint32_t*)(HF + ho_po);
            hipLaunchKernelGGL(k_hkeys, dim3(gh_), dim3(256), 0, w->stream, hc, (int32_t)nhq,
                               (const int32_t*)w->obj_slot_d, k1, i1);
            size_t sb = hf_sort;
            if (nhq <= (size_t)kSmallPairs)
                hipLaunchKernelGGL(k_sort_small_pairs, dim3((unsigned)((nhq + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream,
                                   (const uint64_t*)k1, k2, (const uint32_t*)i1, i2, (int)nhq);
            else
                HIPCHK(rocprim::radix_sort_pairs(HF + ho_tmp, sb, k1, k2, i1, i2, nhq, 0, hkey_bits, w->stream));
            hipLaunchKernelGGL(k_hfold<false>, dim3((unsigned)((nhq + 1 + 255) / 256)), dim3(256), 0, w->stream,
                               (const uint64_t*)k2, (const uint32_t*)i2,
                               hc, (int32_t)nhq, cp, cq, (const uint32_t*)nullptr, (const uint32_t*)nullptr, ps, po, hpost);
            size_t tb = hf_sort;  // (a mass AddSchedule at start: millions of calls, so a device-wide scan)
            HIPCHK(rocprim::exclusive_scan(HF + ho_tmp, tb, (const uint32_t*)cp, op, 0u, nhq + 1, rocprim::plus<uint32_t>(),
                                           w->stream));
            tb = hf_sort;
            HIPCHK(rocprim::exclusive_scan(HF + ho_tmp, tb, (const uint32_t*)cq, oq, 0u, nhq + 1, rocprim::plus<uint32_t>(),
                                           w->stream));
            hipLaunchKernelGGL(k_hfold<true>, dim3(gh_), dim3(256), 0, w->stream, (const uint64_t*)k2, (const uint32_t*)i2,
                               hc, (int32_t)nhq, cp, cq, (const uint32_t*)op, (const uint32_t*)oq, ps, po, hpost);
            hipLaunchKernelGGL(k_pre_hostops, dim3((unsigned)((npre + 255) / 256)), dim3(256), 0, w->stream,
                               (const uint32_t*)ps, (const uint32_t*)po, (int32_t)npre, d.e_flags, d.s_hot, d.n_kind,
                               d.s_kstr, (const uint32_t*)op + nhq);
        }
        HIPCHK(hipGetLastError());
    }
    // k_tick writes its tiles' fan-out itself (its LDS image is reused for the events): property
    // tile t's messages sit at t * msg_tcap, msg_tcap = writable properties x slots x most
    // recipients of one event, so no tile waits for another tile's count.  Worlds whose bound
    // would reserve more than kMsgStrideLimit run k_fanout after k_scan_tiles instead.
    // With the property tiles at a fixed stride, k_records fans out its record tiles the same way
    // after them: msg_rtcap = slots x cells the record ops may change x most recipients of one
    // record event (the scene group's players for a public record, 1 for a private one).
    d.msg_tcap = 0;
    d.fuse_rec = 0;
    d.msg_rb0 = d.msg_rtcap = 0;
    if (use_u && d.n_tiles && !(d.ablate & (kAblNoFuse | kAblNoEmit))) {
        int64_t tcap = (((int64_t)std::max(d.n_w, 1) * kTile + max_sa) * std::max(w->max_np, 1) + 3) & ~(int64_t)3;
        if (d.ablate & kAblTinyTcap) tcap = 4;  // test hook: a bound every busy tile exceeds (kErrFanBound)
        int64_t rtcap = 0;
        bool rfuse = false;
        if (d.has_recops && d.n_rtiles) {
            int64_t cells = 0, per = 0;
            for (int j = 0; j < d.n_rops; j++) cells += d.rops[j].rows;
            auto rper = [&](int rec) {
                for (int c = 0; c < NFK_MAX_CLASSES; c++) {
                    const uint8_t f = w->tab.rflags[c][rec];
                    per = std::max<int64_t>(per, (f & NFK_PUBLIC) ? std::max(w->max_np, 1)
                                                 : ((f & NFK_PRIVATE) && !(f & NFK_UPLOAD)) ? 1 : 0);
                }
            };
            for (int j = 0; j < d.n_rops; j++) rper(d.rops[j].rec);
            if (nrss)  // SetRecord groups and row operations may hit any record
                for (int r = 0; r < d.n_rec; r++)
                    if (w->rec_defined[r]) rper(r);
            rtcap = (((int64_t)kRTile * cells + max_rs_tile) * per + 3) & ~(int64_t)3;  // (16-byte aligned runs)
            rfuse = tcap * d.n_tiles + rtcap * d.n_rtiles <= kMsgStrideLimit;
        }
        const int64_t need = tcap * d.n_tiles + (rfuse ? rtcap * d.n_rtiles
                                                       : w->last_rec_msgs + w->last_rec_msgs / 4) + 1024;
        if (tcap * d.n_tiles <= kMsgStrideLimit) {
            if (need > w->d.msg_cap) {  // grow before the frame (the previous frame's messages are dropped)
                HIPCHK(hipStreamSynchronize(w->stream));
                int r = regrow(w, (void**)&w->d.msg_rcpt, (size_t)need * 4);
                if (r) {
                    w->d.msg_cap = 0;
                    return drop_window(w, r);
                }
                w->d.msg_cap = need;
                d.msg_rcpt = w->d.msg_rcpt;
                d.msg_cap = need;
            }
            d.msg_tcap = (uint32_t)tcap;
            if (rfuse) {
                d.fuse_rec = 1;
                d.msg_rb0 = (uint32_t)(tcap * d.n_tiles);
                d.msg_rtcap = (uint32_t)rtcap;
            }
        }
    }
    d.fuse_fan = d.msg_tcap != 0;
    // A small world with no record pipeline after k_tick: its last tile ranks the frame's tiles
    // and the frame has no k_scan_tiles launch (profiles/r09a_*)
    d.lb_rank = (d.fuse_fan && !d.has_recops && d.n_tiles && d.n_tiles <= kLbMaxTiles &&
                 !(d.ablate & kAblScanKernel) && (!(use_u && w->jit_fn) || w->jit_lb)) ? 1 : 0;
    if (d.lb_rank) {
        if (++w->lb_epoch == 0xFFFFFFFFu) {  // (clear the tags before they could repeat)
            HIPCHK(hipMemsetAsync(w->d.lb_st, 0, std::min<size_t>(w->obj_of_slot.size() / kTile, kLbMaxTiles) * 4 * 8,
                                  w->stream));
            w->lb_epoch = 1;
        }
        d.lb_epoch = w->lb_epoch;
    }
    w->last_tcap = d.msg_tcap;
    w->last_rtcap = d.fuse_rec ? d.msg_rtcap : 0u;
    // per-Set chains of the watched properties: the programs re-run read-only before k_tick
    // (k_chain); a calls-only pass fires nothing and keeps the frame's log
    if (!calls_only) w->chain_ran = false;
    if (!calls_only && (w->chain_watch[0] | w->chain_watch[1]) && d.N) {
        uint32_t kinds = 0;
        int64_t wops = 0;  // (kind, op) pairs whose destination is watched: a bound of the log per slot
        for (int k = 0; k < d.n_kind; k++)
            for (int i = 0; i < w->tab.nops[k]; i++) {
                const nfk_op& op = w->tab.ops[k][i];
                const bool prop_op = op.code == NFK_OP_IADD_CLAMP || op.code == NFK_OP_FLERP ||
                                     op.code == NFK_OP_FAFFINE || op.code == NFK_OP_ISET || op.code == NFK_OP_FSET;
                if (prop_op && op.dst < 128 && ((w->chain_watch[op.dst >> 6] >> (op.dst & 63)) & 1)) {
                    kinds |= 1u << k;
                    wops++;
                }
            }
        // ... and every kind before one of those whose program writes a property a later re-run kind
        // reads (an operand, a guard, or a destination's current value): the reference's functors run
        // in name order on what the earlier ones left (SM:52-80), so the logged (old, new) of a watched
        // Set depend on them.  Closed transitively, latest kind first.  (NFGPU_CHAIN_NO_CLOSURE=1: test
        // hook, the watched kinds only — the round-5 form, which logged wrong (old, new) for such Sets)
        static const bool no_closure = getenv("NFGPU_CHAIN_NO_CLOSURE") && getenv("NFGPU_CHAIN_NO_CLOSURE")[0] == '1';
        if (kinds && !no_closure) {
            auto bit = [](uint64_t (&m)[2], uint32_t p) {
                if (p < 128) m[p >> 6] |= 1ull << (p & 63);
            };
            uint64_t rd[NFK_MAX_KINDS][2] = {}, wr[NFK_MAX_KINDS][2] = {};
            for (int k = 0; k < d.n_kind; k++)
                for (int i = 0; i < w->tab.nops[k]; i++) {
                    const nfk_op& op = w->tab.ops[k][i];
                    if (op.code != NFK_OP_IADD_CLAMP && op.code != NFK_OP_FLERP && op.code != NFK_OP_FAFFINE &&
                        op.code != NFK_OP_ISET && op.code != NFK_OP_FSET)
                        continue;
                    bit(wr[k], op.dst);
                    bit(rd[k], op.dst);
                    if (op.flags & NFK_GUARD) {
                        bit(rd[k], op.guard & 0xFFFFu);
                        if (op.guard & NFK_GUARD_PROP) bit(rd[k], op.guard >> 19);
                    }
                    if (op.code == NFK_OP_FLERP || ((op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) && (op.flags & NFK_A_PROP)))
                        bit(rd[k], (uint32_t)op.a);
                    if (op.code == NFK_OP_IADD_CLAMP) {
                        if (op.flags & NFK_A_PROP) bit(rd[k], (uint32_t)op.a);
                        if (op.flags & NFK_LO_PROP) bit(rd[k], (uint32_t)op.b);
                        if (op.flags & NFK_HI_PROP) bit(rd[k], (uint32_t)op.c);
                    }
                }
            uint64_t need[2] = {0, 0};  // what the re-run kinds after position k read
            for (int k = d.n_kind - 1; k >= 0; k--) {
                if (!((kinds >> k) & 1) && ((wr[k][0] & need[0]) | (wr[k][1] & need[1]))) kinds |= 1u << k;
                if ((kinds >> k) & 1) {
                    need[0] |= rd[k][0];
                    need[1] |= rd[k][1];
                }
            }
        }
        if (kinds) {
            // tile-staged: kTPB slots x the watched (kind, op) pairs per tile (each logs at most once)
            const int32_t nt = (int32_t)((d.N + kTPB - 1) / kTPB);
            const uint32_t tcap = (uint32_t)(kTPB * wops);
            const size_t need = (size_t)nt * tcap;
            if (need > w->chain_cap || nt > w->chain_tiles) {
                HIPCHK(hipStreamSynchronize(w->stream));
                if (need > w->chain_cap) {
                    if (w->chain_d) HIPCHK(hipFree(w->chain_d));
                    w->chain_d = nullptr;
                    w->chain_cap = 0;
                    if (hipMalloc(&w->chain_d, need * sizeof(ChainEnt)) != hipSuccess)
                        return drop_window(w, fail(NFK_ERR_CAPACITY, "hipMalloc (per-Set chain log)"));
                    w->chain_cap = need;
                }
                if (nt > w->chain_tiles) {
                    if (w->chain_cnt_d) HIPCHK(hipFree(w->chain_cnt_d));
                    w->chain_cnt_d = nullptr;
                    w->chain_tiles = 0;
                    HIPCHK(hipMalloc(&w->chain_cnt_d, ((size_t)nt + 1) * sizeof(uint32_t)));
                    w->chain_tiles = nt;
                }
            }
            w->chain_tcap = tcap;
            TimeScope ts(w, KT_CHAIN);
            // on the frame's register working set (the world's hipRTC policy, or the library's tables),
            // else on k_tick_touch's written-property list (NFGPU_CHAIN_U=0 forces that one, for A/B)
            static const bool chain_u = !getenv("NFGPU_CHAIN_U") || getenv("NFGPU_CHAIN_U")[0] != '0';
            ChainEnt* cd = (ChainEnt*)w->chain_d;
            uint32_t* cc = w->chain_cnt_d;
            uint64_t w0 = w->chain_watch[0], w1 = w->chain_watch[1];
            if (chain_u && use_u && w->jit_chain_fn) {
                void* args[] = {&d, &cd, &cc, (void*)&tcap, &kinds, &w0, &w1};
                HIPCHK(hipModuleLaunchKernel(w->jit_chain_fn, (unsigned)nt, 1, 1, kTPB, 1, 1, 0, w->stream, args, nullptr));
            } else if (chain_u && use_u && d.n_u <= 8) {
                hipLaunchKernelGGL((k_chain_u<8, DynSchema>), dim3((unsigned)nt), dim3(kTPB), 0, w->stream, d, cd, cc, tcap, kinds, w0, w1);
            } else if (chain_u && use_u && d.n_u <= 12) {
                hipLaunchKernelGGL((k_chain_u<12, DynSchema>), dim3((unsigned)nt), dim3(kTPB), 0, w->stream, d, cd, cc, tcap, kinds, w0, w1);
            } else if (chain_u && use_u) {
                hipLaunchKernelGGL((k_chain_u<16, DynSchema>), dim3((unsigned)nt), dim3(kTPB), 0, w->stream, d, cd, cc, tcap, kinds, w0, w1);
            } else {
                hipLaunchKernelGGL(k_chain, dim3((unsigned)nt), dim3(kTPB), 0, w->stream, d, w->chain_d, w->chain_cnt_d, tcap,
                                   kinds, w->chain_watch[0], w->chain_watch[1]);
            }
            HIPCHK(hipGetLastError());
            w->chain_ran = true;
            w->chain_tiles = nt;
        }
    }
    if (d.n_tiles) {
        TimeScope ts(w, KT_TICK);
        size_t lds = (size_t)std::max(d.n_w, 1) * kTPB * 8 + (size_t)std::max(d.n_kind, 1) * kTPB * 4;
        const bool jit = use_u && w->jit_fn;
        if (d.fuse_fan) {  // the fan-out's message window takes what LDS the variant's occupancy
                           // leaves (waves per SIMD = workgroups per CU; ~2.3 KB static each)
            const int waves = jit ? w->jit_waves : tick_waves(d.n_u, d.ablate);
            lds = std::max(lds, (size_t)(163840 / waves - 2560) & ~(size_t)1023);
        }
        d.lds_words = (int32_t)(lds / 4);
        {  // XCD-contiguous tiles (Dev::xcd_map; NFGPU_TICK_XCD=0 deals them round-robin):
           // config[3] 342 -> 331 us, config[1] unchanged (profiles/r11o_ktick_xcd_map_ab.txt)
            static const int xm = getenv("NFGPU_TICK_XCD") ? atoi(getenv("NFGPU_TICK_XCD")) : 1;
            d.xcd_map = xm;
        }
        // the variant whose register slots hold the frame's working set (no spills at 6 or more
        // waves per SIMD): this schema's own k_tick, else a generic instantiation
        const dim3 g((unsigned)d.n_tiles), b(kTPB);
        if (jit) {
            void* args[] = {&d};
            HIPCHK(hipModuleLaunchKernel(w->jit_fn, (unsigned)d.n_tiles, 1, 1, kTPB, 1, 1, (unsigned)lds, w->stream,
                                         args, nullptr));
        } else if (use_u && d.n_u <= 8 && !(d.ablate & kAblWaves6))
            hipLaunchKernelGGL((k_tick<kWavesU8, 8>), g, b, lds, w->stream, d);
        else if (use_u && d.n_u <= 12 && !(d.ablate & kAblWaves6))
            hipLaunchKernelGGL((k_tick<kWavesU12, 12>), g, b, lds, w->stream, d);
        else if (use_u)
            hipLaunchKernelGGL((k_tick<6, 16>), g, b, lds, w->stream, d);
        else
            hipLaunchKernelGGL(k_tick_touch, dim3((unsigned)d.n_tiles), dim3(kTPB), 0, w->stream, d);
        HIPCHK(hipGetLastError());
    }
    if (d.has_recops && d.n_rtiles) {
        TimeScope ts(w, KT_REC);
        constexpr int kWpb = kTPB / 64;  // record tiles (waves) per workgroup
        const dim3 g((unsigned)((d.n_rtiles + kWpb - 1) / kWpb)), b(kTPB);
        if (nrss)  // the SetRecord slots' events and messages, for k_records to reserve
            hipLaunchKernelGGL((k_rset_slots<false>), dim3((unsigned)((nrss + kWpb - 1) / kWpb)), b, 0, w->stream, d);
        // (the SetRecord slots' instantiation, and the unfused one: the fast path stays lean)
        auto launch = [&](auto sets, auto fuse) {
            constexpr bool kS = decltype(sets)::value, kF = decltype(fuse)::value;
            if (d.n_rops <= 1)
                hipLaunchKernelGGL((k_records<1, 4, kS, kF>), g, b, 0, w->stream, d);
            else if (d.n_rops <= 2) {
                // two known op codes (the fast path's common shape): compiled in
                const unsigned c0 = d.rops[0].code == NFK_OP_RIADD_CLAMP ? 1u : 2u;
                const unsigned c1 = d.rops[1].code == NFK_OP_RIADD_CLAMP ? 1u : 2u;
                if (kS || !kF || d.n_rops != 2)
                    hipLaunchKernelGGL((k_records<2, 4, kS, kF>), g, b, 0, w->stream, d);
                else if (c0 == 1 && c1 == 1)
                    hipLaunchKernelGGL((k_records<2, 4, kS, kF, 5u>), g, b, 0, w->stream, d);
                else if (c0 == 1 && c1 == 2)
                    hipLaunchKernelGGL((k_records<2, 4, kS, kF, 9u>), g, b, 0, w->stream, d);
                else if (c0 == 2 && c1 == 1)
                    hipLaunchKernelGGL((k_records<2, 4, kS, kF, 6u>), g, b, 0, w->stream, d);
                else
                    hipLaunchKernelGGL((k_records<2, 4, kS, kF, 10u>), g, b, 0, w->stream, d);
            }
            else
                hipLaunchKernelGGL((k_records<NFK_MAX_REC_OPS, 2, kS, kF>), g, b, 0, w->stream, d);
        };
        using T = std::true_type;
        using F = std::false_type;
        if (nrss)
            d.fuse_rec ? launch(T{}, T{}) : launch(T{}, F{});
        else
            d.fuse_rec ? launch(F{}, T{}) : launch(F{}, F{});
        if (nrss)  // ... and written into the room k_records left
            hipLaunchKernelGGL((k_rset_slots<true>), dim3((unsigned)((nrss + kWpb - 1) / kWpb)), b, 0, w->stream, d);
        HIPCHK(hipGetLastError());
    }
    if (nhq) {  // the post-scan entries (their count is the fold's, on the device)
        TimeScope ts(w, KT_AUX);
        hipLaunchKernelGGL(k_post_hostops, dim3((unsigned)((npost + 255) / 256)), dim3(256), 0, w->stream,
                           (const uint32_t*)hpost.slot, (const uint32_t*)hpost.kind, (const uint32_t*)hpost.op,
                           (const float*)hpost.interval, (const int32_t*)hpost.count, (const int64_t*)hpost.time,
                           (int32_t)npost, (uint8_t*)(HF + ho_ad), d, w->hf_npost);
        HIPCHK(hipGetLastError());
    }
    // Dense global ranks of the tile-staged outputs (ev_base, fi_base, totals): the frame's own
    // work needs them only when k_fanout runs after it (record tiles, unfused property tiles).
    // Otherwise the frame's outputs are complete as tiles + per-tile counts, and the ranks are
    // built on the first read (nfk_summary_get, nfk_outputs_get, nfk_read_*).
    w->scan_pending = false;
    if (d.lb_rank) {
        // (written by k_tick's last tile)
    } else if (d.fuse_fan && (!d.has_recops || d.fuse_rec) && !(d.ablate & kAblScanInFrame)) {
        w->scan_pending = true;
        w->scan_dev = d;
    } else {
        TimeScope ts(w, KT_SCAN);
        hipLaunchKernelGGL(k_scan_tiles, dim3(4), dim3(kScanTPB), 0, w->stream, d);
        HIPCHK(hipGetLastError());
    }
    // the tiles k_tick / k_records did not fan out: record tiles, and property tiles after
    // k_tick_touch
    const int fan0 = d.fuse_fan ? d.n_tiles : 0;
    const int nfan = d.n_tiles + (d.has_recops && !d.fuse_rec ? d.n_rtiles : 0) - fan0;
    if (nfan > 0 && !(d.ablate & kAblNoEmit)) {  // (timing ablation: events were not written)
        {
            TimeScope ts(w, KT_FAN);
            hipLaunchKernelGGL(k_fanout, dim3((unsigned)nfan), dim3(kTPB), 0, w->stream, d, (int32_t)fan0);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemcpyAsync(w->err_pin, &w->ctrl->err, sizeof(unsigned), hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipEventRecord(w->err_done, w->stream));
        w->fan_unchecked = true;
    }
    w->ticks++;
    if (trace) {
        tp[5] = clk::now();
        auto ms = [&](int a, int b) { return std::chrono::duration<double, std::milli>(tp[b] - tp[a]).count(); };
        fprintf(stderr, "nfk_execute: membership %.3f ms, SetProperty groups %.3f ms (%zu calls), schedule "
                "calls %.3f ms (%zu), upload %.3f ms, launches %.3f ms\n", ms(0, 1), ms(1, 2), n_xq, ms(2, 3),
                n_hq, ms(3, 4), ms(4, 5));
    }
    return NFK_OK;
}

int nfk_execute(void* world, int64_t now_ms) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    return execute_frame(w, now_ms, false);
}

int nfk_execute_calls(void* world) {
    // a frame at the earliest time: `now > next` holds for no schedule, so nothing fires and no
    // record is rescheduled; the queued calls run through the ordinary frame path, k_tick only on
    // the tiles their SetProperty groups touch
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    return execute_frame(w, INT64_MIN, true);
}

int nfk_sync(void* world) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    HIPCHK(hipStreamSynchronize(w->stream));
    return NFK_OK;
}

int nfk_get_stream(void* world, void** stream) {
    World* w = (World*)world;
    if (!w || !stream) return fail(NFK_ERR_ARG, "null argument");
    *stream = (void*)w->stream;
    return NFK_OK;
}

static int ensure_ranks(World* w) {
    if (!w->scan_pending) return NFK_OK;
    w->scan_pending = false;
    TimeScope ts(w, KT_SCAN);
    hipLaunchKernelGGL(k_scan_tiles, dim3(4), dim3(kScanTPB), 0, w->stream, w->scan_dev);
    HIPCHK(hipGetLastError());
    return NFK_OK;
}

static int read_ctrl(World* w, Ctrl* c) {
    int r = ensure_ranks(w);
    if (r) return r;
    HIPCHK(hipMemcpyAsync(w->ctrl_pin, w->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    memcpy(c, w->ctrl_pin, sizeof(Ctrl));
    return NFK_OK;
}
// the control block and the byte tallies (read_tallies) behind the frame, one synchronisation
static int read_ctrl_tallies(World* w, Ctrl* c, uint64_t tb[3]) {
    int r = ensure_ranks(w);
    if (r) return r;
    char* tp = w->ctrl_pin + kCtrlPinTally;
    HIPCHK(hipMemcpyAsync(w->ctrl_pin, w->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipMemcpyAsync(tp, w->d.tally, kTallyBytes, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    memcpy(c, w->ctrl_pin, sizeof(Ctrl));
    const unsigned long long* t = (const unsigned long long*)tp;
    for (int k = 0; k < 3; k++) {
        tb[k] = 0;
        for (int i = 0; i < kTallyN; i++) tb[k] += t[((size_t)k * kTallyN + i) * 8];
    }
    return NFK_OK;
}

// entries of msg_rcpt reserved by the fixed-stride tiles of the last frame (property tiles, and
// record tiles when k_records fanned them out)
static int64_t fixed_msgs_reserved(const World* w) {
    return (int64_t)w->last_tcap * w->d.n_tiles + (int64_t)w->last_rtcap * (w->d.has_recops ? w->d.n_rtiles : 0);
}

// messages of the last frame: the runs are dense unless k_tick placed property tiles at a stride
static int64_t frame_msgs(const World* w, const Ctrl& c) {
    if (!w->last_tcap) return (int64_t)c.msg_extent;
    return (int64_t)c.n_msgs_ptiles + (int64_t)c.msg_extent - fixed_msgs_reserved(w);
}

// The last frame's k_fanout found msg_rcpt too small: it wrote nothing (it checks the scanned
// extent first) and only reads the event tiles and the membership CSR, so grow the message buffer
// (keeping what k_tick's / k_records' own fan-out wrote) and re-run it for that frame.
static int regrow_fanout(World* w, Ctrl& c) {
    const int64_t extent = (int64_t)c.msg_extent;
    const int64_t need = extent + extent / 4 + 1024;
    if (need > 0xFFFFFFFFll) return fail(NFK_ERR_CAPACITY, "fan-out exceeds 2^32 messages per frame");
    uint32_t* grown = nullptr;
    int r = alloc_track(w, (void**)&grown, (size_t)need * 4);
    if (r) return r;
    if (w->last_tcap)
        HIPCHK(hipMemcpy(grown, w->d.msg_rcpt, (size_t)fixed_msgs_reserved(w) * 4, hipMemcpyDeviceToDevice));
    HIPCHK(hipFree(w->d.msg_rcpt));
    w->allocs.erase(std::remove(w->allocs.begin(), w->allocs.end(), (void*)w->d.msg_rcpt), w->allocs.end());
    w->d.msg_rcpt = grown;
    w->d.msg_cap = need;
    HIPCHK(hipMemset(&w->ctrl->err, 0, sizeof(unsigned)));
    Dev d = w->d;
    const int fan0 = w->last_tcap ? d.n_tiles : 0;
    const int nfan = d.n_tiles + (d.has_recops && !w->last_rtcap ? d.n_rtiles : 0) - fan0;
    if (nfan > 0) hipLaunchKernelGGL(k_fanout, dim3((unsigned)nfan), dim3(kTPB), 0, w->stream, d, (int32_t)fan0);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(w->stream));
    HIPCHK(hipMemcpy(&c, w->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost));
    return NFK_OK;
}

// Before anything reads or replaces the last frame's fan-out: if its k_fanout overflowed the
// message buffer, recover that frame now (whether or not nfk_summary_get was called).
static int check_fanout(World* w) {
    if (!w->fan_unchecked) return NFK_OK;
    HIPCHK(hipEventSynchronize(w->err_done));
    w->fan_unchecked = false;
    if (!(*w->err_pin & kErrMsgCap)) return NFK_OK;
    Ctrl c;
    int r = read_ctrl(w, &c);
    if (r) return r;
    if (c.err & ~kErrMsgCap) return NFK_OK;  // (another device error: reported by nfk_summary_get)
    return regrow_fanout(w, c);
}

int nfk_summary_get(void* world, nfk_summary* out) {
    World* w = (World*)world;
    if (!w || !out) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    uint64_t tb[3];
    {
        int r = check_fanout(w);
        if (r) return r;
    }
    {
        int r = read_ctrl_tallies(w, &c, tb);
        if (r) return r;
    }
    memset(out, 0, sizeof *out);
    {
        int64_t live = 0;
        for (const auto& g : w->segs) live += (int64_t)g.objs.size();
        out->n_entities = live;
    }
    out->n_prop_events = (int64_t)c.n_ev;
    out->n_rec_events = (int64_t)c.n_re;
    out->n_fired = (int64_t)c.n_fi;
    out->n_msgs = frame_msgs(w, c);
    {
        out->alg_bytes_tick = (int64_t)(tb[0] - w->last_bytes[0]);
        out->alg_bytes_rec = (int64_t)(tb[1] - w->last_bytes[1]);
        out->alg_bytes_fan = (int64_t)(tb[2] - w->last_bytes[2]);
        for (int k = 0; k < 3; k++) w->last_bytes[k] = tb[k];
    }
    if ((c.err & kErrMsgCap) && !(c.err & ~kErrMsgCap)) {
        int r = regrow_fanout(w, c);
        if (r) return r;
    }
    w->last_rec_msgs = frame_msgs(w, c) - (int64_t)c.n_msgs_ptiles;
    out->device_error = (int32_t)c.err;
    out->tick = w->ticks;
    if (c.err) HIPCHK(hipMemset(&w->ctrl->err, 0, sizeof(unsigned)));
    clear_err_host(w);  // (the stream is idle: read_ctrl synchronised it)
    if (c.err & kErrTouch) return fail(NFK_ERR_TOUCH, "device touch list overflow");
    if (c.err & kErrFanBound) return fail(NFK_ERR_STATE, "a tile's fan-out exceeded its bound");
    if (c.err & kErrRemain) return fail(NFK_ERR_STATE, "k_tick read a fired heartbeat's remain it never wrote");
    if (c.err & kErrMsgCap)
        return fail(NFK_ERR_CAPACITY, "device output capacity exceeded (err=" + std::to_string(c.err) + ")");
    return NFK_OK;
}

int nfk_outputs_get(void* world, nfk_outputs* o) {
    World* w = (World*)world;
    if (!w || !o) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    int r = check_fanout(w);  // (synchronises only after a frame that ran k_fanout)
    if (r) return r;
    // a device error of a frame that has completed (host-mapped word, no device read); a frame
    // still running reports through the next call that waits for it (nfk_execute, nfk_summary_get)
    if (const unsigned e = err_host_bits(w); e & (kErrFanBound | kErrTouch))
        return fail(NFK_ERR_DEVICE, (e & kErrFanBound) ? "a tile's fan-out exceeded its bound: the recipient lists are truncated"
                                                       : "touch list overflow: events are missing");
    r = ensure_ranks(w);  // (asynchronous, on the world's stream like the frame)
    if (r) return r;
    const Dev& d = w->d;
    o->n_tiles = d.n_tiles; o->tile_slots = kTile;
    o->n_rtiles = d.has_recops ? d.n_rtiles : 0; o->rtile_slots = kRTile;
    o->ev_tile_cap = d.ev_tcap; o->fi_tile_cap = d.fi_tcap; o->re_tile_cap = d.re_tcap;
    o->ev_base = d.ev_base; o->fi_base = d.fi_base; o->re_base = d.re_base; o->msg_base = d.msg_base;
    o->msg_cnt = d.t_msg;
    o->ev_slot = d.ev_slot; o->ev_pid = d.ev_pid; o->ev_old = d.ev_old; o->ev_new = d.ev_new;
    o->ev_moff = w->last_tcap ? nullptr : d.ev_moff;  // (tiles k_tick fanned out store none: nfgpu.h)
    o->re_slot = nullptr;  // (a record event's slot is in its word: nfgpu.h)
    o->re_rrc = d.re_rrc; o->re_old = d.re_old; o->re_new = d.re_new;
    o->re_moff = w->last_rtcap ? nullptr : d.re_moff;  // (fused record tiles store none: nfgpu.h)
    o->fi_slot = d.fi_slot; o->fi_kind = d.fi_kind; o->fi_remain = d.fi_remain;
    o->msg_rcpt = d.msg_rcpt;
    o->slot_obj = w->slot_obj_d;
    o->ev_old_h = d.ev_old_h;
    o->ev_new_h = d.ev_new_h;
    return NFK_OK;
}

int nfk_read_object(void* world, int32_t pid, int64_t* head, int64_t* data) {
    World* w = (World*)world;
    if (!w || !head || !data || pid < w->n_if || pid >= w->n_prop) return fail(NFK_ERR_ARG, "bad argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    HIPCHK(hipStreamSynchronize(w->stream));
    const Dev& d = w->d;
    std::vector<uint64_t> col(2 * (size_t)std::max(d.N, 1));
    if (d.N) HIPCHK(hipMemcpy(col.data(), d.pmem + w->tab.p_off[pid], (size_t)d.N * 16, hipMemcpyDeviceToHost));
    memset(head, 0, (size_t)w->n_obj * 8);  // objects no longer in this world read the null NFGUID
    memset(data, 0, (size_t)w->n_obj * 8);
    for (int32_t s = 0; s < d.N; s++)
        if (w->obj_of_slot[s] >= 0) {
            data[w->obj_of_slot[s]] = (int64_t)col[2 * (size_t)s];
            head[w->obj_of_slot[s]] = (int64_t)col[2 * (size_t)s + 1];
        }
    return NFK_OK;
}

int nfk_read_prop(void* world, int32_t pid, uint64_t* bits) {
    World* w = (World*)world;
    if (!w || !bits || pid < 0 || pid >= w->n_if) return fail(NFK_ERR_ARG, "bad argument (object properties: nfk_read_object)");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    HIPCHK(hipStreamSynchronize(w->stream));
    const Dev& d = w->d;
    std::vector<uint64_t> col(std::max(d.N, 1));
    if (d.N)
        HIPCHK(hipMemcpy2D(col.data(), 8, d.pmem + w->tab.p_off[pid], (size_t)w->tab.p_str[pid] * 8, 8, (size_t)d.N,
                           hipMemcpyDeviceToHost));
    memset(bits, 0, (size_t)w->n_obj * 8);  // objects no longer in this world read 0
    for (int32_t s = 0; s < d.N; s++)
        if (w->obj_of_slot[s] >= 0) bits[w->obj_of_slot[s]] = col[s];
    return NFK_OK;
}

int nfk_read_record(void* world, int32_t rec, uint64_t* cells) {
    World* w = (World*)world;
    if (!w || !cells || rec < 0 || rec >= w->cfg.n_rec) return fail(NFK_ERR_ARG, "bad argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    HIPCHK(hipStreamSynchronize(w->stream));
    const Dev& d = w->d;
    const int rows = w->tab.rec_rows[rec], cols = w->tab.rec_cols[rec];
    const uint64_t rowm = rec_rowm(rows);
    size_t per = (size_t)rows * cols;
    std::vector<uint64_t> buf(per * d.N), used(d.N);
    HIPCHK(hipMemcpy(buf.data(), d.rcells[rec], buf.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(used.data(), d.rused[rec], used.size() * 8, hipMemcpyDeviceToHost));
    memset(cells, 0, (size_t)w->n_obj * per * 8);
    for (int32_t s = 0; s < d.N; s++) {
        if (w->obj_of_slot[s] < 0) continue;
        uint64_t* dst = cells + (size_t)w->obj_of_slot[s] * per;  // row order (from packed, rec_pos)
        const uint64_t* src = &buf[(size_t)s * per];
        for (int c = 0; c < cols; c++)
            for (int q = 0; q < rows; q++) dst[(size_t)c * rows + q] = src[(size_t)c * rows + rec_pos(used[s], rowm, q)];
    }
    return NFK_OK;
}

int nfk_read_schedules(void* world, int64_t* next_ms, int32_t* remain, uint8_t* state) {
    World* w = (World*)world;
    if (!w || !next_ms || !remain || !state) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    HIPCHK(hipStreamSynchronize(w->stream));
    const Dev& d = w->d;
    const int NK = d.n_kind;
    std::vector<SchedHot> hot((size_t)NK * d.s_kstr);
    if (NK) HIPCHK(hipMemcpy(hot.data(), d.s_hot, hot.size() * sizeof(SchedHot), hipMemcpyDeviceToHost));
    memset(state, 0, (size_t)NK * w->n_obj);
    memset(next_ms, 0, (size_t)NK * w->n_obj * 8);
    memset(remain, 0, (size_t)NK * w->n_obj * 4);
    for (int k = 0; k < NK; k++)
        for (int32_t s = 0; s < d.N; s++) {
            if (w->obj_of_slot[s] < 0) continue;
            size_t o = (size_t)k * w->n_obj + w->obj_of_slot[s], a = (size_t)k * d.s_kstr + s;
            const SchedHot& h = hot[a];
            state[o] = (uint8_t)(h.state & (kStPresent | kStForever));
            next_ms[o] = (h.state & 1) ? h.next : 0;
            remain[o] = (h.state & 1) ? h.remain : 0;
        }
    return NFK_OK;
}

int nfk_read_events(void* world, int32_t* ev_obj, int32_t* ev_pid, uint64_t* ev_old, uint64_t* ev_new) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    int r = read_ctrl(w, &c);
    if (r) return r;
    const Dev& d = w->d;
    const size_t n = c.n_ev;
    std::vector<uint32_t> sl(n);
    GATHER(w, d.ev_slot, d.ev_base, d.n_tiles, d.ev_tcap, n, sl.data());
    GATHER(w, d.ev_pid, d.ev_base, d.n_tiles, d.ev_tcap, n, (uint32_t*)ev_pid);
    GATHER(w, d.ev_old, d.ev_base, d.n_tiles, d.ev_tcap, n, ev_old);
    GATHER(w, d.ev_new, d.ev_base, d.n_tiles, d.ev_tcap, n, ev_new);
    for (size_t i = 0; i < n; i++) ev_obj[i] = w->obj_of_slot[sl[i]];
    return NFK_OK;
}

int nfk_read_events_obj(void* world, uint64_t* ev_old_h, uint64_t* ev_new_h) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    int r = read_ctrl(w, &c);
    if (r) return r;
    const Dev& d = w->d;
    const size_t n = c.n_ev;
    if (!d.n_obj) {
        memset(ev_old_h, 0, n * 8);
        memset(ev_new_h, 0, n * 8);
        return NFK_OK;
    }
    std::vector<uint32_t> pid(n);
    GATHER(w, d.ev_pid, d.ev_base, d.n_tiles, d.ev_tcap, n, pid.data());
    GATHER(w, d.ev_old_h, d.ev_base, d.n_tiles, d.ev_tcap, n, ev_old_h);
    GATHER(w, d.ev_new_h, d.ev_base, d.n_tiles, d.ev_tcap, n, ev_new_h);
    for (size_t i = 0; i < n; i++)
        if ((int)pid[i] < d.n_if) ev_old_h[i] = ev_new_h[i] = 0;  // (unwritten for other events)
    return NFK_OK;
}

int nfk_read_rec_events(void* world, int32_t* re_obj, uint32_t* re_rrc, uint64_t* re_old, uint64_t* re_new) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    int r = read_ctrl(w, &c);
    if (r) return r;
    const Dev& d = w->d;
    const size_t n = c.n_re;
    GATHER(w, d.re_rrc, d.re_base, d.n_rtiles, d.re_tcap, n, re_rrc);
    GATHER(w, d.re_old, d.re_base, d.n_rtiles, d.re_tcap, n, re_old);
    GATHER(w, d.re_new, d.re_base, d.n_rtiles, d.re_tcap, n, re_new);
    // each event's slot: its record tile's first slot + the slot field of its word (kRrcHost)
    std::vector<uint32_t> rb((size_t)d.n_rtiles + 1, 0);
    if (n) HIPCHK(hipMemcpy(rb.data(), d.re_base, rb.size() * 4, hipMemcpyDeviceToHost));
    for (int t = 0; t < d.n_rtiles; t++)
        for (uint32_t i = rb[(size_t)t]; i < rb[(size_t)t + 1] && i < n; i++) {
            re_obj[i] = w->obj_of_slot[(size_t)t * kRTile + (re_rrc[i] >> kRrcSitShift)];
            re_rrc[i] &= kRrcHost;
        }
    return NFK_OK;
}

int nfk_read_fired(void* world, int32_t* fi_obj, int32_t* fi_kind, int32_t* fi_remain) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    int r = read_ctrl(w, &c);
    if (r) return r;
    const Dev& d = w->d;
    const size_t n = c.n_fi;
    std::vector<uint32_t> sl(n);
    GATHER(w, d.fi_slot, d.fi_base, d.n_tiles, d.fi_tcap, n, sl.data());
    GATHER(w, d.fi_kind, d.fi_base, d.n_tiles, d.fi_tcap, n, (uint32_t*)fi_kind);
    GATHER(w, d.fi_remain, d.fi_base, d.n_tiles, d.fi_tcap, n, fi_remain);
    for (size_t i = 0; i < n; i++) fi_obj[i] = w->obj_of_slot[sl[i]];
    return NFK_OK;
}

int nfk_read_fanout(void* world, uint32_t* msg_off, int32_t* msg_rcpt_obj) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    Ctrl c;
    int r = check_fanout(w);
    if (r) return r;
    r = read_ctrl(w, &c);
    if (r) return r;
    if (c.msg_extent > (unsigned long long)w->d.msg_cap) return fail(NFK_ERR_CAPACITY, "fan-out not recovered");
    const Dev& d = w->d;
    const size_t nm = (size_t)frame_msgs(w, c);
    // each tile's messages are one run at msg_base[tile]; the dense CSR walks tiles in order
    const int ntt = d.n_tiles + (d.has_recops ? d.n_rtiles : 0);
    std::vector<uint32_t> mb(ntt), mc(ntt), eb(d.n_tiles + 1), rb(d.n_rtiles + 1);
    std::vector<uint64_t> db(ntt);
    if (ntt) {
        HIPCHK(hipMemcpy(mb.data(), d.msg_base, (size_t)ntt * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(mc.data(), d.t_msg, (size_t)ntt * 4, hipMemcpyDeviceToHost));
    }
    HIPCHK(hipMemcpy(eb.data(), d.ev_base, eb.size() * 4, hipMemcpyDeviceToHost));
    if (d.has_recops) HIPCHK(hipMemcpy(rb.data(), d.re_base, rb.size() * 4, hipMemcpyDeviceToHost));
    uint64_t acc = 0;
    for (int t = 0; t < ntt; t++) {
        db[t] = acc;
        acc += mc[t];
    }
    if (acc != nm) return fail(NFK_ERR_STATE, "message cursor and tile counts disagree");
    // (tiles k_tick / k_records fanned out themselves store no offsets: counted on the device below)
    const bool ev_counted = w->last_tcap != 0, rec_counted = d.has_recops && w->last_rtcap;
    if (!ev_counted) GATHER(w, d.ev_moff, d.ev_base, d.n_tiles, d.ev_tcap, (size_t)c.n_ev, msg_off);
    if (d.has_recops && !rec_counted)
        GATHER(w, d.re_moff, d.re_base, d.n_rtiles, d.re_tcap, (size_t)c.n_re, msg_off + c.n_ev);
    if (!ev_counted)
        for (int t = 0; t < d.n_tiles; t++)
            for (uint32_t i = eb[t]; i < eb[t + 1]; i++) msg_off[i] = (uint32_t)(msg_off[i] - mb[t] + db[t]);
    if (d.has_recops && !rec_counted)
        for (int t = 0; t < d.n_rtiles; t++)
            for (uint32_t i = rb[t]; i < rb[t + 1]; i++) {
                const int tg = d.n_tiles + t;
                msg_off[c.n_ev + i] = (uint32_t)(msg_off[c.n_ev + i] - mb[tg] + db[tg]);
            }
    const size_t ncnt = (ev_counted ? (size_t)c.n_ev : 0) + (rec_counted ? (size_t)c.n_re : 0);
    if (ncnt) {  // counted on the device (k_counted_moff) from the dense bases
        std::vector<uint32_t> dbv(ntt);
        for (int t = 0; t < ntt; t++) dbv[t] = (uint32_t)db[t];
        // (a world-owned scratch, grown as needed: no allocation per call, nothing to free on errors)
        r = dev_reserve(w, (void**)&w->moff_tmp, &w->moff_tmp_cap, ((size_t)ntt + (size_t)c.n_ev + (size_t)c.n_re) * 4);
        if (r) return r;
        uint32_t* const tmp = w->moff_tmp;
        HIPCHK(hipMemcpy(tmp, dbv.data(), (size_t)ntt * 4, hipMemcpyHostToDevice));
        uint32_t* out = tmp + ntt;  // [n_ev ++ n_re], as msg_off
        hipError_t ce = hipSuccess;
        if (ev_counted && c.n_ev) {
            const unsigned g = (unsigned)std::max(1, std::min(d.n_tiles, 4096));
            hipLaunchKernelGGL(k_counted_moff, dim3(g), dim3(kTPB), 0, w->stream, d, 0, out, (const uint32_t*)tmp);
            ce = hipGetLastError();
            if (ce == hipSuccess)
                ce = hipMemcpyAsync(msg_off, out, (size_t)c.n_ev * 4, hipMemcpyDeviceToHost, w->stream);
        }
        if (ce == hipSuccess && rec_counted && c.n_re) {
            const unsigned g = (unsigned)std::max(1, std::min(d.n_rtiles, 4096));
            hipLaunchKernelGGL(k_counted_moff, dim3(g), dim3(kTPB), 0, w->stream, d, 1, out + c.n_ev, (const uint32_t*)tmp);
            ce = hipGetLastError();
            if (ce == hipSuccess)
                ce = hipMemcpyAsync(msg_off + c.n_ev, out + c.n_ev, (size_t)c.n_re * 4, hipMemcpyDeviceToHost, w->stream);
        }
        if (ce == hipSuccess) ce = hipStreamSynchronize(w->stream);
        if (ce != hipSuccess) return fail(NFK_ERR_HIP, std::string("k_counted_moff: ") + hipGetErrorString(ce));
    }
    msg_off[c.n_ev + c.n_re] = (uint32_t)nm;
    // the runs cover [0, extent) with gaps when property tiles sit at a stride
    const size_t ext = (size_t)c.msg_extent;
    std::vector<uint32_t> rc(ext);
    if (ext) HIPCHK(hipMemcpy(rc.data(), d.msg_rcpt, ext * 4, hipMemcpyDeviceToHost));
    for (int t = 0; t < ntt; t++)
        for (uint32_t i = 0; i < mc[t]; i++) msg_rcpt_obj[db[t] + i] = w->obj_of_slot[rc[(size_t)mb[t] + i]];
    return NFK_OK;
}

// The rank of every object's NFGUID among all objects of the world (rank_d, on the device), for
// ordering the fired list as mObjectScheduleMap does: the sorted order is kept and new objects are
// merged into it (an O(n) merge in frames that created objects).
static int update_guid_ranks(World* w) {
    if (w->rank_n == w->n_obj && w->rank_d) return NFK_OK;
    std::vector<int32_t> fresh(w->n_obj - w->rank_n);
    std::iota(fresh.begin(), fresh.end(), w->rank_n);
    auto less = [w](int32_t a, int32_t b) { return guid_less(w, a, b); };
    std::sort(fresh.begin(), fresh.end(), less);
    std::vector<int32_t> merged(w->n_obj);
    std::merge(w->guid_sorted.begin(), w->guid_sorted.end(), fresh.begin(), fresh.end(), merged.begin(), less);
    w->guid_sorted.swap(merged);
    std::vector<int32_t> rank(w->n_obj);
    for (int32_t i = 0; i < w->n_obj; i++) rank[w->guid_sorted[i]] = i;
    if ((size_t)w->n_obj > w->rank_cap) {
        HIPCHK(hipStreamSynchronize(w->stream));
        if (w->rank_d) HIPCHK(hipFree(w->rank_d));
        w->rank_d = nullptr;
        w->rank_cap = (size_t)w->n_obj + w->n_obj / 4 + 1024;
        HIPCHK(hipMalloc((void**)&w->rank_d, w->rank_cap * 4));
    }
    HIPCHK(hipMemcpy(w->rank_d, rank.data(), rank.size() * 4, hipMemcpyHostToDevice));
    w->rank_n = w->n_obj;
    return NFK_OK;
}

int nfk_read_frame(void* world, uint32_t what, nfk_frame_host* o) {
    World* w = (World*)world;
    if (!w || !o) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    memset(o, 0, sizeof *o);
    int r = check_fanout(w);
    if (r) return r;
    Ctrl c;
    r = read_ctrl(w, &c);
    if (r) return r;
    if (c.err & (kErrFanBound | kErrTouch))
        return fail(NFK_ERR_DEVICE, "the frame's outputs are incomplete (device error " + std::to_string(c.err) + ")");
    if (c.msg_extent > (unsigned long long)w->d.msg_cap) return fail(NFK_ERR_CAPACITY, "fan-out not recovered");
    const Dev& d = w->d;
    const bool fired = what & NFK_READ_FIRED, order = fired && (what & NFK_READ_FIRED_GUID_ORDER);
    const bool events = what & NFK_READ_EVENTS, fan = events && (what & NFK_READ_FANOUT);
    const bool heads = events && d.n_obj > 0;
    const size_t ne = events ? c.n_ev : 0, nr = events && d.has_recops ? c.n_re : 0, nf = fired ? c.n_fi : 0;
    const size_t nm = fan ? (size_t)frame_msgs(w, c) : 0;
    const int ntt = d.n_tiles + (d.has_recops ? d.n_rtiles : 0);
    // one region, the same layout on the device and in pinned host memory
    size_t at = 0;
    auto take = [&](size_t bytes) {
        const size_t a = at;
        at += (bytes + 255) & ~(size_t)255;
        return a;
    };
    const size_t o_eo = take(ne * 4), o_ep = take(ne * 4), o_eold = take(ne * 8), o_enew = take(ne * 8);
    const size_t o_eoh = take(heads ? ne * 8 : 0), o_enh = take(heads ? ne * 8 : 0);
    const size_t o_ro = take(nr * 4), o_rr = take(nr * 4), o_rold = take(nr * 8), o_rnew = take(nr * 8);
    const size_t o_fo = take(nf * 4), o_fk = take(nf * 4), o_fr = take(nf * 4);
    const size_t o_mo = take(fan ? (ne + nr + 1) * 4 : 0), o_mr = take(nm * 4);
    const size_t total = at;
    // device scratch: dense message bases, and the fired sort's keys / indices / unsorted copies
    const size_t s_db = 0, s_keys = (((size_t)ntt + 1) * 4 + 255) & ~(size_t)255;
    const size_t s_k2 = s_keys + ((nf * 8 + 255) & ~(size_t)255), s_i1 = s_k2 + ((nf * 8 + 255) & ~(size_t)255);
    const size_t s_i2 = s_i1 + ((nf * 4 + 255) & ~(size_t)255), s_f = s_i2 + ((nf * 4 + 255) & ~(size_t)255);
    size_t s_tmp = s_f + 3 * ((nf * 4 + 255) & ~(size_t)255);
    size_t sort_bytes = 0;
    int key_bits = 5;
    if (order) {
        r = update_guid_ranks(w);
        if (r) return r;
        while ((1ll << (key_bits - 5)) < (long long)std::max(w->n_obj, 1)) key_bits++;
        HIPCHK(rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (uint32_t*)nullptr, (uint32_t*)nullptr, nf, 0, key_bits, w->stream));
    }
    const size_t scratch = s_tmp + sort_bytes + 256;
    if (total > w->fr_cap || scratch > w->fr_scap) {
        HIPCHK(hipStreamSynchronize(w->stream));
        if (total > w->fr_cap) {
            if (w->fr_dev) HIPCHK(hipFree(w->fr_dev));
            if (w->fr_pin) HIPCHK(hipHostFree(w->fr_pin));
            w->fr_dev = nullptr;
            w->fr_pin = nullptr;
            w->fr_cap = total + total / 4 + 4096;
            HIPCHK(hipMalloc(&w->fr_dev, w->fr_cap));
            HIPCHK(hipHostMalloc((void**)&w->fr_pin, w->fr_cap, hipHostMallocDefault));
        }
        if (scratch > w->fr_scap) {
            if (w->fr_scr) HIPCHK(hipFree(w->fr_scr));
            w->fr_scr = nullptr;
            w->fr_scap = scratch + scratch / 4 + 4096;
            HIPCHK(hipMalloc(&w->fr_scr, w->fr_scap));
        }
    }
    char* D = (char*)w->fr_dev;
    char* S = (char*)w->fr_scr;
    const unsigned gt = (unsigned)std::max(1, std::min(d.n_tiles, 4096));
    const unsigned grt = (unsigned)std::max(1, std::min(d.n_rtiles, 4096));
    const int32_t* so = w->slot_obj_d;
    // the fired list's destination: dense, or the sort's unsorted copies
    int32_t* const fo = (int32_t*)(order ? S + s_f : D + o_fo);
    int32_t* const fk = (int32_t*)(order ? S + s_f + ((nf * 4 + 255) & ~(size_t)255) : D + o_fk);
    int32_t* const fr = (int32_t*)(order ? S + s_f + 2 * ((nf * 4 + 255) & ~(size_t)255) : D + o_fr);
    // events and fired list of the property tiles in one launch (k_compact_frame)
    if (ne || nf)
        hipLaunchKernelGGL(k_compact_frame, dim3(gt), dim3(kTPB), 0, w->stream, d, so,
                           ne ? (int32_t*)(D + o_eo) : nullptr, (uint32_t*)(D + o_ep), (uint64_t*)(D + o_eold),
                           (uint64_t*)(D + o_enew), nf ? fo : nullptr, (uint32_t*)fk, fr);
    if (ne) {
        if (heads) {
            hipLaunchKernelGGL(k_compact_h, dim3(gt), dim3(kTPB), 0, w->stream, d.ev_old_h, (uint64_t*)(D + o_eoh),
                               d.ev_pid, d.ev_base, d.n_tiles, d.ev_tcap, d.n_if);
            hipLaunchKernelGGL(k_compact_h, dim3(gt), dim3(kTPB), 0, w->stream, d.ev_new_h, (uint64_t*)(D + o_enh),
                               d.ev_pid, d.ev_base, d.n_tiles, d.ev_tcap, d.n_if);
        }
    }
    if (nr) {
        hipLaunchKernelGGL(k_compact_rec, dim3(grt), dim3(kTPB), 0, w->stream, d.re_rrc, (int32_t*)(D + o_ro),
                           (uint32_t*)(D + o_rr), d.re_base, d.n_rtiles, d.re_tcap, so);
        hipLaunchKernelGGL(k_compact<uint64_t>, dim3(grt), dim3(kTPB), 0, w->stream, d.re_old, (uint64_t*)(D + o_rold),
                           d.re_base, d.n_rtiles, d.re_tcap);
        hipLaunchKernelGGL(k_compact<uint64_t>, dim3(grt), dim3(kTPB), 0, w->stream, d.re_new, (uint64_t*)(D + o_rnew),
                           d.re_base, d.n_rtiles, d.re_tcap);
    }
    if (fan && ntt && nm == 0) {
        // (a frame without messages, e.g. Tutorial3's private World Sets: every offset is 0)
        HIPCHK(hipMemsetAsync(D + o_mo, 0, (ne + nr + 1) * 4, w->stream));
    } else if (fan && ntt) {
        uint32_t* db = (uint32_t*)(S + s_db);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, w->stream, d.t_msg, db, ntt);
        // (tiles k_tick / k_records fanned out themselves store no offsets: counted here)
        if (ne && w->last_tcap)
            hipLaunchKernelGGL(k_counted_moff, dim3(gt), dim3(kTPB), 0, w->stream, d, 0, (uint32_t*)(D + o_mo), db);
        else if (ne)
            hipLaunchKernelGGL(k_compact_moff, dim3(gt), dim3(kTPB), 0, w->stream, d.ev_moff, (uint32_t*)(D + o_mo),
                               d.ev_base, d.n_tiles, d.ev_tcap, d.msg_base, db);
        if (nr && w->last_rtcap)
            hipLaunchKernelGGL(k_counted_moff, dim3(grt), dim3(kTPB), 0, w->stream, d, 1, (uint32_t*)(D + o_mo) + ne, db);
        else if (nr)
            hipLaunchKernelGGL(k_compact_moff, dim3(grt), dim3(kTPB), 0, w->stream, d.re_moff,
                               (uint32_t*)(D + o_mo) + ne, d.re_base, d.n_rtiles, d.re_tcap, d.msg_base + d.n_tiles,
                               db + d.n_tiles);
        // the CSR's last offset: the frame's message count
        HIPCHK(hipMemcpyAsync(D + o_mo + (ne + nr) * 4, db + ntt, 4, hipMemcpyDeviceToDevice, w->stream));
        if (nm)
            hipLaunchKernelGGL(k_runs_obj, dim3((unsigned)std::min(ntt, 8192)), dim3(kTPB), 0, w->stream, d.msg_rcpt,
                               (int32_t*)(D + o_mr), d.msg_base, d.t_msg, db, ntt, so);
    } else if (fan) {
        HIPCHK(hipMemsetAsync(D + o_mo, 0, 4, w->stream));
    }
    if (nf) {
        if (order && nf <= (size_t)kSmallSort) {
            hipLaunchKernelGGL(k_fired_small, dim3((unsigned)((nf + kTPB - 1) / kTPB)), dim3(kTPB), 0, w->stream, (const int32_t*)fo,
                               (const int32_t*)fk, (const int32_t*)fr, w->rank_d, (int32_t*)(D + o_fo),
                               (int32_t*)(D + o_fk), (int32_t*)(D + o_fr), (int)nf);
        } else if (order) {
            const unsigned g = (unsigned)((nf + kTPB - 1) / kTPB);
            uint64_t* k1 = (uint64_t*)(S + s_keys);
            uint64_t* k2 = (uint64_t*)(S + s_k2);
            uint32_t* i1 = (uint32_t*)(S + s_i1);
            uint32_t* i2 = (uint32_t*)(S + s_i2);
            hipLaunchKernelGGL(k_fired_keys, dim3(g), dim3(kTPB), 0, w->stream, fo, fk, w->rank_d, k1, i1, (int)nf);
            size_t sb = sort_bytes;
            HIPCHK(rocprim::radix_sort_pairs(S + s_tmp, sb, k1, k2, i1, i2, nf, 0, key_bits, w->stream));
            hipLaunchKernelGGL(k_permute3, dim3(g), dim3(kTPB), 0, w->stream, i2, fo, fk, fr, (int32_t*)(D + o_fo),
                               (int32_t*)(D + o_fk), (int32_t*)(D + o_fr), (int)nf);
        }
    }
    HIPCHK(hipGetLastError());
    if (total) HIPCHK(hipMemcpyAsync(w->fr_pin, D, total, hipMemcpyDeviceToHost, w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
    char* H = w->fr_pin;
    o->n_ev = (int64_t)ne;
    o->n_re = (int64_t)nr;
    o->n_fi = (int64_t)nf;
    o->n_msgs = (int64_t)nm;
    o->bytes = (int64_t)total;
    if (events) {
        o->ev_obj = (const int32_t*)(H + o_eo);
        o->ev_pid = (const int32_t*)(H + o_ep);
        o->ev_old = (const uint64_t*)(H + o_eold);
        o->ev_new = (const uint64_t*)(H + o_enew);
        if (heads) {
            o->ev_old_h = (const uint64_t*)(H + o_eoh);
            o->ev_new_h = (const uint64_t*)(H + o_enh);
        }
        o->re_obj = (const int32_t*)(H + o_ro);
        o->re_rrc = (const uint32_t*)(H + o_rr);
        o->re_old = (const uint64_t*)(H + o_rold);
        o->re_new = (const uint64_t*)(H + o_rnew);
    }
    if (fired) {
        o->fi_obj = (const int32_t*)(H + o_fo);
        o->fi_kind = (const int32_t*)(H + o_fk);
        o->fi_remain = (const int32_t*)(H + o_fr);
    }
    if (fan) {
        o->msg_off = (const uint32_t*)(H + o_mo);
        o->msg_rcpt = (const int32_t*)(H + o_mr);
    }
    return NFK_OK;
}

int nfk_rank_top(void* world, int32_t pid, int32_t k, int32_t* n_out, int64_t* guid_head, int64_t* guid_data,
                 double* score) {
    World* w = (World*)world;
    if (!w || !n_out || (k > 0 && (!guid_head || !guid_data || !score))) return fail(NFK_ERR_ARG, "null argument");
    if (!w->committed) return fail(NFK_ERR_STATE, "commit first");
    if (pid < 0 || pid >= w->n_if || k < 0) return fail(NFK_ERR_ARG, "bad property / k (int or float properties rank)");
    *n_out = 0;
    const Dev& d = w->d;
    if (k == 0 || d.N == 0) return NFK_OK;
    HIPCHK(hipStreamSynchronize(w->stream));
    unsigned* hist = nullptr;
    HIPCHK(hipMalloc((void**)&hist, 257 * 4));
    const unsigned grid = std::min<unsigned>((d.N + kTPB - 1) / kTPB, 2048);
    // radix select of the k-th largest key, 8 bits at a time
    uint64_t prefix = 0, pmask = 0;
    uint64_t above = 0;  // entities with a key above the current prefix range
    for (int shift = 56; shift >= 0; shift -= 8) {
        hipError_t e1 = hipMemsetAsync(hist, 0, 256 * 4, w->stream);
        hipLaunchKernelGGL(k_rank_hist, dim3(grid), dim3(kTPB), 0, w->stream, d, pid, prefix, pmask, shift, hist);
        unsigned h[256];
        hipError_t e2 = hipMemcpyAsync(h, hist, sizeof h, hipMemcpyDeviceToHost, w->stream);
        hipError_t e3 = hipStreamSynchronize(w->stream);
        if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
            (void)hipFree(hist);
            return fail(NFK_ERR_HIP, "rank histogram failed");
        }
        int dg = 255;
        for (; dg > 0; dg--) {
            if (above + h[dg] >= (uint64_t)k) break;
            above += h[dg];
        }
        prefix |= (uint64_t)dg << shift;
        pmask |= 0xFFull << shift;
    }
    // everything at or above the k-th key: fewer than k above it plus all its ties
    const uint64_t thr = prefix;
    unsigned cnt = 0;
    std::vector<int64_t> cand;  // (slot, raw property word) pairs
    for (int attempt = 0; attempt < 2; attempt++) {
        const unsigned cap = attempt == 0 ? (unsigned)std::min<int64_t>(4 * (int64_t)k + 1024, d.N) : cnt;
        int64_t* out = nullptr;
        HIPCHK(hipMalloc((void**)&out, (size_t)std::max(cap, 1u) * 16));
        HIPCHK(hipMemsetAsync(hist + 256, 0, 4, w->stream));
        hipLaunchKernelGGL(k_rank_collect, dim3(grid), dim3(kTPB), 0, w->stream, d, pid, thr, hist + 256, out, cap);
        HIPCHK(hipMemcpyAsync(&cnt, hist + 256, 4, hipMemcpyDeviceToHost, w->stream));
        HIPCHK(hipStreamSynchronize(w->stream));
        if (cnt <= cap) {
            cand.resize((size_t)cnt * 2);
            if (cnt) HIPCHK(hipMemcpy(cand.data(), out, (size_t)cnt * 16, hipMemcpyDeviceToHost));
            (void)hipFree(out);
            break;
        }
        (void)hipFree(out);
    }
    (void)hipFree(hist);
    // ZREVRANGE order: score desc, member (NFGUID::ToString, NFGUID.h:93) desc
    struct C { double s; int32_t o; std::string m; };
    std::vector<C> cs;
    cs.reserve(cand.size() / 2);
    for (size_t i = 0; i < cand.size(); i += 2) {
        const int32_t sl = (int32_t)cand[i];
        const uint64_t raw = (uint64_t)cand[i + 1];
        double sc;
        if (pid < d.n_int) sc = (double)(int64_t)raw;
        else memcpy(&sc, &raw, 8);
        const int32_t o = w->obj_of_slot[sl];
        cs.push_back({sc, o, std::to_string(w->gh[o]) + "-" + std::to_string(w->gd[o])});
    }
    std::sort(cs.begin(), cs.end(), [](const C& a, const C& b) { return a.s != b.s ? a.s > b.s : a.m > b.m; });
    const int32_t n = (int32_t)std::min<size_t>(cs.size(), (size_t)k);
    for (int32_t i = 0; i < n; i++) {
        guid_head[i] = w->gh[cs[i].o];
        guid_data[i] = w->gd[cs[i].o];
        score[i] = cs[i].s;
    }
    *n_out = n;
    return NFK_OK;
}

static void copy_msg(const std::string& m, char* out, int32_t cap) {
    if (!out || cap <= 0) return;
    const size_t n = std::min(m.size(), (size_t)cap - 1);
    memcpy(out, m.data(), n);
    out[n] = 0;
}

int nfk_jit_status(void* world, int32_t* on, char* msg, int32_t cap) {
    World* w = (World*)world;
    if (!w || !on) return fail(NFK_ERR_ARG, "null argument");
    *on = w->jit_fn != nullptr;
    copy_msg(w->jit_msg, msg, cap);
    return NFK_OK;
}

int nfk_jit_preview(int32_t n_int, int32_t n_flt, int32_t n_class, int32_t n_kind, const uint8_t* prop_flags,
                    const nfk_op* ops, const int32_t* n_ops, int32_t compile, int32_t* ok, char* src, int32_t src_cap,
                    char* msg, int32_t msg_cap) {
    if (!ok || !prop_flags || (n_kind && (!ops || !n_ops)) || n_int < 0 || n_flt < 0 || n_int > NFK_MAX_INT_PROPS ||
        n_flt > NFK_MAX_FLT_PROPS || n_class <= 0 || n_class >= NFK_MAX_CLASSES || n_kind < 0 || n_kind > NFK_MAX_KINDS)
        return fail(NFK_ERR_ARG, "bad schema");
    *ok = 0;
    std::unique_ptr<Tables> tab(new Tables());
    memset(tab.get(), 0, sizeof(Tables));
    const int np = n_int + n_flt;
    for (int c = 0; c < n_class; c++)
        for (int p = 0; p < np; p++) tab->pflags[c][p] = prop_flags[(size_t)c * np + p];
    for (int k = 0; k < n_kind; k++) {
        if (n_ops[k] < 0 || n_ops[k] > NFK_MAX_OPS) return fail(NFK_ERR_ARG, "bad op count");
        tab->nops[k] = n_ops[k];
        for (int i = 0; i < n_ops[k]; i++) tab->ops[k][i] = ops[(size_t)k * NFK_MAX_OPS + i];
    }
    std::vector<int> wp, rp;
    const bool u_ok = build_u_tables(*tab, n_kind, wp, rp);
    Dev d{};
    d.n_kind = n_kind;
    fill_u_dev(d, *tab, wp, rp, u_ok);
    if (!u_ok) {
        copy_msg("working set does not fit k_tick (k_tick_touch runs)", msg, msg_cap);
        return NFK_OK;
    }
    const char* es = getenv("NFGPU_JIT_SPEC");
    uint32_t nt = kJitNtDefault;
    if (const char* en = getenv("NFGPU_JIT_NT")) nt = (uint32_t)strtoul(en, nullptr, 0);
    const std::string s = jit_schema_source(*tab, d, es && es[0] == '1', nt);
    copy_msg(s, src, src_cap);
    if (!compile) {
        *ok = 1;
        return NFK_OK;
    }
    const int u = std::max(d.n_u, 1), waves = kWavesJit;
    JitBuild b = jit_compile(s, waves, u);
    *ok = b.ok;
    copy_msg(b.ok ? b.lowered + " (" + std::to_string(b.code.size()) + " B code object)\n" + b.log : b.log, msg, msg_cap);
    return NFK_OK;
}

int nfk_set_profiling(void* world, int32_t on) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    w->profiling = on != 0;
    return NFK_OK;
}

int nfk_kernel_times(void* world, double* ms, int64_t* launches, int64_t* bytes) {
    World* w = (World*)world;
    if (!w || !ms || !launches || !bytes) return fail(NFK_ERR_ARG, "null argument");
    int r = drain_timings(w);
    if (r) return r;
    if (w->committed) {
        Ctrl c;
        r = read_ctrl(w, &c);
        if (r) return r;
        uint64_t tb[3];
        r = read_tallies(w, tb);
        if (r) return r;
        for (int k = 0; k < 3; k++) w->kt_bytes[k] = (int64_t)tb[k];
    }
    for (int i = 0; i < KT_N; i++) {
        ms[i] = w->kt_ms[i];
        launches[i] = w->kt_n[i];
        bytes[i] = w->kt_bytes[i];
    }
    return NFK_OK;
}

int nfk_membership_stats(void* world, int64_t* n_full, int64_t* n_seg, double* host_ms_full, double* host_ms_seg) {
    World* w = (World*)world;
    if (!w || !n_full || !n_seg || !host_ms_full || !host_ms_seg) return fail(NFK_ERR_ARG, "null argument");
    *n_full = w->n_relayout_full;
    *n_seg = w->n_relayout_seg;
    *host_ms_full = w->ms_relayout_full;
    *host_ms_seg = w->ms_relayout_seg;
    return NFK_OK;
}

int nfk_reset_kernel_times(void* world) {
    World* w = (World*)world;
    if (!w) return fail(NFK_ERR_ARG, "null world");
    int r = drain_timings(w);
    if (r) return r;
    for (int i = 0; i < KT_N; i++) {
        w->kt_ms[i] = 0;
        w->kt_n[i] = 0;
    }
    if (w->committed) {
        Ctrl c;
        r = read_ctrl(w, &c);
        if (r) return r;
        // byte tallies restart from zero
        HIPCHK(hipMemset(w->d.tally, 0, (size_t)3 * kTallyN * 8 * 8));
        w->last_bytes[0] = w->last_bytes[1] = w->last_bytes[2] = 0;
    }
    return NFK_OK;
}

}  // extern "C"
