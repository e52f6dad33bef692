// nfgpu_device.hpp — device-side data layout and wave/block primitives for gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nfgpu.h"

namespace nfgpu {

constexpr int kTPB = 256;     // 4 waves of 64 (128-slot tiles measured: not faster, profiles/r04t_ab_tile128.txt)
constexpr int kTile = 256;    // slots per property/fired tile (one k_tick workgroup)
#ifndef NFGPU_RTILE
#define NFGPU_RTILE 64
#endif
constexpr int kRTile = NFGPU_RTILE;  // slots per record-event tile (one k_records wave; <= 64)
static_assert(kRTile >= 1 && kRTile <= 64, "a record tile is at most one wave of slots");
// A record event's word in the raw device outputs (re_rrc): record << 16 | row << 8 | column, the
// row-event op (0 a cell's update, 1 AddRow, 2 Remove, 3 Clear / Cover) in bits 24-25, and the slot's
// index within its record tile in bits 26-31 (the tile is where the event sits), so no slot word is
// stored per event.  The host formats carry op << 24 | record << 16 | row << 8 | column.
constexpr uint32_t kRrcHost = 0x03FFFFFFu;
constexpr int kRrcSitShift = 26;

// device error word bits (Ctrl::err); kErrRemain: a fired heartbeat's remain was read from an LDS slot
// this launch never wrote (only with kAblCheckRem)
constexpr unsigned kErrMsgCap = 4, kErrTouch = 8, kErrFanBound = 16, kErrRemain = 32;

// Control block: frame totals written by k_scan_tiles, byte tallies accumulated across frames,
// the error word is sticky until nfk_summary_get clears it.  msg_extent = end of the last tile's
// message run (= n_msgs unless k_tick's fan-out placed property tiles at a fixed stride).
struct alignas(64) Ctrl {
    unsigned err, pad_u[3];                                             // 16 B
    unsigned long long n_ev, n_fi, n_re, n_msgs;                        // 32 B
    unsigned long long msg_extent, n_msgs_ptiles;  // n_msgs_ptiles: messages of fixed-stride tiles
    unsigned long long bytes_tick, bytes_rec, bytes_fan, pad2;          // accumulated across frames
};

// Schedule table, one 16-byte hot record per (kind, slot) read every frame by the timer scan,
// and one 16-byte cold record read only when the heartbeat fires (NFCScheduleElement fields).
struct alignas(16) SchedHot {
    int64_t next;    // mnNextTriggerTime
    int32_t remain;  // mnRemainCount
    uint32_t state;  // kSt* bits below; bits 4..31 = step ms (signed 28-bit) when kStStep
};
// SchedHot::state.  The reference reschedules with next = start + step * (all - remain)
// (SM:71-72, step = (int64)(interval * 1000)).  Between two fires (all - remain) grows by one,
// so next advances by exactly `step` — except at the first fire after AddSchedule (next stays
// start + step) and once a forever schedule's remain has wrapped past INT32_MIN (the int32
// difference wraps).  The hot record therefore carries step and a fired-once bit, and only
// those two cases (or a step that does not fit 28 bits) read the cold record.
constexpr uint32_t kStPresent = 1, kStForever = 2, kStFired = 4, kStStep = 8;
__host__ __device__ __forceinline__ int64_t st_step(uint32_t st) { return (int64_t)((int32_t)st >> 4); }
__host__ __device__ __forceinline__ uint32_t st_pack_step(int64_t step) {
    return (step >= -(1ll << 27) && step < (1ll << 27)) ? (kStStep | ((uint32_t)step << 4)) : 0u;
}
struct alignas(16) SchedCold {
    int64_t start;   // mnStartTime
    int32_t all;     // mnAllCount
    float interval;  // mfIntervalTime
};

// timing-only ablations (NFGPU_ABLATE env var); outputs are wrong when set
constexpr unsigned kAblPrograms = 4;
constexpr unsigned kAblPerKind = 8;  // not an ablation: force the per-kind operand path (outputs stay exact)
constexpr unsigned kAblWaves6 = 16, kAblWaves8 = 32;  // k_tick register budgets (outputs stay exact)
constexpr unsigned kAblWaves5 = 8192;                  // (6 is the default)
constexpr unsigned kAblNoRun = 512, kAblNoLoads = 1024, kAblNoEmit = 2048;  // timing only (k_tick)
constexpr unsigned kAblNoWriteBack = 1u << 18, kAblNoSchedStore = 1u << 19;  // timing only (k_tick)
constexpr unsigned kAblNoFiStore = 128, kAblNoEvStore = 256;  // timing only (k_tick): no fired-list / event-array stores
constexpr unsigned kAblGroupColumns = 1u << 20, kAblSigGroups = 1u << 21;  // column layouts (outputs exact)
constexpr unsigned kAblNoPad = 1u << 22;  // columns / schedule kinds at power-of-two strides (outputs exact)
constexpr unsigned kAblFanWin16 = 1u << 24, kAblFanWin32 = 1u << 25;  // k_tick fan-out LDS window up to 16 / 32 recipients (outputs exact)
constexpr unsigned kAblFan1 = 1u << 26;      // k_tick fan-out: one recipient per lane (the round-1 form; outputs exact)
constexpr unsigned kAblFanNoWin = 1u << 30;  // k_tick fan-out: lane groups for every run length, no LDS window (outputs exact)
constexpr unsigned kAblTinyTcap = 1u << 27;  // test hook: k_tick's fan-out bound set to 4 messages (kErrFanBound)
constexpr unsigned kAblForceMsgCap = 1u << 29;  // test hook: the frame's ranks also raise kErrMsgCap
// four u32 at a dword-aligned address (gfx950 global memory allows it; one 16-byte store)
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
// Pad between consecutive property columns and schedule-kind arrays (bytes): with cap a power of
// two, unpadded columns sit exactly 2^k bytes apart and one entity's values of every column fall
// on the same HBM channel.
constexpr int64_t kColPad = 2304;
constexpr unsigned kAblScanInFrame = 131072;  // k_scan_tiles in every frame, not on first read
constexpr unsigned kAblScanKernel = 1u << 28;  // dense ranks by k_scan_tiles in small worlds too (outputs exact)
// k_tick ranks its own tiles up to this many (one agent-scope add per tile on one address: they
// serialise at ~7 ns each, profiles/r08s_last_arrival_ranks_ab.txt, so only small worlds gain)
constexpr int kLbMaxTiles = 256;
constexpr unsigned kAblNoFuse = 4096;  // fan-out in k_fanout instead of k_tick's tail (outputs stay exact)
// a check, outputs exact: k_tick marks every kind's remain slot (s_rem) unwritten at its start and
// raises kErrRemain when the fired list reads one for a counted heartbeat that the schedule scan
// did not write (a counted heartbeat's remain is >= 0 after a fire; a forever one's may be the
// sentinel itself, so those are not checked) (the r10w
// hipRTC fired-list corruption read such slots: DESIGN.md §3)
constexpr unsigned kAblCheckRem = 64;
constexpr int32_t kRemUnset = (int32_t)0x80000001;

// Where row r of a record sits in its slot's [rows] vector of one column: the used rows first, in
// row order, then the unused rows in row order (a stable partition by the used-row mask, so the
// mask alone maps rows to places and back).  A wave reading the used rows of a column reads one
// dense run of popcount(used) cells instead of the whole row-vector; an unused row keeps its
// cells (RC:1086-1107: Remove does not clear them).  rowm: the record's row mask.
__host__ __device__ inline uint32_t rec_pos(uint64_t used, uint64_t rowm, int r) {
    const uint64_t below = (1ull << r) - 1;  // (r < 64)
    return ((used >> r) & 1) ? (uint32_t)__builtin_popcountll(used & below)
                             : (uint32_t)(__builtin_popcountll(used & rowm) + __builtin_popcountll(~used & rowm & below));
}
__host__ __device__ inline uint64_t rec_rowm(int rows) { return rows >= 64 ? ~0ull : ((1ull << rows) - 1); }

// record op compiled from the kind programs, sorted by (rec, col)
struct RecOp {
    int32_t kind, rec, col, code;
    int64_t a, b, c;
};

// Frame working set U (k_tick).  Slots [0, kMaxW) hold properties that may be written this
// frame: the program destinations (fixed at commit, property-id order) followed by this frame's
// queued-SetProperty properties; slots [kMaxW, kMaxU) hold properties programs only read.
constexpr int kMaxU = 16, kMaxW = 12;
constexpr uint8_t kNoU = 0xFF;
static_assert(kMaxW == NFK_MAX_TOUCH, "writable slots = touch capacity");

// record op as k_records sees it (Dev::rops, kernel-argument space, so every field is a scalar):
// cells/used of its record, its shape, and the [gfirst, glast] span of ops on the same record
struct RecOpX {
    uint64_t* cells;
    uint64_t* used;
    int64_t a, b, c;
    int32_t kind, rec, col, code, rows, cols, gfirst, glast;
};

constexpr int kMaxProps = NFK_MAX_PROPS;
static_assert(NFK_MAX_INT_PROPS + NFK_MAX_FLT_PROPS <= NFK_MAX_PROPS, "property id space");

// a kind-program op in scalar-loadable form (32/64-bit fields only: gfx950 has no byte-sized
// scalar loads): code | flags << 8 | dst << 16, and the U slots of dst/a/b/c one per byte
struct OpX {
    uint32_t cfd;
    uint32_t slots;
    int64_t a, b, c;
    // NFK_GUARD: 0x80000000 | NFK_GUARD_* << 8 | the guard's U slot, and with NFK_GUARD_PROP
    // 0x40000000 | the compared property's U slot << 16, else the guard's constant (13 bits, signed)
    // << 16; else 0
    uint32_t gd;
};
// an NFK_GUARD op's condition on the guard property's current value g and what it is compared to
// (h: another int property's current value under NFK_GUARD_PROP, else the constant NFK_GUARD_K)
__host__ __device__ __forceinline__ bool guard_ok(uint32_t cmp, int64_t g, int64_t h = 0) {
    return cmp == NFK_GUARD_GT0 ? g > h : cmp == NFK_GUARD_LE0 ? g <= h : cmp == NFK_GUARD_NE0 ? g != h : g == h;
}

struct Tables {
    nfk_op ops[NFK_MAX_KINDS][NFK_MAX_OPS];
    OpX opx[NFK_MAX_KINDS][NFK_MAX_OPS];
    // property storage: property p of slot e is the 64-bit word pmem[p_off[p] + e * p_str[p]].
    // Properties that one heartbeat program touches together share a column group stored
    // interleaved ([cap][group size]), so a sparse heartbeat reads one line per entity.
    int64_t p_off[kMaxProps];
    int32_t p_str[kMaxProps];
    uint32_t umask[NFK_MAX_KINDS];                 // kind k's U slots: writable bits | read-only indices << 16
    uint8_t opu[NFK_MAX_KINDS][NFK_MAX_OPS][4];    // U slot of dst, a, b, c (0x80 | r: read-only r; kNoU = immediate)
    uint8_t opg[NFK_MAX_KINDS][NFK_MAX_OPS];       // U slot of an NFK_GUARD op's guard property (kNoU: none)
    uint8_t opg2[NFK_MAX_KINDS][NFK_MAX_OPS];      // U slot of the property it is compared to (NFK_GUARD_PROP; kNoU: 0)
    // property -> writable U slot (a program destination), kNoU otherwise.  A queued Set of a
    // property with a slot joins that slot's diff; any other queued Set is a "standalone" event.
    uint8_t w_slot[kMaxProps];
    int32_t nops[NFK_MAX_KINDS];
    uint8_t pflags[NFK_MAX_CLASSES][kMaxProps];
    uint8_t rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    RecOp recops[NFK_MAX_REC_OPS];
    int32_t n_recops;
    int32_t rec_rows[NFK_MAX_RECORDS], rec_cols[NFK_MAX_RECORDS];
    uint32_t kind_has_recop;  // bit k: kind k has record ops
    uint8_t rec_ctype[NFK_MAX_RECORDS][NFK_MAX_REC_COLS];  // 0 = int64, 1 = f64
};

// Everything a kernel needs, passed by value.
struct Dev {
    int32_t N, cap, n_int, n_flt, n_kind, n_rec, n_class;
    int32_t n_obj;   // object (NFGUID) properties: prop ids [n_if, n_if + n_obj), two words per entity
    int32_t n_if;    // n_int + n_flt: the first object property id
    int32_t s_kstr;  // kind stride of s_hot / s_cold in records: cap + a pad (see kColPad)
    int64_t now;
    int32_t has_recops;
    int32_t has_pre;     // RemoveSchedule(self, name) calls are queued this frame (e_flags live)
    const Tables* tab;
    Ctrl* ctrl;
    // property words (see Tables::p_off / p_str)
    uint64_t* pmem;
    // schedules [kind][cap]
    SchedHot* s_hot;
    SchedCold* s_cold;
    uint8_t* e_flags;  // bit0: a RemoveSchedule(self, name) is queued (owns the remove-list key)
    // queued SetProperty* calls folded into (slot, property) GROUPS, sorted by (slot, property);
    // group g's calls are x_bits[x_first[g], x_first[g + 1]) in call order.  k_sets applies each
    // group through the change predicates before the frame's heartbeat scan and leaves the
    // frame-start value in x_old[g] and the value after the group in x_new[g].
    uint32_t* ext_head;  // [cap] 0 = none, else 1 + first group of the slot
    const uint32_t* x_slot;
    const uint32_t* x_pid;
    const uint32_t* x_first;  // [n_x + 1]
    const uint64_t* x_bits;
    uint64_t* x_old;
    uint64_t* x_new;
    // object-property groups (x_pid >= n_if): the NFGUID head halves of the calls and of the
    // group's frame-start / after values (x_bits / x_old / x_new hold the data halves)
    const uint64_t* x_bits_h;
    uint64_t* x_old_h;
    uint64_t* x_new_h;
    int32_t n_x;              // groups
    // a calls-only pass (nfk_execute_calls: nothing fires): the tiles with SetProperty groups;
    // k_tick's other tiles only write empty outputs.  Null: every tile runs.
    const uint8_t* tile_work;
    uint32_t* fired_mask;  // [cap]
    // queued SetRecordInt / SetRecordFloat calls folded into (slot, cell) GROUPS sorted by (slot,
    // rec << 16 | row << 8 | col), each group's calls rs_bits[rs_first[g], rs_first[g + 1]) in call
    // order.  k_rsets applies each group through NFCRecord's predicates before the frame and leaves
    // the frame-start cell in rs_old[g] and the value after the group in rs_new[g]; k_records
    // merges them into the slot's record events.
    uint32_t* rs_head;  // [cap] 0 = none, else 1 + the slot's index among the SetRecord slots
    const uint32_t* rs_slot;
    const uint32_t* rs_rrc;
    const uint32_t* rs_first;  // [n_rs + 1]
    const uint64_t* rs_bits;
    uint64_t* rs_old;
    uint64_t* rs_new;
    uint8_t* rs_has;           // the group's calls logged an Update: rs_old / rs_new = first old / last new
    int32_t n_rs;              // groups (rs_rrc bit 31: a group of a row-operation list, run by k_rrows)
    // record row operations (NFCRecord::AddRow / Remove, NFCKernelModule::ClearRecord) of this window:
    // one LIST per (slot, record) with row operations, sorted by (slot, record); a list's calls (its
    // row operations and that pair's SetRecord calls) in call order.  k_rrows runs each list; its row
    // events (op << 8 | row) go to rl_ev[rl_ev0[l] ...], rl_cnt[l] of them.
    int32_t n_rl;
    const uint32_t* rl_slot;
    const uint32_t* rl_rec;
    const uint32_t* rl_c0;     // [n_rl + 1] call range
    const uint32_t* rl_ev0;
    uint32_t* rl_cnt;
    uint32_t* rl_ev;
    const uint32_t* rc_code;   // op | row << 8 | col << 16 (op 0 SetRecord, 1 AddRow (row 0xFF: -1), 2 Remove, 3 Clear)
    const uint32_t* rc_aux;    // SetRecord: its group; AddRow: its values' index (0xFFFFFFFF: the initial 0s)
    const uint64_t* rc_bits;   // SetRecord: the value
    const uint64_t* rvals;     // AddRow values [][NFK_MAX_REC_COLS]
    const uint32_t* rss_l0;    // [n_rss] the slot's first list
    // the slots with groups (k_rset_slots: one wave each), their first group, and per slot its
    // record events and messages (counted before k_records) and where k_records placed them
    const uint32_t* rss_slot;
    const uint32_t* rss_g0;
    uint32_t* rss_ev;
    uint32_t* rss_msg;
    uint32_t* rss_pos;
    uint32_t* rss_pmsg;
    int32_t n_rss;
    // records: cells [cap][cols][rows] in packed row order (rec_pos), used masks [cap]
    uint64_t* rcells[NFK_MAX_RECORDS];
    uint64_t* rused[NFK_MAX_RECORDS];
    // membership (slots sorted by (scene, group, guid))
    const int32_t* pl_slot;
    // [cap] fan-out descriptor: bits 0-31 first player index of the slot's group in pl_slot,
    // 32-45 players in the group, 46-59 1 + rank of the slot among them (0 = not a player),
    // 60-63 class id
    const uint64_t* fan_desc;
    uint32_t ablate;
    RecOpX rops[NFK_MAX_REC_OPS];  // record ops sorted by (rec, col)
    int32_t n_rops;
    uint32_t rop_kinds;        // kinds with record ops
    // algorithmic-byte tallies: [3 kernels][kTallyN][8] (one 64-byte line per counter), spread
    // over kTallyN addresses so that workgroups do not serialise on one atomic
    unsigned long long* tally;
    // working set of the programs (k_tick, fixed at commit): properties of the U slots, their
    // columns, writable slots in property-id order
    int32_t n_w, n_u;         // writable slots [0, n_w), read-only slots [n_w, n_u)
    int32_t u_pid[kMaxU];
    uint64_t* u_col[kMaxU];   // property of slot e at u_col[j][e * u_str[j]]
    int32_t u_str[kMaxU];
    int32_t u_order[kMaxW];
    uint32_t u_lower[kMaxW];  // writable slots whose property id is below slot j's (event order)
    // per class: writable slots whose events go to the scene group (public, bits 0-15) and to the
    // entity itself only (private & !upload & !public, bits 16-31); GetBroadCastObject (AOI:531)
    uint32_t u_cmask[NFK_MAX_CLASSES];
    // tiles: property/fired tile t = slots [t*kTile, (t+1)*kTile); record tile r = slots
    // [r*kRTile, (r+1)*kRTile).  Outputs of a tile sit at [t*tile_cap, t*tile_cap + count).
    int32_t n_tiles, n_rtiles;
    int32_t ev_tcap, fi_tcap, re_tcap;
    uint32_t* t_ev;    // [n_tiles] dirty property events per tile (k_tick)
    uint32_t* t_fi;    // [n_tiles] fired heartbeats per tile (k_tick)
    uint32_t* t_re;    // [n_rtiles] dirty record cells per record tile (k_records)
    uint32_t* t_msg;   // [n_tiles + n_rtiles] fan-out messages per tile (prop tiles, then record tiles)
    uint32_t* ev_base; // [n_tiles + 1] exclusive scans (k_scan_tiles)
    uint32_t* fi_base; // [n_tiles + 1]
    uint32_t* re_base; // [n_rtiles + 1]
    uint32_t* msg_base;// [n_tiles + n_rtiles + 1] first message of each tile (k_scan_tiles)
    // lb_rank (small worlds): k_tick writes ev_base / fi_base / msg_base and the frame totals
    // itself — its last tile to publish counts scans them (lb_st [n_tiles][4] count words tagged
    // with lb_epoch, one epoch per launch; lb_cnt the arrivals; nfgpu_tick.hpp) — and no
    // k_scan_tiles runs for the frame
    uint64_t* lb_st;
    uint32_t* lb_cnt;
    uint32_t lb_epoch;
    int32_t lb_rank;
    // msg_tcap > 0: k_tick writes its tile's fan-out itself, property tile t's messages at
    // t * msg_tcap (an upper bound of one tile's messages this frame); record tiles follow densely
    uint32_t msg_tcap;
    int32_t fuse_fan;
    // fuse_rec: k_records writes its record tiles' fan-out itself (only with fuse_fan), record
    // tile r's messages at msg_rb0 + r * msg_rtcap (msg_rb0 = n_tiles * msg_tcap; msg_rtcap = an
    // upper bound of one record tile's messages: slots x cells the record ops may change x the
    // most recipients of one record event)
    int32_t fuse_rec;
    uint32_t msg_rb0, msg_rtcap;
    int32_t lds_words; // k_tick's dynamic LDS in 4-byte words (message window + staged players)
    // xcd_map: k_tick's workgroup b runs tile xcd_tile(b): the workgroups the dispatcher deals to
    // one XCD (b mod 8) take one contiguous range of tiles (their L2 holds neighbouring tiles)
    int32_t xcd_map;
    // outputs (tile-staged)
    uint32_t* ev_slot; uint32_t* ev_pid; uint64_t* ev_old; uint64_t* ev_new; uint32_t* ev_moff;
    uint32_t* fi_slot; uint32_t* fi_kind; int32_t* fi_remain;
    uint32_t* re_rrc; uint64_t* re_old; uint64_t* re_new; uint32_t* re_moff;  // (re_rrc: see kRrcHost)
    uint32_t* msg_rcpt; int64_t msg_cap;
    uint64_t* ev_old_h; uint64_t* ev_new_h;  // head halves of object-property events (n_obj > 0)
    // host-mapped error words [kErrHostWords]: a kernel that sets bit b of ctrl->err also stores 1
    // into err_host[log2 b], so the host sees it without a device read (nfk_outputs_get, nfk_execute)
    unsigned* err_host;
};

// The host-mapped error word is one word PER BIT (err_host[log2 bit] = 1): plain stores only, no
// read-modify-write over PCIe, and a later error never overwrites an earlier one's bit.
constexpr int kErrHostWords = 16;
__device__ __forceinline__ void dev_error(const Dev& d, unsigned bit) {
    atomicOr(&d.ctrl->err, bit);
    if (d.err_host) __hip_atomic_store(d.err_host + __builtin_ctz(bit), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kTallyN = 64, kTallyTick = 0, kTallyRec = 1, kTallyFan = 2;
__device__ __forceinline__ void tally_add(const Dev& d, int k, unsigned long long v) {
    atomicAdd(&d.tally[((size_t)k * kTallyN + (blockIdx.x % kTallyN)) * 8], v);
}

// ---------------- 64-lane primitives ----------------
__device__ __forceinline__ unsigned long long shfl_up_u64(unsigned long long v, int d) {
    unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
    lo = __shfl_up(lo, d, 64);
    hi = __shfl_up(hi, d, 64);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
    lo = __shfl_xor(lo, m, 64);
    hi = __shfl_xor(hi, m, 64);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = shfl_up_u64(v, d);
        if (lane >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_u64(v, m);
    return v;
}
__device__ __forceinline__ unsigned wave_incl_scan_u32(unsigned v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Tables through the constant address space: wave-uniform reads become scalar loads (s_load)
// instead of vector loads, so a kind program's op fields cost no vector memory round trip
typedef const __attribute__((address_space(4))) Tables CTables;
__device__ __forceinline__ CTables* ctab(const Tables* t) { return (CTables*)t; }

__device__ __forceinline__ uint64_t* prop_ptr(const Dev& d, uint32_t p, int e) {
    return d.pmem + d.tab->p_off[p] + (size_t)e * d.tab->p_str[p];
}

// fan_desc of a slot that holds no entity (slack of a scene group's slot range)
constexpr uint64_t kDeadDesc = 0xFull << 60;
__host__ __device__ __forceinline__ bool desc_dead(uint64_t desc) { return (desc >> 60) == 0xF; }

// Recipients of one dirty event (NFCSceneAOIModule::GetBroadCastObject, AOI:531-593):
// public -> every player of the group but self; private && !upload -> self; else none.
// a store at a 32-bit byte offset from a wave-uniform base (global store, SGPR base + VGPR offset:
// no 64-bit address arithmetic per lane); i * sizeof(T) must fit 32 bits
template <typename T>
__device__ __forceinline__ void st_off(T* base, uint32_t i, T x) {
    *(T*)((char*)base + i * (uint32_t)sizeof(T)) = x;
}
// loads / stores with the non-temporal hint when NT (global_load / global_store ... nt): data
// streamed once per frame, not worth keeping in L2 / the Infinity Cache for this frame
typedef uint32_t u32x4_v __attribute__((ext_vector_type(4)));
template <bool NT, typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
    if constexpr (!NT) {
        return *p;
    } else if constexpr (sizeof(T) == 16) {
        const u32x4_v v = __builtin_nontemporal_load((const u32x4_v*)p);
        T r;
        __builtin_memcpy(&r, &v, 16);
        return r;
    } else if constexpr (sizeof(T) == 8) {
        const uint64_t v = __builtin_nontemporal_load((const uint64_t*)p);
        T r;
        __builtin_memcpy(&r, &v, 8);
        return r;
    } else {
        static_assert(sizeof(T) == 4, "ld_nt: 4, 8 or 16 bytes");
        const uint32_t v = __builtin_nontemporal_load((const uint32_t*)p);
        T r;
        __builtin_memcpy(&r, &v, 4);
        return r;
    }
}
template <bool NT, typename T>
__device__ __forceinline__ void st_nt(T* p, T x) {
    if constexpr (!NT) {
        *p = x;
    } else if constexpr (sizeof(T) == 16) {
        u32x4_v v;
        __builtin_memcpy(&v, &x, 16);
        __builtin_nontemporal_store(v, (u32x4_v*)p);
    } else if constexpr (sizeof(T) == 8) {
        uint64_t v;
        __builtin_memcpy(&v, &x, 8);
        __builtin_nontemporal_store(v, (uint64_t*)p);
    } else {
        static_assert(sizeof(T) == 4, "st_nt: 4, 8 or 16 bytes");
        uint32_t v;
        __builtin_memcpy(&v, &x, 4);
        __builtin_nontemporal_store(v, (uint32_t*)p);
    }
}
// a vector of u32 (u32x2_a4 / u32x4_a4: dword-aligned) at a 32-bit byte offset from a wave-uniform base
template <bool NT, typename V>
__device__ __forceinline__ void st_vec(void* base, uint32_t byte_off, V x) {
    V* p = (V*)((char*)base + byte_off);
    if constexpr (NT)
        __builtin_nontemporal_store(x, p);
    else
        *p = x;
}
template <bool NT, typename T>
__device__ __forceinline__ void st_off_nt(T* base, uint32_t i, T x) {
    st_nt<NT>((T*)((char*)base + i * (uint32_t)sizeof(T)), x);
}
__device__ __forceinline__ unsigned event_msgs(uint64_t desc, uint8_t fl) {
    if (fl & NFK_PUBLIC) {
        const unsigned np = (unsigned)((desc >> 32) & 0x3FFF);
        const unsigned r1 = (unsigned)((desc >> 46) & 0x3FFF);
        return np - (r1 ? 1u : 0u);
    }
    if ((fl & NFK_PRIVATE) && !(fl & NFK_UPLOAD)) return 1;
    return 0;
}

}  // namespace nfgpu
