// nfgpu_device.hpp — device-side data layout and wave/block primitives for gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nfgpu.h"

namespace nfgpu {

constexpr int kTPB = 256;                 // 4 waves of 64
constexpr unsigned kSpinLimit = 1u << 22; // bounded spins (~0.2 s) before the error word is set

// device error word bits (Ctrl::err)
constexpr unsigned kErrSpin = 1, kErrEvCap = 2, kErrMsgCap = 4, kErrTouch = 8, kErrFiCap = 16, kErrReCap = 32;

// Control block.  Tickets are reset in-kernel by a later kernel of the same frame (k_fanout
// resets k_tick's, k_tick resets k_records'/k_fanout's); totals are overwritten by the last
// virtual block; the error word is sticky until nfk_summary_get clears it.  Look-back
// granules carry a per-frame tag, so nothing is memset per frame.
struct alignas(64) Ctrl {
    unsigned ticket_tick, ticket_rec, ticket_fan, err;                  // 16 B
    unsigned long long n_ev, n_fi, n_re, n_msgs;                        // 32 B
    unsigned long long pad0, pad1;                                      // 16 B
    unsigned long long bytes_tick, bytes_rec, bytes_fan, pad2;          // accumulated across frames
};

// Schedule table, one 16-byte hot record per (kind, slot) read every frame by the timer scan,
// and one 16-byte cold record read only when the heartbeat fires (NFCScheduleElement fields).
struct alignas(16) SchedHot {
    int64_t next;    // mnNextTriggerTime
    int32_t remain;  // mnRemainCount
    uint32_t state;  // bit0 present, bit1 forever (mbForever)
};
struct alignas(16) SchedCold {
    int64_t start;   // mnStartTime
    int32_t all;     // mnAllCount
    float interval;  // mfIntervalTime
};

// timing-only ablations (NFGPU_ABLATE env var); outputs are wrong when set
constexpr unsigned kAblTickLookback = 1, kAblFanLookback = 2, kAblPrograms = 4;

// record op compiled from the kind programs, sorted by (rec, col)
struct RecOp {
    int32_t kind, rec, col, code;
    int64_t a, b, c;
};

struct Tables {
    nfk_op ops[NFK_MAX_KINDS][NFK_MAX_OPS];
    int32_t nops[NFK_MAX_KINDS];
    uint8_t pflags[NFK_MAX_CLASSES][NFK_MAX_INT_PROPS + NFK_MAX_FLT_PROPS];
    uint8_t rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    RecOp recops[NFK_MAX_OPS];
    int32_t n_recops;
    int32_t rec_rows[NFK_MAX_RECORDS], rec_cols[NFK_MAX_RECORDS];
    uint32_t kind_has_recop;  // bit k: kind k has record ops
};

// Everything a kernel needs, passed by value.
struct Dev {
    int32_t N, cap, n_int, n_flt, n_kind, n_rec;
    int64_t now;
    uint32_t tag;
    int32_t has_recops;
    const Tables* tab;
    Ctrl* ctrl;
    // SoA entity columns, column-major [col][cap]
    int64_t* icol;
    double* fcol;
    // schedules [kind][cap]
    SchedHot* s_hot;
    SchedCold* s_cold;
    uint8_t* e_flags;  // bit0: a RemoveSchedule(self, name) is queued (owns the remove-list key)
    // queued SetProperty* calls, sorted by slot (stable)
    uint32_t* ext_head;  // [cap] 0 = none, else 1 + first op index
    const uint32_t* x_slot;
    const uint32_t* x_pid;
    const uint64_t* x_bits;
    int32_t n_x;
    uint32_t* fired_mask;  // [cap]
    // records: cells [cap][cols][rows], used masks [cap]
    uint64_t* rcells[NFK_MAX_RECORDS];
    uint64_t* rused[NFK_MAX_RECORDS];
    // membership (slots sorted by (scene, group, guid))
    const int32_t* seg_of;
    const uint8_t* cls;
    const uint8_t* isplayer;
    const int32_t* seg_pl_off;
    const int32_t* pl_slot;
    const int32_t* pl_rank;  // [cap] rank of a player slot in its group's player list, -1 otherwise
    // [cap] fan-out descriptor: bits 0-31 first player index of the slot's group in pl_slot,
    // 32-45 players in the group, 46-59 1 + rank of the slot among them (0 = not a player),
    // 60-63 class id
    const uint64_t* fan_desc;
    uint32_t ablate;
    // outputs
    uint32_t* ev_slot; uint32_t* ev_pid; uint64_t* ev_old; uint64_t* ev_new; int64_t ev_cap;
    uint32_t* fi_slot; uint32_t* fi_kind; int32_t* fi_remain; int64_t fi_cap;
    uint32_t* re_slot; uint32_t* re_rrc; uint64_t* re_old; uint64_t* re_new; int64_t re_cap;
    uint32_t* msg_off; uint32_t* msg_rcpt; int64_t msg_cap;
    // look-back granules
    unsigned long long* g_ev;
    unsigned long long* g_fi;
    unsigned long long* g_re;
    unsigned long long* g_msg;
};

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

// ---------------- decoupled look-back (single-pass ordered compaction) ----------------
// Granule = {tag:16 | status:2 | value:46}, one 8-byte relaxed agent-scope store (sc1):
// the data is the flag (MI355X guide, Guideline 16 recipe R2).  Polls are relaxed
// agent-scope loads; a bounded spin sets the error word instead of hanging.
constexpr unsigned long long kStAgg = 1, kStInc = 2;
__device__ __forceinline__ unsigned long long gmk(unsigned tag, unsigned long long st, unsigned long long v) {
    return ((unsigned long long)(tag & 0xFFFF) << 48) | (st << 46) | (v & ((1ull << 46) - 1));
}
__device__ __forceinline__ void gstore(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gload(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by all 64 lanes of ONE wave.  Publishes `agg` for virtual block `vb`,
// returns the exclusive prefix of all blocks before it, publishes the inclusive value.
__device__ __forceinline__ unsigned long long lookback(unsigned long long* gran, unsigned vb, unsigned tag,
                                                       unsigned long long agg, Ctrl* ctrl) {
    const int lane = threadIdx.x & 63;
    if (vb == 0) {
        if (lane == 0) gstore(&gran[0], gmk(tag, kStInc, agg));
        return 0;
    }
    if (lane == 0) gstore(&gran[vb], gmk(tag, kStAgg, agg));
    unsigned long long excl = 0;
    long long base = (long long)vb - 1;
    unsigned spins = 0;
    while (true) {
        const long long idx = base - lane;
        bool valid = true, inc = true;
        unsigned long long v = 0;
        if (idx >= 0) {
            const unsigned long long g = gload(&gran[idx]);
            const unsigned gt = (unsigned)(g >> 48);
            const unsigned long long st = (g >> 46) & 3;
            valid = gt == (tag & 0xFFFF) && st != 0;
            inc = st == kStInc;
            v = g & ((1ull << 46) - 1);
        }
        const unsigned long long incmask = __ballot(valid && inc);
        const unsigned long long invmask = __ballot(!valid);
        const int first_inc = incmask ? __builtin_ctzll(incmask) : 64;
        const unsigned long long need = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1);
        if (invmask & need) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(&ctrl->err, kErrSpin);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum(lane <= first_inc ? v : 0ull);
        if (first_inc < 64) break;
        base -= 64;
    }
    if (lane == 0) gstore(&gran[vb], gmk(tag, kStInc, excl + agg));
    return excl;
}

}  // namespace nfgpu
