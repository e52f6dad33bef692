// nfgpu_tick.hpp — k_tick, the frame kernel, and its helpers, written over a SCHEMA POLICY:
// DynSchema reads the programs and the working set from Dev / Tables at run time (the kernels
// compiled into libnfgpu.so); a world's own policy, generated from its schema at commit
// (nfgpu_host.hip, jit_*), bakes them in as constants and straight-line code and is compiled
// with this same header by hipRTC.
#pragma once
#include "nfgpu_device.hpp"

namespace nfgpu {

// The next "standalone" dirty Set group of slot e at or after g: a queued Set of a property that
// no program writes, whose value changed over the frame (x_old != x_new).  Returns n_x when none.
__device__ __forceinline__ int next_standalone(const Dev& d, int g, int e) {
    for (; g < d.n_x && d.x_slot[g] == (uint32_t)e; g++)
        if (d.tab->w_slot[d.x_pid[g]] == kNoU &&
            (d.x_old[g] != d.x_new[g] || ((int)d.x_pid[g] >= d.n_if && d.x_old_h[g] != d.x_new_h[g])))
            return g;
    return d.n_x;
}
// recipients of a property event (GetBroadCastObject, AOI:531-593) of slot e's class
struct EvFan {
    uint32_t n;    // messages
    bool pub;      // to the scene group's players but self (else to self)
};
__device__ __forceinline__ EvFan ev_fan(const Dev& d, uint64_t desc, uint32_t pid) {
    const uint8_t fl = d.tab->pflags[desc >> 60][pid];
    return EvFan{event_msgs(desc, fl), (fl & NFK_PUBLIC) != 0};
}

// ---------------------------------------------------------------------------------
// Frame working set (k_tick).  A thread keeps its entity's values of the U slots in registers;
// program operands are addressed by wave-uniform slot numbers (Tables::opu), so a program runs
// without searching a written-property list.
#define NFK_U16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
static_assert(kMaxU == 16, "NFK_U16 enumerates kMaxU slots");

// A frame's U slots: the writable ones [0, n_w), then the read-only ones [n_w, n_w + n_r).  The
// kind tables name a read-only operand by its index r as 0x80 | r, so one table serves every
// frame; kU (template) = the register slots a k_tick variant keeps (n_w + n_r <= kU).
__device__ __forceinline__ uint32_t uslot(uint32_t raw, uint32_t n_w) {
    return (raw & 0x80u) ? n_w + (raw & 0x7Fu) : raw;
}
// j wave-uniform: a scalar branch to one register move
template <int kU>
__device__ __forceinline__ uint64_t uget(const uint64_t (&v)[kU], uint32_t j) {
    switch (__builtin_amdgcn_readfirstlane(j)) {
#define NFK_C(i) \
    case i:      \
        return v[(i) < kU ? (i) : 0];
        NFK_U16(NFK_C)
#undef NFK_C
    }
    return 0;
}
template <int kU>
__device__ __forceinline__ void uput(uint64_t (&v)[kU], uint32_t j, uint64_t x) {
    switch (__builtin_amdgcn_readfirstlane(j)) {
#define NFK_C(i)                   \
    case i:                        \
        v[(i) < kU ? (i) : 0] = x; \
        break;
        NFK_U16(NFK_C)
#undef NFK_C
    }
}
// An accepted Set of a program op, as (kind, op index, U slot, old bits, new bits): k_chain_u's log
// hook; k_tick passes this empty one, which compiles away.
struct NoSetLog {
    __device__ __forceinline__ void operator()(int, int, uint32_t, uint64_t, uint64_t) const {}
};
// The fired kinds' programs in schedule-name order on the register working set.  A Set that
// fails the reference's change predicate leaves the value as it was; wm collects the slots a
// Set changed at least once.
template <int kU, class Log = NoSetLog>
__device__ __forceinline__ void run_programs_u(uint64_t (&v)[kU], uint32_t& wm, const Tables* __restrict__ tab_,
                                               uint32_t fired, int n_kind, uint32_t n_w, const Log& log = Log()) {
    CTables* tab = ctab(tab_);
    for (int k = 0; k < n_kind; k++) {
        if (!((fired >> k) & 1)) continue;
        const int n = tab->nops[k];
        for (int i = 0; i < n; i++) {
            const uint32_t cfd = tab->opx[k][i].cfd, sl = tab->opx[k][i].slots;
            const uint32_t code = cfd & 0xFF, flags = (cfd >> 8) & 0xFF;
            const uint32_t u0 = uslot(sl & 0xFF, n_w), u1 = uslot((sl >> 8) & 0xFF, n_w);
            const uint32_t u2 = uslot((sl >> 16) & 0xFF, n_w), u3 = uslot(sl >> 24, n_w);
            const uint32_t gd = tab->opx[k][i].gd;
            if (gd && !guard_ok((gd >> 8) & 3u, (int64_t)uget(v, uslot(gd & 0xFF, n_w)),
                                (gd & 0x40000000u) ? (int64_t)uget(v, uslot((gd >> 16) & 0xFF, n_w))
                                                   : (int64_t)((int32_t)(gd << 3) >> 19)))  // the constant, bits 16..28
                continue;  // NFK_GUARD
            if (code == NFK_OP_IADD_CLAMP) {
                const int64_t cur = (int64_t)uget(v, u0);
                const int64_t a = (flags & NFK_A_PROP) ? (int64_t)uget(v, u1) : tab->opx[k][i].a;
                const int64_t lo = (flags & NFK_LO_PROP) ? (int64_t)uget(v, u2) : tab->opx[k][i].b;
                const int64_t hi = (flags & NFK_HI_PROP) ? (int64_t)uget(v, u3) : tab->opx[k][i].c;
                int64_t r = (int64_t)((uint64_t)cur + (uint64_t)a);
                r = r < lo ? lo : r;
                r = r > hi ? hi : r;
                uput(v, u0, (uint64_t)r);  // NFCProperty::SetInt (PR:273): r == cur changes nothing
                wm |= (r != cur) ? (1u << u0) : 0u;
                if (r != cur) log(k, i, u0, (uint64_t)cur, (uint64_t)r);
            } else if (code == NFK_OP_FLERP || code == NFK_OP_FAFFINE) {
                const uint64_t xb = uget(v, u0);
                const double x = __longlong_as_double((long long)xb);
                double r;
                if (code == NFK_OP_FLERP) {
                    const double tg = __longlong_as_double((long long)uget(v, u1));
                    const double dd = tg - x;
                    const double m = dd * __longlong_as_double(tab->opx[k][i].b);
                    r = x + m;
                } else {
                    const double m = x * __longlong_as_double(tab->opx[k][i].a);
                    r = m + __longlong_as_double(tab->opx[k][i].b);
                }
                const bool set = !(fabs(r - x) <= 1e-15);  // NFCProperty::SetFloat (PR:314): IsZeroDouble(v - cur)
                uput(v, u0, set ? (uint64_t)__double_as_longlong(r) : xb);
                wm |= set ? (1u << u0) : 0u;
                if (set) log(k, i, u0, xb, (uint64_t)__double_as_longlong(r));
            } else if (code == NFK_OP_ISET) {
                const uint64_t cur = uget(v, u0);
                const uint64_t r = (flags & NFK_A_PROP) ? uget(v, u1) : (uint64_t)tab->opx[k][i].a;
                uput(v, u0, r);  // NFCProperty::SetInt (PR:273): r == cur changes nothing
                wm |= (r != cur) ? (1u << u0) : 0u;
                if (r != cur) log(k, i, u0, cur, r);
            } else if (code == NFK_OP_FSET) {
                const uint64_t xb = uget(v, u0);
                const uint64_t rb = (flags & NFK_A_PROP) ? uget(v, u1) : (uint64_t)tab->opx[k][i].a;
                const double x = __longlong_as_double((long long)xb), r = __longlong_as_double((long long)rb);
                const bool set = !(fabs(r - x) <= 1e-15);  // NFCProperty::SetFloat (PR:314)
                uput(v, u0, set ? rb : xb);
                wm |= set ? (1u << u0) : 0u;
                if (set) log(k, i, u0, xb, rb);
            }
            // record ops run in k_records
        }
    }
}

// Block-wide exclusive scan of a packed 64-bit value (fields must not overflow into each other).
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v, unsigned long long* s_w,
                                                              unsigned long long& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long inc = wave_incl_scan(v);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    unsigned long long before = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < kTPB / 64; i++) {
        const unsigned long long x = s_w[i];
        before += (i < w) ? x : 0ull;
        total += x;
    }
    return before + inc - v;
}

// Element i (stride str elements) of a wave-uniform array.  A policy with kOff32 (its world's arrays
// are all under 4 GiB from their bases: nfgpu_jit.hpp) addresses it as the scalar base plus a 32-bit
// byte offset, so a column access is one saddr load on an offset shared by every column of the same
// stride, with no 64-bit address arithmetic or 64-bit address registers per lane.
// (The base goes through readfirstlane, which the compiler cannot see through: otherwise it
// re-associates base_k = s_hot + k * stride with the lane offset into one 64-bit lane address per
// kind.  Every base here is wave-uniform, so the first lane's is the base.)
template <class S, typename T>
__device__ __forceinline__ T* elem(T* base, uint32_t i, uint32_t str = 1) {
    if constexpr (S::kOff32) {
        const uint64_t p = (uint64_t)base;
        const uint64_t b = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)) << 32);
        typedef __attribute__((address_space(1))) char GChar;  // (global: the saddr forms)
        return (T*)((GChar*)b + i * (uint32_t)(sizeof(T) * str));
    } else
        return base + (size_t)i * str;
}

// The schema k_tick runs: the heartbeat kinds, the programs' working set (U slots) and its event
// order and fan-out classes.  DynSchema reads it at run time (Dev, kernel-argument scalars, and
// Tables through the constant address space); a generated policy (nfgpu_host.hip, jit_source)
// has the same members as constants and the programs as straight-line code on the registers.
struct DynSchema {
    static constexpr bool kStatic = false;
    static constexpr bool kOff32 = false;  // 64-bit element addresses (any world size)
    static constexpr uint32_t kSpecMask = 0;  // operands loaded before the fire test (none)
    // non-temporal hints (kNt* bits): none in the library's instantiations
    static constexpr uint32_t kNt = 0;
    // k_tick may rank a small world's tiles itself (Dev::lb_rank); a policy for a world of more than
    // kLbMaxTiles tiles compiles that code out (kLb = false) and the frame ranks by k_scan_tiles
    static constexpr bool kLb = true;
    static constexpr int kNK = NFK_MAX_KINDS;  // (an upper bound only)
    __device__ static int n_kind(const Dev& d) { return d.n_kind; }
    __device__ static int n_w(const Dev& d) { return d.n_w; }
    __device__ static uint32_t u_lower(const Dev& d, int j) { return d.u_lower[j]; }
    __device__ static int u_pid(const Dev& d, int j) { return d.u_pid[j]; }
    __device__ static int u_order(const Dev& d, int i) { return d.u_order[i]; }
    __device__ static uint32_t u_str(const Dev& d, int j) { return (uint32_t)d.u_str[j]; }
    // the event masks of the entity's class (Dev::u_cmask): a select over kernel-argument scalars,
    // no indexed copy and no barrier
    __device__ static uint32_t class_mask(const Dev& d, unsigned cls) {
        uint32_t cm = 0;
#pragma unroll
        for (int i = 0; i < NFK_MAX_CLASSES; i++) cm = cls == (unsigned)i ? d.u_cmask[i] : cm;
        return cm;
    }
    // the U slots the fired kinds read or write
    __device__ static uint32_t need(const Dev& d, uint32_t fired) {
        uint32_t need = 0;
        for (int k = 0; k < d.n_kind; k++)
            if ((fired >> k) & 1) {
                const uint32_t um = ctab(d.tab)->umask[k];  // writable bits | read-only bits << 16
                need |= (um & 0xFFFFu) | ((um >> 16) << d.n_w);
            }
        return need;
    }
    template <int kU, class Log = NoSetLog>
    __device__ static void run(uint64_t (&v)[kU], uint32_t& wm, const Dev& d, uint32_t fired, const Log& log = Log()) {
        run_programs_u(v, wm, d.tab, fired, d.n_kind, d.n_w, log);
    }
};

constexpr int kKindChunk = 8;  // schedule hot records loaded together per chunk
// non-temporal hint bits of a schema policy's kNt (NFGPU_JIT_NT for the hipRTC specialisation)
// kNtFanStore: the fan-out's LDS-window stores (16-byte aligned runs); kNtFanGroupStore: its lane-group
// stores (runs of 16 or more recipients, 16-byte stores at any dword)
constexpr uint32_t kNtSchedLoad = 1, kNtColLoad = 2, kNtEventStore = 4, kNtStateStore = 8, kNtFanStore = 16,
                   kNtFanGroupStore = 32;

// k_tick register budgets (waves per SIMD) by the frame's U slot count
constexpr int kWavesU8 = 8, kWavesU12 = 7;
constexpr int kWavesJit = 5;  // the hipRTC specialisation (nfgpu_jit.hpp; profiles/r11j_jit_waves_ab.txt)
constexpr long long kMsgStrideLimit = 1ll << 30;  // fixed-stride message runs: at most 4 GiB reserved

template <class S>
__device__ __forceinline__ void sched_load(const Dev& d, int e, int k0, SchedHot (&h)[kKindChunk]) {
    // kinds past n_kind re-read the chunk's first record (a cache hit); a static schema loads
    // exactly its kinds
    const int nk = S::n_kind(d) - k0;
#pragma unroll
    for (int j = 0; j < kKindChunk; j++)
        if (!S::kStatic || j < nk)
            h[j] = ld_nt<(S::kNt & kNtSchedLoad) != 0>(elem<S>(d.s_hot + (size_t)(k0 + (j < nk ? j : 0)) * d.s_kstr, (uint32_t)e));
}
// NFCScheduleModule::Execute (SM:51-81) for one object: its schedules in name order (kind id
// order).  The hot records of a chunk of kinds are loaded together (independent 16 B loads).
// Rescheduled / removed records are stored back.  Every load is issued without a branch and before
// the first use of any of them: a load under a branch is followed by a wait at the join, and a
// first use after the record stores would make the wave wait for the stores too (the vector
// memory counter retires in order), i.e. one round trip per kind or per store batch.
// kStore = false: the fire test only (k_chain re-runs it before k_tick; nothing is stored).
template <class S, bool kFirst, bool kStore = true>
__device__ __forceinline__ void sched_chunk(const Dev& d, int e, int k0, unsigned& bytes, uint64_t& desc,
                                            bool& dead, bool& taken, uint32_t& fired, int32_t* s_rem,
                                            bool oob) {
    SchedHot h[kKindChunk];
    uint8_t ef = 0;
    sched_load<S>(d, e, k0, h);
    if constexpr (kFirst) {
        desc = ld_nt<(S::kNt & kNtSchedLoad) != 0>(elem<S>(d.fan_desc, (uint32_t)e));
        ef = *elem<S>(d.e_flags, (uint32_t)e);  // (always allocated)
        __builtin_amdgcn_sched_barrier(0);  // the scheduler would hoist the first use and its wait
    }
    if constexpr (kFirst) {
        dead = oob || desc_dead(desc);  // a slack slot has no schedules; dead slots store nothing
        taken = d.has_pre && (ef & 1);  // std::map remove-list key already owned (SM:68)
        bytes += d.has_pre ? 1 : 0;
    }
#pragma unroll
    for (int j = 0; j < kKindChunk; j++) {
        const int k = k0 + j;
        if (k >= S::n_kind(d)) break;
        bytes += 16;
        bool fire = false;
        if (!dead && (h[j].state & kStPresent) && d.now > h[j].next) {
            const bool forever = h[j].state & kStForever;
            if (h[j].remain > 0 || forever) {
                fire = true;
                h[j].remain -= 1;
                fired |= 1u << k;
                const uint32_t st = h[j].state;
                if (h[j].remain <= 0 && !forever) {
                    if (!taken) {  // insert into the remove list succeeds for the first one only
                        h[j].state = 0;
                        taken = true;
                    }
                } else {
                    const bool first = !(st & kStFired);
                    if ((st & kStStep) && (first || !forever || h[j].remain < 0)) {
                        // next = start + step * (all - remain) without the cold record (see kSt*)
                        if (!first) h[j].next += st_step(st);
                    } else {
                        const SchedCold c = *elem<S>(d.s_cold + (size_t)k * d.s_kstr, (uint32_t)e);
                        bytes += 16;
                        const int64_t step = (int64_t)(c.interval * 1000.0f);
                        const int32_t done = (int32_t)((uint32_t)c.all - (uint32_t)h[j].remain);
                        h[j].next = c.start + step * (int64_t)done;
                    }
                    h[j].state = st | kStFired;
                }
                if (s_rem) s_rem[k * kTPB + threadIdx.x] = h[j].remain;  // for the fired list
                bytes += 16;
            }
        }
        if (kStore && fire && !(d.ablate & kAblNoSchedStore))
            st_nt<(S::kNt & kNtStateStore) != 0>(elem<S>(d.s_hot + (size_t)k * d.s_kstr, (uint32_t)e), h[j]);
    }
}
// Loads desc = fan_desc[e] with the first chunk; returns the fired-kind mask.  oob: a slot past N
// (e is then a valid slot re-read, treated as dead).
template <class S = DynSchema, bool kStore = true>
__device__ __forceinline__ uint32_t sched_scan(const Dev& d, int e, unsigned& bytes, uint64_t& desc,
                                               int32_t* s_rem = nullptr, bool oob = false) {
    uint32_t fired = 0;
    bool dead = true, taken = false;
    sched_chunk<S, true, kStore>(d, e, 0, bytes, desc, dead, taken, fired, s_rem, oob);
    for (int k0 = kKindChunk; k0 < S::n_kind(d); k0 += kKindChunk)
        sched_chunk<S, false, kStore>(d, e, k0, bytes, desc, dead, taken, fired, s_rem, oob);
    return fired;
}

// ---- dense ranks in k_tick (Dev::lb_rank, worlds of at most kLbMaxTiles tiles) ----
// What k_scan_tiles computes, without its launch: every tile publishes its three counts (events,
// fired, messages) at its block scan and counts itself in lb_cnt; the tile that arrives there last
// computes ev_base / fi_base / msg_base and the frame totals of all tiles at its end and resets
// lb_cnt for the next launch.  The counts are tagged with the launch's epoch (lb_st word:
// epoch << 32 | value), so the last tile waits for a word not yet visible instead of fencing,
// and nothing is cleared between launches.
__device__ __forceinline__ void lb_store(const Dev& d, int tile, int q, uint32_t v) {
    __hip_atomic_store(d.lb_st + (size_t)tile * 4 + q, ((uint64_t)d.lb_epoch << 32) | v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lb_load(const Dev& d, int tile, int q) {
    const uint64_t* p = d.lb_st + (size_t)tile * 4 + q;
    uint64_t s;
    while (((s = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != d.lb_epoch)
        __builtin_amdgcn_s_sleep(1);
    return (uint32_t)s;
}
// threads 0..2 publish; returns (thread 0) whether this tile arrived last
__device__ __forceinline__ bool lb_arrive(const Dev& d, int tile, uint32_t ev, uint32_t fi, uint32_t msg) {
    if (threadIdx.x < 3) lb_store(d, tile, threadIdx.x, threadIdx.x == 0 ? ev : threadIdx.x == 1 ? fi : msg);
    if (threadIdx.x != 0) return false;
    return __hip_atomic_fetch_add(d.lb_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)d.n_tiles - 1u;
}
// the whole workgroup of the last tile (n_tiles <= kLbMaxTiles = kTPB: one count per thread)
__device__ void lb_scan_all(const Dev& d, unsigned long long* s_w) {
    static_assert(kLbMaxTiles <= kTPB, "one tile's counts per thread");
    const int n = d.n_tiles, t = (int)threadIdx.x;
    uint32_t ev = 0, fi = 0, ms = 0;
    if (t < n) {
        ev = lb_load(d, t, 0);
        fi = lb_load(d, t, 1);
        ms = lb_load(d, t, 2);
    }
    unsigned long long tef, tm;
    const unsigned long long xef = block_excl_scan(((unsigned long long)fi << 32) | ev, s_w, tef);
    __syncthreads();
    block_excl_scan(ms, s_w, tm);
    if (t < n) {
        d.ev_base[t] = (uint32_t)xef;
        d.fi_base[t] = (uint32_t)(xef >> 32);
        d.msg_base[t] = (uint32_t)t * d.msg_tcap;
    }
    if (t == 0) {  // (k_scan_tiles' totals; no record tiles in such a frame)
        const unsigned long long ext = (unsigned long long)n * d.msg_tcap;
        d.ev_base[n] = (uint32_t)tef;
        d.fi_base[n] = (uint32_t)(tef >> 32);
        d.msg_base[n] = (uint32_t)ext;
        d.re_base[0] = 0;
        d.ctrl->n_ev = (uint32_t)tef;
        d.ctrl->n_fi = (uint32_t)(tef >> 32);
        d.ctrl->n_re = 0;
        d.ctrl->msg_extent = ext;
        d.ctrl->n_msgs_ptiles = tm;
        if (ext > (unsigned long long)d.msg_cap || (d.ablate & kAblForceMsgCap)) dev_error(d, kErrMsgCap);
        __hip_atomic_store(d.lb_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (every tile has arrived)
    }
}

// k_tick: one thread per slot, one workgroup per 256-slot tile, on the programs' working set
// (Dev::u_*, fixed at commit).  Every value the entity's frame touches is loaded in ONE batch of
// independent loads into registers; the fired kinds' programs run on those registers with
// wave-uniform slot numbers; the slots a program or a queued Set changed are diffed against their
// frame-start values (kept in LDS).  Queued SetProperty calls were applied by k_sets: a Set of a
// program destination joins that slot's diff (frame-start value = the group's x_old), a Set of any
// other property is a "standalone" event (x_old -> x_new) merged into the entity's events in
// property-id order.  Outputs of tile t are written densely at [t * tile_cap, t * tile_cap + count);
// k_scan_tiles, or in a small world this kernel's last tile (Dev::lb_rank), turns the counts into
// global ranks.
// kWPE: waves per SIMD the register allocation aims at.  The LDS image of the frame-start values
// is dynamic: n_w writable slots x kTPB.
// Dev::xcd_map: workgroup b (dealt to XCD b mod 8) -> a tile of that XCD's contiguous range
__device__ __forceinline__ int xcd_tile(int b, int n) {
    const int x = b & 7, i = b >> 3, q = n >> 3, r = n & 7;
    return x * q + min(x, r) + i;
}

// One tile of k_tick (the workgroup's; its LDS passed in).
template <int kU, class S>
__device__ __forceinline__ void tick_tile(const Dev& d, const int tile, unsigned long long* s_w, unsigned& s_bytes,
                                          uint32_t& s_lb_last, uint32_t* s_pb, uint64_t* s_o) {
    constexpr int kW = kU < kMaxW ? kU : kMaxW;  // writable register slots
    const int e = tile * kTile + (int)threadIdx.x;
    if (d.tile_work && !d.tile_work[tile]) {  // (block-uniform) a calls-only pass, no Set group here:
        if (d.has_recops && e < d.N) d.fired_mask[e] = 0;  // nothing fires, nothing is dirty
        if (threadIdx.x == 0) {
            d.t_ev[tile] = 0;
            d.t_fi[tile] = 0;
            d.t_msg[tile] = 0;
        }
        if (S::kLb && d.lb_rank) {
            const bool last = lb_arrive(d, tile, 0u, 0u, 0u);
            if (threadIdx.x == 0) s_lb_last = last;
            __syncthreads();
            if (s_lb_last) lb_scan_all(d, s_w);
        }
        return;
    }
    const bool fuse = d.msg_tcap != 0;  // this tile's fan-out is written here, at tile * msg_tcap
    if (threadIdx.x == 0) {
        s_bytes = 0;
        s_pb[0] = 0xFFFFFFFFu;
        s_pb[1] = 0;
        s_pb[2] = 1;
    }
    int32_t* s_rem = (int32_t*)(s_o + (size_t)S::n_w(d) * kTPB);  // [n_kind][kTPB] remain after a fire
    if (d.ablate & kAblCheckRem)  // (this thread's own column: read back only by this thread)
        for (int k = 0; k < S::n_kind(d); k++) s_rem[k * kTPB + threadIdx.x] = kRemUnset;
    unsigned bytes = 0;
    uint32_t fired = 0, xh = 0, wm = 0;
    uint64_t desc = kDeadDesc;
    uint64_t v[kU];
#pragma unroll
    for (int j = 0; j < kU; j++) v[j] = 0;
    {
        // descriptor and schedule records in one round trip, without a branch: slots past N (the
        // last tile) re-read slot N-1 and count as dead; a dead slot stores nothing
        const int ec = e < d.N ? e : d.N - 1;
        if constexpr (S::kSpecMask != 0) {
            // a policy may load every program operand with the schedule records, before it knows
            // which kinds fire: one round trip instead of two (sparse kinds' columns are read in
            // lines that mostly have to be fetched anyway)
            if (!(d.ablate & kAblNoLoads))
#pragma unroll
                for (int j = 0; j < kU; j++)
                    if ((S::kSpecMask >> j) & 1) v[j] = *elem<S>(d.u_col[j], (uint32_t)ec, S::u_str(d, j));
        }
        fired = sched_scan<S>(d, ec, bytes, desc, s_rem, e >= d.N);  // NFCScheduleModule::Execute (SM:51-81)
        desc = e < d.N ? desc : kDeadDesc;
        bytes = e < d.N ? bytes + 8 + 8u * (uint32_t)__builtin_popcount(S::kSpecMask) : 0u;
    }
    const bool live = !desc_dead(desc);
    // queued Set groups of this slot (k_sets ran them): program destinations among them
    uint32_t xset = 0;
    if (live && d.n_x) {
        xh = *elem<S>(d.ext_head, (uint32_t)e);
        bytes += 4;
        if (xh)
            for (int g = (int)xh - 1; g < d.n_x && d.x_slot[g] == (uint32_t)e; g++) {
                const uint32_t j = d.tab->w_slot[d.x_pid[g]];
                xset |= j != kNoU ? 1u << j : 0u;
                bytes += 8;
            }
    }
    uint32_t need = 0;
    if (live) {
        need = xset;
        if (!(d.ablate & kAblPrograms)) need |= S::need(d, fired);
        // one batch of independent loads: every value this entity's frame reads or writes
#pragma unroll
        for (int j = 0; j < kU; j++)
            if (((need >> j) & 1) && !((S::kSpecMask >> j) & 1) && !(d.ablate & kAblNoLoads)) {
                v[j] = ld_nt<(S::kNt & kNtColLoad) != 0>(elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j)));
                bytes += 8;
            }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < kW; j++)
            if (j < S::n_w(d) && ((need >> j) & 1)) s_o[j * kTPB + threadIdx.x] = v[j];
        // a Set program destination: its frame-start value is the value before the Set group
        if (xset) {
            for (int g = (int)xh - 1; g < d.n_x && d.x_slot[g] == (uint32_t)e; g++) {
                const uint32_t j = d.tab->w_slot[d.x_pid[g]];
                if (j != kNoU) s_o[j * kTPB + threadIdx.x] = d.x_old[g];
                bytes += j != kNoU ? 8 : 0;
            }
            wm = xset;
        }
        // the fired heartbeats' effect programs, in schedule-name order
        if (!(d.ablate & (kAblPrograms | kAblNoRun)) && fired) S::run(v, wm, d, fired);
    }
    // dirty diff against the frame-start values
    uint32_t dm = 0;
#pragma unroll
    for (int j = 0; j < kW; j++)
        if (((wm >> j) & 1) && v[j] != s_o[j * kTPB + threadIdx.x]) dm |= 1u << j;
    // a Set program destination that a program moved back to its frame-start value has no event,
    // but k_sets changed its column: write it back here (the dirty slots are written with their
    // events)
    if (xset & ~dm)
#pragma unroll
        for (int j = 0; j < kW; j++)
            if (j < S::n_w(d) && ((xset & ~dm) >> j) & 1) {
                *elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j)) = v[j];
                bytes += 8;
            }
    // fan-out message counts (event_msgs): a public property's event goes to every player of the
    // group but the entity itself, a private & !upload one to the entity only.  The message offset
    // of a slot's event = the counts of the dirty slots with lower property ids (Dev::u_lower).
    // the entity's class's event masks (Dev::u_cmask; class 15, a free slot: no slots): a select
    // over kernel-argument scalars, no indexed copy and no barrier
    const uint32_t cm = S::class_mask(d, (unsigned)(desc >> 60));
    const uint32_t pubm = cm & 0xFFFFu, privm = cm >> 16;
    const uint32_t r1 = (uint32_t)((desc >> 46) & 0x3FFF);
    const uint32_t npub = (uint32_t)((desc >> 32) & 0x3FFF) - (r1 ? 1u : 0u);
    unsigned nmsg = npub * __builtin_popcount(dm & pubm) + __builtin_popcount(dm & privm);
    unsigned nmax = (dm & pubm) ? npub : ((dm & privm) ? 1u : 0u);
    unsigned nd = __builtin_popcount(dm);
    // standalone Set events (properties no program writes): counted here, merged in property-id
    // order with the slots' events below
    unsigned nsd = 0;
    if (xh) {
        for (int g = next_standalone(d, (int)xh - 1, e); g < d.n_x; g = next_standalone(d, g + 1, e)) {
            const EvFan f = ev_fan(d, desc, d.x_pid[g]);
            nsd++;
            nmsg += f.n;
            nmax = max(nmax, f.n);
            bytes += 8;
        }
        nd += nsd;
    }
    // the entity's events in property-id order: dirty slots (u_order) merged with the standalone
    // groups; emit(rank, message offset, pid, slot or -1, group, recipients) per event
    auto walk = [&](auto&& emit) {
        int g = next_standalone(d, (int)xh - 1, e);
        unsigned at = 0, m = 0;
#pragma unroll 1
        for (int i = 0; i <= S::n_w(d); i++) {
            const int j = i < S::n_w(d) ? S::u_order(d, i) : -1;
            const uint32_t pj = j >= 0 ? (uint32_t)S::u_pid(d, j) : 0xFFFFFFFFu;
            while (g < d.n_x && d.x_pid[g] < pj) {
                const EvFan f = ev_fan(d, desc, d.x_pid[g]);
                emit(at, m, d.x_pid[g], -1, g, f);
                at++;
                m += f.n;
                g = next_standalone(d, g + 1, e);
            }
            if (j >= 0 && ((dm >> j) & 1)) {
                const bool pub = (pubm >> j) & 1;
                const EvFan f{pub ? npub : ((privm >> j) & 1u), pub};
                emit(at, m, pj, j, 0, f);
                at++;
                m += f.n;
            }
        }
    };
    const unsigned nf = __builtin_popcount(fired);
    const uint32_t dm_ = dm;
    // tile-local compaction: one block scan of (fired:16 | events:16 | messages:32)
    unsigned long long tot;
    const unsigned long long excl =
        block_excl_scan(((unsigned long long)nf << 48) | ((unsigned long long)nd << 32) | nmsg, s_w, tot);
    const unsigned pev0 = (unsigned)((excl >> 32) & 0xFFFF);
    unsigned pfi = (unsigned)(excl >> 48);
    const unsigned pmsg0 = (unsigned)excl, tmsg = (unsigned)tot;
    // (after the scan: its barrier orders thread 0's s_pb initialisation before these atomics, and
    // the barrier before the fan-out orders them before its reads)
    if (fuse) {  // the pl_slot run of the groups whose members have messages (they are contiguous)
        const uint32_t np = (uint32_t)((desc >> 32) & 0x3FFF);
        uint32_t lo = nmsg ? (uint32_t)desc : 0xFFFFFFFFu, hi = nmsg ? (uint32_t)desc + np : 0u;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, m, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, m, 64));
            nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, m, 64));
        }
        if ((threadIdx.x & 63) == 0 && hi) {
            atomicMin(&s_pb[0], lo);
            atomicMax(&s_pb[1], hi);
            atomicMax(&s_pb[2], nmax);
        }
    }
    // this tile's counts for the dense ranks; whether it is the last to publish them (thread 0)
    const bool lb_last = S::kLb && d.lb_rank && lb_arrive(d, tile, (unsigned)((tot >> 32) & 0xFFFF), (unsigned)(tot >> 48), tmsg);
    // this tile's output runs (wave-uniform bases, tile-local 32-bit offsets)
    const size_t ev0 = (size_t)tile * d.ev_tcap, fi0 = (size_t)tile * d.fi_tcap;
    uint32_t* const t_evm = d.ev_moff + ev0;

    if (live) {
        // write back the changed values; their events in property-id order (rank among the
        // entity's dirty slots by Dev::u_lower)
        if (nd && !(d.ablate & kAblNoEmit)) {
            uint32_t* const t_evs = d.ev_slot + ev0;
            uint32_t* const t_evp = d.ev_pid + ev0;
            uint64_t* const t_evo = d.ev_old + ev0;
            uint64_t* const t_evn = d.ev_new + ev0;
            if (!nsd) {
                // A thread's events sit at consecutive ranks, so two consecutive ones are stored
                // together (8-byte stores of the slot and pid words, 16-byte stores of the old and
                // new values, at any dword): one store per array covers most of a wave's run instead
                // of one per event slot with the lanes ~2.4 events apart
                // (tools/event_store_probe.hip: 22.4 -> 18.8 us for config[1]'s 2.5M events)
                constexpr bool kNE = (S::kNt & kNtEventStore) != 0;
                bool pend = false;  // an event held back to be stored with the next one
                uint32_t pa = 0, pp = 0;
                uint64_t po = 0, pn = 0;
#pragma unroll
                for (int j = 0; j < kW; j++) {
                    if (j >= S::n_w(d) || !((dm >> j) & 1)) continue;
                    const uint32_t below = dm & S::u_lower(d, j);
                    const uint32_t at = pev0 + __builtin_popcount(below);
                    const uint64_t nv = v[j], ov = s_o[j * kTPB + threadIdx.x];
                    const uint32_t pid = (uint32_t)S::u_pid(d, j);
                    if (!(d.ablate & kAblNoWriteBack)) st_nt<(S::kNt & kNtStateStore) != 0>(elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j)), nv);
                    if (!fuse)  // tile-local; k_fanout adds the tile's message base
                        st_off(t_evm, at, pmsg0 + npub * __builtin_popcount(below & pubm) +
                                              __builtin_popcount(below & privm));
                    if (d.ablate & kAblNoEvStore) {
                    } else if (pend && at == pa + 1) {  // (the writable slots are in property-id order)
                        st_vec<kNE>(t_evs, 4u * pa, u32x2_a4{(uint32_t)e, (uint32_t)e});
                        st_vec<kNE>(t_evp, 4u * pa, u32x2_a4{pp, pid});
                        st_vec<kNE>(t_evo, 8u * pa, u32x4_a4{(uint32_t)po, (uint32_t)(po >> 32), (uint32_t)ov, (uint32_t)(ov >> 32)});
                        st_vec<kNE>(t_evn, 8u * pa, u32x4_a4{(uint32_t)pn, (uint32_t)(pn >> 32), (uint32_t)nv, (uint32_t)(nv >> 32)});
                        pend = false;
                    } else {
                        if (pend) {
                            st_off_nt<kNE>(t_evs, pa, (uint32_t)e);
                            st_off_nt<kNE>(t_evp, pa, pp);
                            st_off_nt<kNE>(t_evo, pa, po);
                            st_off_nt<kNE>(t_evn, pa, pn);
                        }
                        pend = true;
                        pa = at;
                        pp = pid;
                        po = ov;
                        pn = nv;
                    }
                    bytes += 8 + 24;
                }
                if (pend && !(d.ablate & kAblNoEvStore)) {
                    st_off_nt<kNE>(t_evs, pa, (uint32_t)e);
                    st_off_nt<kNE>(t_evp, pa, pp);
                    st_off_nt<kNE>(t_evo, pa, po);
                    st_off_nt<kNE>(t_evn, pa, pn);
                }
            } else {
                // (rare: an entity with standalone Set events) write back the slots, then every
                // event by the merged walk, which reads the slots' new values back from their
                // columns so that no register of the working set stays live in it
#pragma unroll
                for (int j = 0; j < kW; j++)
                    if (j < S::n_w(d) && ((dm >> j) & 1)) {
                        *elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j)) = v[j];
                        bytes += 8;
                    }
                walk([&](unsigned at, unsigned m, uint32_t pid, int j, int g, EvFan) {
                    uint64_t ov, nv;
                    if (j >= 0) {
                        ov = s_o[j * kTPB + threadIdx.x];
                        nv = __hip_atomic_load(elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j)), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WAVEFRONT);
                    } else {  // (k_sets wrote the column)
                        ov = d.x_old[g];
                        nv = d.x_new[g];
                        if ((int)pid >= d.n_if) {  // an object property: its head halves beside
                            st_off(d.ev_old_h + ev0, pev0 + at, d.x_old_h[g]);
                            st_off(d.ev_new_h + ev0, pev0 + at, d.x_new_h[g]);
                            bytes += 16;
                        }
                    }
                    st_off(t_evs, pev0 + at, (uint32_t)e);
                    st_off(t_evp, pev0 + at, pid);
                    st_off(t_evo, pev0 + at, ov);
                    st_off(t_evn, pev0 + at, nv);
                    if (!fuse) st_off(t_evm, pev0 + at, pmsg0 + m);
                    bytes += 24;
                });
            }
        }
        uint32_t* const t_fis = d.fi_slot + fi0;
        uint32_t* const t_fik = d.fi_kind + fi0;
        int32_t* const t_fir = d.fi_remain + fi0;
        uint32_t fl = fired;
        while (fl) {
            const int k = __builtin_ctz(fl);
            fl &= fl - 1;
            constexpr bool kNE = (S::kNt & kNtEventStore) != 0;
            const int32_t rem = s_rem[k * kTPB + threadIdx.x];
            // (a forever heartbeat's remain may be any int32, the sentinel too: sched_edges worlds
            // wrap it through INT32_MIN; a counted one is >= 0 after a fire.  The forever bit is the
            // same before and after the scan, so the record's state is read whatever the L1 holds)
            if ((d.ablate & kAblCheckRem) && rem == kRemUnset &&
                !(elem<S>(d.s_hot + (size_t)k * d.s_kstr, (uint32_t)e)->state & kStForever))
                dev_error(d, kErrRemain);
            if (!(d.ablate & kAblNoFiStore)) {
                st_off_nt<kNE>(t_fis, pfi, (uint32_t)e);
                st_off_nt<kNE>(t_fik, pfi, (uint32_t)k);
                st_off_nt<kNE>(t_fir, pfi, rem);
            }
            pfi++;
            bytes += 12;
        }
        if (xh) *elem<S>(d.ext_head, (uint32_t)e) = 0;
    }
    if (d.has_recops && e < d.N) {  // slack slots too: a slot's previous occupant left a mask
        *elem<S>(d.fired_mask, (uint32_t)e) = fired;
        bytes += 4;
    }
    if (!fuse && !(d.ablate & kAblNoEmit)) bytes += 4 * nd;  // ev_moff
    // Fan-out of the tile's events (GetBroadCastObject, AOI:531-593; see k_fanout), into the
    // tile's fixed-stride run mb.  The LDS region of the frame-start image is reused for a chunk
    // of the tile's events as (first message, first player | slot, count | rank | public) triples
    // and the groups' player run; each event is then expanded by a group of L lanes (L = the
    // tile's largest recipient count rounded up to a power of two), so consecutive lane groups
    // store consecutive events' runs.  Runs of 16 or more recipients are stored that way straight
    // to HBM; shorter ones are written one thread per event into an LDS message window stored
    // with 16-byte stores (short runs stored directly leave lines partly written by several
    // waves, and lane groups would re-read each event's triple once per lane).
    if (fuse) {
        __syncthreads();  // s_pb; every read of s_o and s_rem is done: the region is reused
        uint32_t dm = dm_;
        const unsigned mb = (unsigned)tile * d.msg_tcap;
        const unsigned tev = (unsigned)((tot >> 32) & 0xFFFF);
        const bool fan = tmsg && tmsg <= d.msg_tcap;
        if (tmsg > d.msg_tcap && threadIdx.x == 0) dev_error(d, kErrFanBound);  // (host bound)
        // No per-event message offsets: the tile's run holds its events' recipients in event order
        // (the readers count through it: k_counted_moff)
        if (fan) {
            const unsigned R = (unsigned)d.lds_words;
            const uint32_t pb_lo = s_pb[0], npl = s_pb[1] > s_pb[0] ? s_pb[1] - s_pb[0] : 0u;
            const uint32_t nm = s_pb[2];
            const uint32_t L = nm <= 1 ? 1u : nm >= 64 ? 64u : 1u << (32 - __builtin_clz(nm - 1));
            const uint32_t sub = threadIdx.x & (L - 1);
            const bool win = !(d.ablate & kAblFanNoWin) &&
                             L < ((d.ablate & kAblFanWin32) ? 64u : (d.ablate & kAblFanWin16) ? 32u : 16u);
            const bool staged = npl <= R / 4;
            const unsigned room = R - (staged ? npl : 0u);
            // events per chunk: all of them, or what leaves the window half of the room
            const unsigned ecap = (min(tev, win ? room / 6u : room / 3u) + 3u) & ~3u;
            const unsigned W = win ? (room - 3u * ecap) & ~3u : 0u;  // window entries
            uint32_t* s_ev = (uint32_t*)s_o;
            uint32_t* s_win = s_ev + 3u * ecap;
            uint32_t* s_pl = s_ev + (R - npl);
            uint32_t* out = d.msg_rcpt + mb;
            if (staged) {
                for (uint32_t i = threadIdx.x; i < npl; i += kTPB) s_pl[i] = (uint32_t)d.pl_slot[pb_lo + i];
                bytes += 4 * ((npl + kTPB - 1 - threadIdx.x) / kTPB);
            }
            bytes += 4 * nmsg;
            for (unsigned c0 = 0; c0 < tev; c0 += ecap) {  // uniform
                const unsigned c1 = min(tev, c0 + ecap);
                // a runtime loop over the slots (an unrolled one gets hoisted out of the chunk loop
                // and spills: 12 slots x 4 values)
                if (nd && pev0 < c1 && pev0 + nd > c0) {
                    if (nsd) {
                        walk([&](unsigned at, unsigned m, uint32_t, int, int, EvFan f) {
                            const unsigned a = pev0 + at;
                            if (a < c0 || a >= c1) return;
                            uint32_t* x = s_ev + 3u * (a - c0);
                            x[0] = pmsg0 + m;
                            x[1] = f.pub ? (uint32_t)desc : (uint32_t)e;
                            x[2] = f.n | (r1 << 14) | (f.pub ? 0x80000000u : 0u);
                        });
                    } else {
#pragma unroll 1
                        for (int j = 0; j < S::n_w(d); j++) {
                            if (!((dm >> j) & 1)) continue;
                            const uint32_t below = dm & S::u_lower(d, j);
                            const uint32_t at = pev0 + __builtin_popcount(below);
                            if (at < c0 || at >= c1) continue;
                            const bool pub = (pubm >> j) & 1;
                            const uint32_t m = pmsg0 + npub * __builtin_popcount(below & pubm) +
                                               __builtin_popcount(below & privm);
                            const uint32_t n = pub ? npub : ((privm >> j) & 1u);
                            uint32_t* x = s_ev + 3u * (at - c0);
                            x[0] = m;
                            x[1] = pub ? (uint32_t)desc : (uint32_t)e;
                            x[2] = n | (r1 << 14) | (pub ? 0x80000000u : 0u);
                        }
                    }
                }
                __syncthreads();
                if (!win && !(d.ablate & kAblFan1)) {
                    // lane groups of L/4 lanes, four consecutive recipients per lane in one 16-byte
                    // store (dword-aligned: runs start anywhere); consecutive events' runs are
                    // adjacent, so a wave writes 64 x 16 B of one contiguous stretch
                    const uint32_t L4 = L >= 4 ? L / 4 : 1u, sub4 = threadIdx.x & (L4 - 1);
                    for (uint32_t i = threadIdx.x / L4; i < c1 - c0; i += kTPB / L4) {
                        const uint32_t ms = s_ev[3 * i], a = s_ev[3 * i + 1], b = s_ev[3 * i + 2];
                        const uint32_t n = b & 0x3FFFu, r1 = (b >> 14) & 0x3FFFu;
                        if (!(b >> 31)) {  // private & !upload: the entity itself (n is 0 or 1)
                            if (sub4 == 0 && n) out[ms] = a;
                            continue;
                        }
                        for (uint32_t p = 4 * sub4; p < n; p += 4 * L4) {  // every player of the group but self
                            uint32_t x[4];
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                const uint32_t pq = p + (uint32_t)q;
                                const uint32_t pp = pq + ((r1 && pq + 1 >= r1) ? 1u : 0u);
                                x[q] = pq < n ? (staged ? s_pl[a - pb_lo + pp] : (uint32_t)d.pl_slot[a + pp]) : 0u;
                            }
                            if (p + 4 <= n) {
                                if constexpr ((S::kNt & kNtFanGroupStore) != 0)
                                    __builtin_nontemporal_store(u32x4_a4{x[0], x[1], x[2], x[3]}, (u32x4_a4*)(out + ms + p));
                                else
                                    *(u32x4_a4*)(out + ms + p) = u32x4_a4{x[0], x[1], x[2], x[3]};
                            } else {
#pragma unroll
                                for (int q = 0; q < 3; q++)
                                    if (p + (uint32_t)q < n) out[ms + p + q] = x[q];
                            }
                        }
                    }
                } else if (!win) {
                    for (uint32_t i = threadIdx.x / L; i < c1 - c0; i += kTPB / L) {
                        const uint32_t ms = s_ev[3 * i], a = s_ev[3 * i + 1], b = s_ev[3 * i + 2];
                        const uint32_t n = b & 0x3FFFu, r1 = (b >> 14) & 0x3FFFu;
                        if (!(b >> 31)) {  // private & !upload: the entity itself (n is 0 or 1)
                            if (sub < n) out[ms] = a;
                            continue;
                        }
                        for (uint32_t p = sub; p < n; p += L) {  // every player of the group but self
                            const uint32_t pp = p + ((r1 && p + 1 >= r1) ? 1u : 0u);
                            out[ms + p] = staged ? s_pl[a - pb_lo + pp] : (uint32_t)d.pl_slot[a + pp];
                        }
                    }
                } else {
                    const unsigned last = 3u * (c1 - c0 - 1u);
                    const unsigned m_lo = s_ev[0], m_hi = s_ev[last] + (s_ev[last + 2] & 0x3FFFu);
                    for (unsigned w0 = m_lo; w0 < m_hi; w0 += W) {  // uniform
                        const unsigned w1 = min(m_hi, w0 + W);
                        // short runs: one thread per event (fewer LDS reads than lane groups)
                        for (uint32_t i = threadIdx.x; i < c1 - c0; i += kTPB) {
                            const uint32_t ms = s_ev[3 * i], a = s_ev[3 * i + 1], b = s_ev[3 * i + 2];
                            const uint32_t n = b & 0x3FFFu, r1 = (b >> 14) & 0x3FFFu;
                            if (n == 0 || ms >= w1 || ms + n <= w0) continue;
                            if (!(b >> 31)) {
                                s_win[ms - w0] = a;
                                continue;
                            }
                            const uint32_t np = n + (r1 ? 1u : 0u);
                            uint32_t k = ms;
                            for (uint32_t p = 0; p < np; p++) {
                                if (p + 1 == r1) continue;
                                if (k >= w0 && k < w1)
                                    s_win[k - w0] = staged ? s_pl[a - pb_lo + p] : (uint32_t)d.pl_slot[a + p];
                                k++;
                            }
                        }
                        __syncthreads();
                        const uint32_t n = w1 - w0;
                        if ((w0 & 3u) == 0) {  // mb is a multiple of 4 (msg_tcap is): 16-byte stores
                            const uint32_t n4 = n >> 2;
                            uint4* dst4 = (uint4*)(out + w0);
                            const uint4* src4 = (const uint4*)s_win;
                            for (uint32_t i = threadIdx.x; i < n4; i += kTPB) st_nt<(S::kNt & kNtFanStore) != 0>(dst4 + i, src4[i]);
                            if (threadIdx.x < (n & 3u)) out[w0 + 4 * n4 + threadIdx.x] = s_win[4 * n4 + threadIdx.x];
                        } else {
                            for (uint32_t i = threadIdx.x; i < n; i += kTPB) out[w0 + i] = s_win[i];
                        }
                        __syncthreads();
                    }
                }
                if (c1 < tev) __syncthreads();  // s_ev is refilled
            }
        }
    }
    // tile counts and algorithmic-byte tally
    const unsigned wb = (unsigned)wave_sum(bytes);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_bytes, wb);
    if (S::kLb && threadIdx.x == 0) s_lb_last = lb_last;
    __syncthreads();
    const bool lb_scan = S::kLb && d.lb_rank && s_lb_last;
    if (threadIdx.x == 0) {
        d.t_ev[tile] = (unsigned)((tot >> 32) & 0xFFFF);
        d.t_fi[tile] = (unsigned)(tot >> 48);
        d.t_msg[tile] = (unsigned)tot;
        tally_add(d, kTallyTick, (unsigned long long)(s_bytes + 12 + (fuse ? 16 : 0)));
    }
    if constexpr (S::kLb)
        if (lb_scan) lb_scan_all(d, s_w);
}

template <int kWPE, int kU, class S = DynSchema>
__global__ __launch_bounds__(kTPB) __attribute__((amdgpu_waves_per_eu(kWPE, 8))) void k_tick(Dev d) {
    __shared__ unsigned long long s_w[kTPB / 64];
    __shared__ unsigned s_bytes;
    __shared__ uint32_t s_lb_last;  // this tile ranks the frame's tiles (Dev::lb_rank)
    __shared__ uint32_t s_pb[3];   // pl_slot run of the groups with dirty events [lo, hi), most recipients
    extern __shared__ __align__(16) uint64_t s_o[];  // [n_w][kTPB] frame-start values of the writable slots
    const int tile = d.xcd_map ? xcd_tile((int)blockIdx.x, d.n_tiles) : (int)blockIdx.x;
    tick_tile<kU, S>(d, tile, s_w, s_bytes, s_lb_last, s_pb, s_o);
}


// ---------------------------------------------------------------------------------
// The per-Set log of the watched properties (nfk_watch_props; see k_chain in nfgpu_kernels.hip) on
// the frame's register working set, under the world's schema policy: the fire test without its
// stores, the operand loads and the fired kinds' programs exactly as k_tick runs them (its hipRTC
// specialisation's straight-line programs, or the library's tables), on the values k_sets left,
// before k_tick.  The programs run twice on register copies — count the watched Sets, then write
// them at their places from a block scan — so the log is tile-staged in (slot, kind, op) order with
// no atomics: tile t's entries at t * tcap, t_cnt[t] of them.
struct ChainEnt {
    uint32_t slot;
    uint16_t pid;
    uint8_t kind, op;
    uint64_t old_bits, new_bits;
};
static_assert(sizeof(ChainEnt) == 24, "ChainEnt is read back as 24-byte records");

template <int kU, class S>
__global__ __launch_bounds__(kTPB) void k_chain_u(Dev d, ChainEnt* __restrict__ out, uint32_t* __restrict__ t_cnt,
                                                  uint32_t tcap, uint32_t kinds, uint64_t watch0, uint64_t watch1) {
    __shared__ unsigned long long s_w[kTPB / 64];
    const int e = blockIdx.x * kTPB + (int)threadIdx.x;
    uint32_t fired = 0;
    uint64_t v[kU];
#pragma unroll
    for (int j = 0; j < kU; j++) v[j] = 0;
    if (e < d.N) {
        unsigned bytes = 0;
        uint64_t desc = kDeadDesc;
        fired = sched_scan<S, false>(d, e, bytes, desc) & kinds;
        if (desc_dead(desc)) fired = 0;
    }
    if (fired) {
        const uint32_t need = S::need(d, fired);
#pragma unroll
        for (int j = 0; j < kU; j++)
            if ((need >> j) & 1) v[j] = *elem<S>(d.u_col[j], (uint32_t)e, S::u_str(d, j));
    }
    const auto watched = [&](uint32_t u) {
        const uint32_t p = (uint32_t)S::u_pid(d, (int)u);
        return ((p < 64 ? watch0 >> p : watch1 >> (p - 64)) & 1ull) != 0;
    };
    uint32_t cnt = 0;
    if (fired) {
        uint64_t c[kU];
#pragma unroll
        for (int j = 0; j < kU; j++) c[j] = v[j];
        uint32_t wm = 0;
        S::run(c, wm, d, fired, [&](int, int, uint32_t u, uint64_t, uint64_t) { cnt += watched(u) ? 1u : 0u; });
    }
    unsigned long long tot;
    uint32_t at = (uint32_t)block_excl_scan(cnt, s_w, tot);
    if (cnt) {
        ChainEnt* t_out = out + (size_t)blockIdx.x * tcap;
        uint32_t wm = 0;
        S::run(v, wm, d, fired, [&](int k, int i, uint32_t u, uint64_t o, uint64_t n) {
            if (watched(u) && at < tcap)
                t_out[at++] = ChainEnt{(uint32_t)e, (uint16_t)S::u_pid(d, (int)u), (uint8_t)k, (uint8_t)i, o, n};
        });
    }
    if (threadIdx.x == 0) t_cnt[blockIdx.x] = (uint32_t)tot;
}

}  // namespace nfgpu
