// nfgpu_kernels.hip — hand-written gfx950 kernels for one NoahGameFrame server frame.
//
//   k_ext_scatter   index queued SetProperty* calls by slot
//   k_pre_hostops   RemoveSchedule(self[, name]) effects that precede the scan
//   k_tick          heartbeat timer scan (NFCScheduleModule::Execute, SM:45-80) + effect
//                   programs + property change predicates (NFCProperty::SetInt/SetFloat,
//                   PR:254/295) + dirty diff + ordered compaction of dirty events and fired
//                   heartbeats (wave ballot/scan + decoupled look-back)
//   k_records       record-cell effects (NFCRecord::SetInt/SetFloat, RC:182/243) + diff,
//                   one wave per entity, lane = row
//   k_post_hostops  remove list then add list (SM:82-117)
//   k_fanout        GetBroadCastObject recipient lists (AOI:531-593) for every dirty event,
//                   CSR over the (scene, group, guid)-sorted slots, LDS-staged so message
//                   stores are coalesced
//
// Compiled with -ffp-contract=off: f64 effects round exactly like the reference's C++.
#include "nfgpu_device.hpp"

namespace nfgpu {

// ---------------------------------------------------------------------------------
__global__ void k_ext_scatter(const uint32_t* __restrict__ x_slot, int32_t n, uint32_t* __restrict__ ext_head) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0 || x_slot[i] != x_slot[i - 1]) ext_head[x_slot[i]] = (uint32_t)i + 1;
}

// op: 1 = RemoveSchedule(self, name) queued (owns the remove-list key), 2 = RemoveSchedule(self)
__global__ void k_pre_hostops(const uint32_t* __restrict__ slot, const uint32_t* __restrict__ op, int32_t n,
                              uint8_t* __restrict__ e_flags, SchedHot* __restrict__ s_hot, int32_t n_kind,
                              int32_t cap) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot[i];
    if (op[i] == 1) e_flags[s] |= 1;
    if (op[i] == 2)
        for (int k = 0; k < n_kind; k++) s_hot[(size_t)k * cap + s].state = 0;
}

// post-scan host ops, one entry per (slot, kind): bit0 remove, bit1 add (remove first), bit2 clear key
__global__ void k_post_hostops(const uint32_t* __restrict__ slot, const uint32_t* __restrict__ kind,
                               const uint32_t* __restrict__ op, const float* __restrict__ interval,
                               const int32_t* __restrict__ count, const int64_t* __restrict__ time, int32_t n,
                               Dev d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot[i];
    const size_t at = (size_t)kind[i] * d.cap + s;
    SchedHot h = d.s_hot[at];
    if (op[i] & 1) h.state = 0;
    if (op[i] & 4) d.e_flags[s] = 0;
    if ((op[i] & 2) && !(h.state & 1)) {  // AddSchedule (SM:236): an existing name wins
        const float f = interval[i];
        const int32_t c = count[i];
        h.state = 1u | (c < 0 ? 2u : 0u);
        h.next = time[i] + (int64_t)(f * 1000.0f);
        h.remain = c;
        SchedCold cold;
        cold.start = time[i];
        cold.all = c;
        cold.interval = f;
        d.s_cold[at] = cold;
    }
    d.s_hot[at] = h;
}

// ---------------------------------------------------------------------------------
// Per-entity written-property list: ids and current values in registers (all indices
// compile-time), frame-start values in LDS (written once per property, read at the diff).
struct Ent {
    uint32_t pid[NFK_MAX_TOUCH];
    uint64_t cur[NFK_MAX_TOUCH];
    uint64_t* old;  // LDS, [NFK_MAX_TOUCH][kTPB] with this thread's column
    int n;
    bool ovf;
    unsigned bytes;
    const int64_t* icol;
    const double* fcol;
    size_t cap;
    int n_int;
    int e;

    __device__ __forceinline__ bool tget(uint32_t p, uint64_t& v) const {
        bool f = false;
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++) {
            const bool m = (j < n) && (pid[j] == p);
            v = m ? cur[j] : v;
            f |= m;
        }
        return f;
    }
    __device__ __forceinline__ void tput(uint32_t p, uint64_t oldv, uint64_t newv) {
        bool f = false;
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++) {
            const bool m = (j < n) && (pid[j] == p);
            if (m) cur[j] = newv;
            f |= m;
        }
        if (f) return;
        if (n >= NFK_MAX_TOUCH) {
            ovf = true;
            return;
        }
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++)
            if (j == n) {
                pid[j] = p;
                cur[j] = newv;
            }
        old[n * kTPB] = oldv;
        n++;
    }
    __device__ __forceinline__ uint64_t getb(uint32_t p) {
        uint64_t v = 0;
        if (tget(p, v)) return v;
        bytes += 8;
        if ((int)p < n_int) return (uint64_t)icol[(size_t)p * cap + e];
        return (uint64_t)__double_as_longlong(fcol[(size_t)(p - n_int) * cap + e]);
    }
    __device__ __forceinline__ int64_t geti(uint32_t p) { return (int64_t)getb(p); }
    __device__ __forceinline__ double getf(uint32_t p) { return __longlong_as_double((long long)getb(p)); }
    // NFCProperty::SetInt (PR:254): stored (and an event fired) only when the value changes
    __device__ __forceinline__ void seti(uint32_t p, int64_t v) {
        const int64_t c = geti(p);
        if (v == c) return;
        tput(p, (uint64_t)c, (uint64_t)v);
    }
    // NFCProperty::SetFloat (PR:295): IsZeroDouble(v - cur), eps 1e-15 (NFPlatform.h:362)
    __device__ __forceinline__ void setf(uint32_t p, double v) {
        const double c = getf(p);
        if (fabs(v - c) <= 1e-15) return;
        tput(p, (uint64_t)__double_as_longlong(c), (uint64_t)__double_as_longlong(v));
    }
};

// One heartbeat callback = the kind's program.  Pass 1 issues every operand load of the
// program at once (independent loads, one memory round trip); pass 2 runs the ops in order,
// reading a property from the frame's written-property list when an earlier op (or kind, or
// queued SetProperty) wrote it, else from the prefetched column value.
__device__ __forceinline__ void run_program(Ent& en, const Tables* __restrict__ tab, int k) {
    const int n = tab->nops[k];
    uint64_t pre[NFK_MAX_OPS][4];
#pragma unroll
    for (int i = 0; i < NFK_MAX_OPS; i++) {
        if (i >= n) break;
        const nfk_op op = tab->ops[k][i];
        if (op.code != NFK_OP_IADD_CLAMP && op.code != NFK_OP_FLERP && op.code != NFK_OP_FAFFINE) continue;
        const uint32_t p0 = op.dst;
        const bool isf = op.code != NFK_OP_IADD_CLAMP;
        pre[i][0] = isf ? (uint64_t)__double_as_longlong(en.fcol[(size_t)(p0 - en.n_int) * en.cap + en.e])
                        : (uint64_t)en.icol[(size_t)p0 * en.cap + en.e];
        en.bytes += 8;
        if (op.code == NFK_OP_FLERP) {
            pre[i][1] = (uint64_t)__double_as_longlong(en.fcol[(size_t)(op.a - en.n_int) * en.cap + en.e]);
            en.bytes += 8;
        } else if (op.code == NFK_OP_IADD_CLAMP) {
            if (op.flags & NFK_A_PROP) { pre[i][1] = (uint64_t)en.icol[(size_t)op.a * en.cap + en.e]; en.bytes += 8; }
            if (op.flags & NFK_LO_PROP) { pre[i][2] = (uint64_t)en.icol[(size_t)op.b * en.cap + en.e]; en.bytes += 8; }
            if (op.flags & NFK_HI_PROP) { pre[i][3] = (uint64_t)en.icol[(size_t)op.c * en.cap + en.e]; en.bytes += 8; }
        }
    }
#pragma unroll
    for (int i = 0; i < NFK_MAX_OPS; i++) {
        if (i >= n) break;
        const nfk_op op = tab->ops[k][i];
        if (op.code == NFK_OP_IADD_CLAMP) {
            uint64_t t;
            const int64_t cur = en.tget(op.dst, t) ? (int64_t)t : (int64_t)pre[i][0];
            const int64_t a = (op.flags & NFK_A_PROP) ? (en.tget((uint32_t)op.a, t) ? (int64_t)t : (int64_t)pre[i][1]) : op.a;
            const int64_t lo = (op.flags & NFK_LO_PROP) ? (en.tget((uint32_t)op.b, t) ? (int64_t)t : (int64_t)pre[i][2]) : op.b;
            const int64_t hi = (op.flags & NFK_HI_PROP) ? (en.tget((uint32_t)op.c, t) ? (int64_t)t : (int64_t)pre[i][3]) : op.c;
            int64_t v = (int64_t)((uint64_t)cur + (uint64_t)a);
            v = v < lo ? lo : v;
            v = v > hi ? hi : v;
            if (v != cur) en.tput(op.dst, (uint64_t)cur, (uint64_t)v);  // NFCProperty::SetInt (PR:273)
        } else if (op.code == NFK_OP_FLERP || op.code == NFK_OP_FAFFINE) {
            uint64_t t;
            const double x = __longlong_as_double((long long)(en.tget(op.dst, t) ? t : pre[i][0]));
            double v;
            if (op.code == NFK_OP_FLERP) {
                const double tg = __longlong_as_double((long long)(en.tget((uint32_t)op.a, t) ? t : pre[i][1]));
                const double dd = tg - x;
                const double m = dd * __longlong_as_double(op.b);
                v = x + m;
            } else {
                const double m = x * __longlong_as_double(op.a);
                v = m + __longlong_as_double(op.b);
            }
            if (!(fabs(v - x) <= 1e-15))  // NFCProperty::SetFloat (PR:314): IsZeroDouble(v - cur)
                en.tput(op.dst, (uint64_t)__double_as_longlong(x), (uint64_t)__double_as_longlong(v));
        }
        // record ops run in k_records
    }
}

// Block-wide exclusive scan of a packed pair of 32-bit counts (sums stay < 2^32 per block).
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

constexpr int kKindChunk = 8;  // schedule hot records loaded together per chunk

__global__ __launch_bounds__(kTPB) void k_tick(Dev d) {
    __shared__ unsigned s_vb;
    __shared__ unsigned long long s_w[kTPB / 64];
    __shared__ unsigned long long s_base[2];
    __shared__ unsigned s_bytes;
    __shared__ uint64_t s_old[NFK_MAX_TOUCH * kTPB];
    if (threadIdx.x == 0) {
        s_vb = atomicAdd(&d.ctrl->ticket_tick, 1u);
        s_bytes = 0;
        if (blockIdx.x == 0) {  // last frame's k_records / k_fanout are complete
            d.ctrl->ticket_rec = 0;
            d.ctrl->ticket_fan = 0;
        }
    }
    __syncthreads();
    const unsigned vb = s_vb;
    const int e = (int)(vb * kTPB + threadIdx.x);
    const bool live = e < d.N;
    Ent en;
    en.n = 0;
    en.old = s_old + threadIdx.x;
    en.ovf = false;
    en.bytes = 0;
    en.icol = d.icol;
    en.fcol = d.fcol;
    en.cap = (size_t)d.cap;
    en.n_int = d.n_int;
    en.e = live ? e : 0;
    uint32_t fired = 0;
    uint32_t xh = 0;
    if (live) {
        // 1. SetProperty* calls queued before this frame, in call order
        xh = d.ext_head[e];
        en.bytes += 4;
        if (xh) {
            for (int i = (int)xh - 1; i < d.n_x && d.x_slot[i] == (uint32_t)e; i++) {
                const uint32_t pid = d.x_pid[i];
                const uint64_t b = d.x_bits[i];
                en.bytes += 16;
                if ((int)pid < d.n_int) en.seti(pid, (int64_t)b);
                else en.setf(pid, __longlong_as_double((long long)b));
            }
        }
        // 2. NFCScheduleModule::Execute (SM:45-80): this object's schedules in name order.
        //    The hot records of a chunk of kinds are loaded together (independent 16 B loads).
        bool taken = d.e_flags[e] & 1;  // std::map remove-list key already owned (SM:72)
        en.bytes += 1;
        for (int k0 = 0; k0 < d.n_kind; k0 += kKindChunk) {
            SchedHot h[kKindChunk];
#pragma unroll
            for (int j = 0; j < kKindChunk; j++)
                if (k0 + j < d.n_kind) h[j] = d.s_hot[(size_t)(k0 + j) * d.cap + e];
#pragma unroll
            for (int j = 0; j < kKindChunk; j++) {
                const int k = k0 + j;
                if (k >= d.n_kind) break;
                en.bytes += 16;
                if (!(h[j].state & 1) || !(d.now > h[j].next)) continue;
                const bool forever = h[j].state & 2;
                if (!(h[j].remain > 0 || forever)) continue;
                h[j].remain -= 1;
                fired |= 1u << k;
                if (h[j].remain <= 0 && !forever) {
                    if (!taken) {  // insert into the remove list succeeds for the first one only
                        h[j].state = 0;
                        taken = true;
                    }
                } else {
                    const SchedCold c = d.s_cold[(size_t)k * d.cap + e];
                    en.bytes += 16;
                    const int64_t step = (int64_t)(c.interval * 1000.0f);
                    const int32_t done = (int32_t)((uint32_t)c.all - (uint32_t)h[j].remain);
                    h[j].next = c.start + step * (int64_t)done;
                }
                d.s_hot[(size_t)k * d.cap + e] = h[j];
                en.bytes += 16;
            }
        }
        // 3. the fired heartbeats' effect programs, in schedule-name order
        if (!(d.ablate & kAblPrograms)) {
            for (int k = 0; k < d.n_kind; k++)
                if ((fired >> k) & 1) run_program(en, d.tab, k);
        }
    }
    // 4. dirty diff: written properties whose bits changed since the frame began
    uint32_t dmask = 0;
#pragma unroll
    for (int j = 0; j < NFK_MAX_TOUCH; j++)
        if (j < en.n && en.cur[j] != en.old[j * kTPB]) dmask |= 1u << j;
    const unsigned nd = __builtin_popcount(dmask);
    const unsigned nf = __builtin_popcount(fired);
    if (en.ovf) atomicOr(&d.ctrl->err, kErrTouch);

    // 5. ordered compaction: block scan + look-back (events chain on wave 0, fired chain on wave 1)
    unsigned long long tot;
    const unsigned long long excl = block_excl_scan(((unsigned long long)nf << 32) | nd, s_w, tot);
    const int w = threadIdx.x >> 6;
    if (d.ablate & kAblTickLookback) {
        if (threadIdx.x == 0) {
            s_base[0] = (unsigned long long)vb * kTPB * NFK_MAX_TOUCH;
            s_base[1] = (unsigned long long)vb * kTPB * d.n_kind;
        }
    } else if (w == 0) {
        const unsigned long long b = lookback(d.g_ev, vb, d.tag, tot & 0xFFFFFFFFull, d.ctrl);
        if ((threadIdx.x & 63) == 0) s_base[0] = b;
    } else if (w == 1) {
        const unsigned long long b = lookback(d.g_fi, vb, d.tag, tot >> 32, d.ctrl);
        if ((threadIdx.x & 63) == 0) s_base[1] = b;
    }
    __syncthreads();
    unsigned long long pev = s_base[0] + (excl & 0xFFFFFFFFull);
    unsigned long long pfi = s_base[1] + (excl >> 32);

    if (live) {
        // write back changed columns
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++) {
            if (!((dmask >> j) & 1)) continue;
            const uint32_t pid = en.pid[j];
            if ((int)pid < d.n_int) d.icol[(size_t)pid * d.cap + e] = (int64_t)en.cur[j];
            else d.fcol[(size_t)(pid - d.n_int) * d.cap + e] = __longlong_as_double((long long)en.cur[j]);
            en.bytes += 8;
        }
        // events in property-id order
        uint32_t left = dmask;
        for (unsigned q = 0; q < nd; q++) {
            uint32_t best = 0xFFFFFFFFu;
            int bj = 0;
#pragma unroll
            for (int j = 0; j < NFK_MAX_TOUCH; j++)
                if (((left >> j) & 1) && en.pid[j] < best) {
                    best = en.pid[j];
                    bj = j;
                }
            uint64_t nv = 0;
#pragma unroll
            for (int j = 0; j < NFK_MAX_TOUCH; j++)
                if (j == bj) nv = en.cur[j];
            const uint64_t ov = en.old[bj * kTPB];
            left &= ~(1u << bj);
            if ((long long)pev < d.ev_cap) {
                d.ev_slot[pev] = (uint32_t)e;
                d.ev_pid[pev] = best;
                d.ev_old[pev] = ov;
                d.ev_new[pev] = nv;
            } else {
                atomicOr(&d.ctrl->err, kErrEvCap);
            }
            pev++;
            en.bytes += 24;
        }
        uint32_t fl = fired;
        while (fl) {
            const int k = __builtin_ctz(fl);
            fl &= fl - 1;
            if ((long long)pfi < d.fi_cap) {
                d.fi_slot[pfi] = (uint32_t)e;
                d.fi_kind[pfi] = (uint32_t)k;
                d.fi_remain[pfi] = d.s_hot[(size_t)k * d.cap + e].remain;
            } else {
                atomicOr(&d.ctrl->err, kErrFiCap);
            }
            pfi++;
            en.bytes += 16;
        }
        if (d.has_recops) {
            d.fired_mask[e] = fired;
            en.bytes += 4;
        }
        if (xh) d.ext_head[e] = 0;
    }
    // totals (last virtual block) and algorithmic-byte tally
    const unsigned wb = (unsigned)wave_sum(en.bytes);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_bytes, wb);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&d.ctrl->bytes_tick, (unsigned long long)s_bytes);
        if (vb == gridDim.x - 1) {
            d.ctrl->n_ev = s_base[0] + (tot & 0xFFFFFFFFull);
            d.ctrl->n_fi = s_base[1] + (tot >> 32);
        }
    }
}

// ---------------------------------------------------------------------------------
// Record effects: one wave per entity, lane = row.  Cells [cap][cols][rows] so the
// wave reads one (entity, col) row-vector contiguously.
__global__ __launch_bounds__(kTPB) void k_records(Dev d) {
    __shared__ unsigned s_vb;
    __shared__ unsigned long long s_w[kTPB / 64];
    __shared__ unsigned long long s_base;
    __shared__ unsigned s_bytes;
    if (threadIdx.x == 0) {
        s_vb = atomicAdd(&d.ctrl->ticket_rec, 1u);
        s_bytes = 0;
    }
    __syncthreads();
    const unsigned vb = s_vb;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = (int)(vb * (kTPB / 64) + w);
    const Tables* tab = d.tab;
    const int nro = tab->n_recops;
    unsigned bytes = 0;
    uint32_t mask = 0;
    if (e < d.N) {
        mask = d.fired_mask[e];
        if (lane == 0) bytes += 4;
    }
    mask &= tab->kind_has_recop;
    // apply (at most NFK_MAX_OPS record ops, distinct (rec, col), sorted by (rec, col))
    bool ch[NFK_MAX_OPS];
    uint64_t ov[NFK_MAX_OPS], nv[NFK_MAX_OPS];
#pragma unroll
    for (int j = 0; j < NFK_MAX_OPS; j++) {
        ch[j] = false;
        ov[j] = nv[j] = 0;
        if (j >= nro || !mask) continue;
        const RecOp ro = tab->recops[j];
        if (!((mask >> ro.kind) & 1)) continue;
        const int rows = tab->rec_rows[ro.rec], cols = tab->rec_cols[ro.rec];
        const uint64_t used = d.rused[ro.rec][e];
        if (lane == 0) bytes += 8;
        if (lane >= rows || !((used >> lane) & 1)) continue;
        uint64_t* cp = d.rcells[ro.rec] + ((size_t)e * cols + ro.col) * rows + lane;
        const uint64_t cur = *cp;
        bytes += 8;
        uint64_t nb;
        bool changed;
        if (ro.code == NFK_OP_RIADD_CLAMP) {
            int64_t v = (int64_t)(cur + (uint64_t)ro.a);
            v = v < ro.b ? ro.b : v;
            v = v > ro.c ? ro.c : v;
            nb = (uint64_t)v;
            changed = v != (int64_t)cur;  // TData::operator== (NFIDataList.h:98)
        } else {
            const double x = __longlong_as_double((long long)cur);
            const double m = x * __longlong_as_double(ro.a);
            const double v = m + __longlong_as_double(ro.b);
            const double df = v - x;
            changed = !(df < 0.001 && df > -0.001);  // NFIDataList.h:106-113
            nb = (uint64_t)__double_as_longlong(v);
        }
        if (changed) {
            *cp = nb;
            bytes += 8;
            ch[j] = nb != cur;  // coalesced diff: bits must differ
            ov[j] = cur;
            nv[j] = nb;
        }
    }
    // per-entity event order: (rec, row, col) -> records outer, lanes (rows), cols inner
    unsigned cnt = 0;
#pragma unroll
    for (int j = 0; j < NFK_MAX_OPS; j++) cnt += ch[j] ? 1 : 0;
    const unsigned long long wtot = wave_sum(cnt);
    if (lane == 0) s_w[w] = wtot;
    __syncthreads();
    unsigned long long before = 0, btot = 0;
#pragma unroll
    for (int i = 0; i < kTPB / 64; i++) {
        before += (i < w) ? s_w[i] : 0ull;
        btot += s_w[i];
    }
    if (w == 0) {
        const unsigned long long b = lookback(d.g_re, vb, d.tag, btot, d.ctrl);
        if (lane == 0) s_base = b;
    }
    __syncthreads();
    unsigned long long pos = s_base + before;
    int j0 = 0;
    while (j0 < nro) {
        const int rec = tab->recops[j0].rec;
        int j1 = j0;
        while (j1 < nro && tab->recops[j1].rec == rec) j1++;
        unsigned c = 0;
#pragma unroll
        for (int j = 0; j < NFK_MAX_OPS; j++) c += (j >= j0 && j < j1 && ch[j]) ? 1 : 0;
        const unsigned long long inc = wave_incl_scan(c);
        unsigned long long p = pos + inc - c;
#pragma unroll
        for (int j = 0; j < NFK_MAX_OPS; j++) {
            if (!(j >= j0 && j < j1 && ch[j])) continue;
            if ((long long)p < d.re_cap) {
                d.re_slot[p] = (uint32_t)e;
                d.re_rrc[p] = ((uint32_t)rec << 16) | ((uint32_t)lane << 8) | (uint32_t)tab->recops[j].col;
                d.re_old[p] = ov[j];
                d.re_new[p] = nv[j];
            } else {
                atomicOr(&d.ctrl->err, kErrReCap);
            }
            p++;
            bytes += 24;
        }
        pos += __shfl(inc, 63, 64);
        j0 = j1;
    }
    const unsigned wb = (unsigned)wave_sum(bytes);
    if (lane == 0) atomicAdd(&s_bytes, wb);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&d.ctrl->bytes_rec, (unsigned long long)s_bytes);
        if (vb == gridDim.x - 1) d.ctrl->n_re = s_base + btot;
    }
}

// ---------------------------------------------------------------------------------
// Fan-out over the virtual event stream [prop events ++ record events].  Persistent grid,
// 256-event tiles pulled from a ticket; message offsets by look-back; the tile's recipient
// lists are expanded cooperatively from an LDS descriptor table so consecutive lanes store
// consecutive messages.
__global__ __launch_bounds__(kTPB) void k_fanout(Dev d) {
    __shared__ unsigned s_tile;
    __shared__ unsigned long long s_w[kTPB / 64];
    __shared__ unsigned long long s_base;
    __shared__ uint32_t s_off[kTPB];
    __shared__ int32_t s_src[kTPB];   // public: first player index in pl_slot; private: -1 - slot
    __shared__ int32_t s_rank[kTPB];  // public: rank of self in the player list to skip, else -1
    __shared__ uint8_t s_pflags[NFK_MAX_CLASSES][NFK_MAX_INT_PROPS + NFK_MAX_FLT_PROPS];
    __shared__ uint8_t s_rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0) d.ctrl->ticket_tick = 0;  // this frame's k_tick is complete
    for (int i = threadIdx.x; i < (int)sizeof(s_pflags) / 4; i += kTPB)
        ((uint32_t*)s_pflags)[i] = ((const uint32_t*)d.tab->pflags)[i];
    for (int i = threadIdx.x; i < (int)sizeof(s_rflags) / 4; i += kTPB)
        ((uint32_t*)s_rflags)[i] = ((const uint32_t*)d.tab->rflags)[i];
    const unsigned long long nev = d.ctrl->n_ev < (unsigned long long)d.ev_cap ? d.ctrl->n_ev : d.ev_cap;
    const unsigned long long nre = d.ctrl->n_re < (unsigned long long)d.re_cap ? d.ctrl->n_re : d.re_cap;
    const unsigned long long total = nev + nre;
    const unsigned long long ntiles = (total + kTPB - 1) / kTPB;
    unsigned bytes = 0;
    while (true) {
        if (threadIdx.x == 0) s_tile = atomicAdd(&d.ctrl->ticket_fan, 1u);
        __syncthreads();
        const unsigned tile = s_tile;
        if (tile >= ntiles) break;
        const unsigned long long i = (unsigned long long)tile * kTPB + threadIdx.x;
        unsigned cnt = 0;
        int32_t src = 0, rank = -1;
        if (i < total) {
            int32_t slot;
            uint32_t key;  // property id or record id
            const bool isprop = i < nev;
            if (isprop) {
                slot = (int32_t)d.ev_slot[i];
                key = d.ev_pid[i];
            } else {
                slot = (int32_t)d.re_slot[i - nev];
                key = d.re_rrc[i - nev] >> 16;
            }
            const uint64_t desc = d.fan_desc[slot];
            bytes += 4 + 4 + 8;
            const unsigned cls = (unsigned)(desc >> 60);
            const uint8_t fl = isprop ? s_pflags[cls][key] : s_rflags[cls][key];
            if (fl & NFK_PUBLIC) {  // every player of the group but self, NFGUID order
                src = (int32_t)(uint32_t)desc;
                const int np = (int)((desc >> 32) & 0x3FFF);
                rank = (int)((desc >> 46) & 0x3FFF) - 1;
                cnt = (unsigned)(np - (rank >= 0 ? 1 : 0));
            } else if ((fl & NFK_PRIVATE) && !(fl & NFK_UPLOAD)) {  // self only
                cnt = 1;
                src = -1 - slot;
            }
        }
        unsigned long long tot;
        const unsigned long long excl = block_excl_scan(cnt, s_w, tot);
        if (d.ablate & kAblFanLookback) {
            if (threadIdx.x == 0) s_base = (unsigned long long)tile * kTPB * 8;
        } else if (w == 0) {
            const unsigned long long b = lookback(d.g_msg, tile, d.tag, tot, d.ctrl);
            if (lane == 0) s_base = b;
        }
        s_off[threadIdx.x] = (uint32_t)excl;
        s_src[threadIdx.x] = src;
        s_rank[threadIdx.x] = rank;
        __syncthreads();
        const unsigned long long base = s_base;
        if (i < total) {
            d.msg_off[i] = (uint32_t)(base + excl);
            bytes += 4;
        }
        if (base + tot > (unsigned long long)d.msg_cap) {
            if (threadIdx.x == 0) atomicOr(&d.ctrl->err, kErrMsgCap);
        } else {
            for (unsigned q = threadIdx.x; q < (unsigned)tot; q += kTPB) {
                // owner: the last event whose local offset <= q (it has cnt > 0)
                int lo = 0, hi = kTPB - 1;
#pragma unroll
                for (int step = 0; step < 8; step++) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_off[mid] <= q) lo = mid;
                    else hi = mid - 1;
                }
                const int32_t sr = s_src[lo];
                const uint32_t idx = q - s_off[lo];
                int32_t r;
                if (sr < 0) {
                    r = -1 - sr;
                } else {
                    const int32_t rk = s_rank[lo];
                    r = d.pl_slot[sr + idx + ((rk >= 0 && (int32_t)idx >= rk) ? 1 : 0)];
                }
                d.msg_rcpt[base + q] = (uint32_t)r;
            }
            bytes += 8 * (unsigned)tot / kTPB + ((threadIdx.x < (tot % kTPB)) ? 8 : 0);
        }
        if (tile == ntiles - 1 && threadIdx.x == 0) {
            d.ctrl->n_msgs = base + tot;
            d.msg_off[total] = (uint32_t)(base + tot);
        }
        __syncthreads();
    }
    const unsigned wb = (unsigned)wave_sum(bytes);
    if (lane == 0 && wb) atomicAdd(&d.ctrl->bytes_fan, (unsigned long long)wb);
    if (ntiles == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        d.ctrl->n_msgs = 0;
        d.msg_off[0] = 0;
    }
}

}  // namespace nfgpu
