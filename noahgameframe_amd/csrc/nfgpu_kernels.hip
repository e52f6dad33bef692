// nfgpu_kernels.hip — hand-written gfx950 kernels for one NoahGameFrame server frame.
//
//   k_xkeys / k_scan_heads / k_xgroups   queued SetProperty* calls folded into (slot, property)
//                   groups (with a device radix sort between k_xkeys and k_scan_heads)
//   k_pre_hostops   RemoveSchedule(self[, name]) effects that precede the scan
//   k_tick          heartbeat timer scan (NFCScheduleModule::Execute, SM:49-81) + effect
//                   programs + property change predicates (NFCProperty::SetInt/SetFloat,
//                   PR:254/295) + dirty diff; dirty events and fired heartbeats are compacted
//                   per 256-slot tile (wave ballot/scan + block scan, no inter-block chain) and
//                   each event's fan-out message count is scanned in the same pass
//   k_records       record-cell effects (NFCRecord::SetInt/SetFloat, RC:182/243) + diff,
//                   one wave per 64-slot record tile, lane = row
//   k_post_hostops  remove list then add list (SM:83-119)
//   k_scan_tiles    exclusive scans of the per-tile counts (events, fired, record events,
//                   messages) -> tile bases and frame totals
//   k_fanout        GetBroadCastObject recipient lists (AOI:531-593) for every dirty event:
//                   one workgroup per tile, LDS owner search so message stores are coalesced
//   k_compact_*     readback only: tile-staged outputs -> dense arrays
//
// Compiled with -ffp-contract=off: f64 effects round exactly like the reference's C++.
#include "nfgpu_device.hpp"

namespace nfgpu {

// ---------------------------------------------------------------------------------
// The window's SetProperty* calls folded into (slot, property) groups on the device.  The host
// hands the calls over as they were queued (object index, property, value bits, in call order);
// each resolves to its slot after the window's membership changes, a stable radix sort by
// (slot, property) keeps call order inside a group, and the groups are laid out as k_sets and
// k_tick read them (Dev::x_*).  Group entries past the frame's groups hold kNoGroupSlot, so Dev::n_x
// may be the call count (an upper bound the host knows without a read-back).
constexpr uint32_t kNoGroupSlot = 0xFFFFFFFFu;
struct XCall {  // (World::XOp's layout)
    uint32_t obj, pid;
    uint64_t bits;
};

// ---------------------------------------------------------------------------------
// NFGUID -> object index lookups of a large call batch (NFCKernelModule's GetElement(self) of every
// SetProperty* / schedule call, KM:323), on the device mirror of the host's open-addressing table
// (include/nfgpu_guidmap.hpp GuidMap: same entries, same hash, linear probing, no tombstones).
struct GuidEntry {  // (GuidMap::E's layout)
    int64_t h, d;
    int32_t v;
};
__device__ __forceinline__ uint64_t guid_home(int64_t h, int64_t d, uint64_t mask) {  // GuidMap::home
    uint64_t x = (uint64_t)h * 0x9E3779B97F4A7C15ull ^ (uint64_t)d;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x & mask;
}
// q = [n] heads then [n] data halves; out[i] = the object index, -1 when absent
__global__ void k_guid_find(const GuidEntry* __restrict__ t, uint64_t mask, const int64_t* __restrict__ q, int32_t n,
                            int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t h = q[i], dd = q[(size_t)n + i];
    int32_t r = -1;
    for (uint64_t s = guid_home(h, dd, mask);; s = (s + 1) & mask) {  // (the table is at most half full)
        const GuidEntry e = t[s];
        if (e.v < 0) break;
        if (e.h == h && e.d == dd) {
            r = e.v;
            break;
        }
    }
    out[i] = r;
}
// the entries the host table's inserts / erases wrote since the last batch, at their indices
__global__ void k_guid_patch(GuidEntry* __restrict__ t, const uint32_t* __restrict__ idx,
                             const GuidEntry* __restrict__ e, int32_t n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) t[idx[i]] = e[i];
}

// A batch of SetProperty* calls queued on the device (nfgpu_host.hip set_props_dev): each call's
// object looked up, the call written at its place in the window's device queue q; miss = the first
// call whose NFGUID is no object (the batch is then not queued: "There is no object", KM:331).
// b = [n] heads, [n] data halves, [n] values; pid = [n] property ids (checked on the host)
__global__ void k_guid_queue(const GuidEntry* __restrict__ t, uint64_t mask, const int64_t* __restrict__ b,
                             const int32_t* __restrict__ pid, int32_t n, XCall* __restrict__ q,
                             int32_t* __restrict__ miss) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t h = b[i], dd = b[(size_t)n + i];
    int32_t r = -1;
    for (uint64_t s = guid_home(h, dd, mask);; s = (s + 1) & mask) {
        const GuidEntry e = t[s];
        if (e.v < 0) break;
        if (e.h == h && e.d == dd) {
            r = e.v;
            break;
        }
    }
    if (r < 0) {
        atomicMin(miss, i);
        return;
    }
    q[i] = XCall{(uint32_t)r, (uint32_t)pid[i], (uint64_t)b[2 * (size_t)n + i]};
}

// obj_slot[o] = the slot object o holds (entries start at -1); slack slots are skipped
__global__ void k_obj_slots(const int32_t* __restrict__ slot_obj, const uint64_t* __restrict__ fan_desc, int32_t n,
                            int32_t* __restrict__ obj_slot) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int32_t o = slot_obj[s];
    if (o >= 0 && !desc_dead(fan_desc[s])) obj_slot[o] = s;
}

// key of call i: slot << 7 | property, ~0 when the object holds no slot ("There is no object":
// destroyed or exported in this window); the group entries start empty
__global__ void k_xkeys(const XCall* __restrict__ x, int32_t n, const int32_t* __restrict__ obj_slot,
                        uint64_t* __restrict__ keys, uint32_t* __restrict__ idx, uint32_t* __restrict__ x_slot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const XCall c = x[i];
    const int32_t sl = obj_slot[c.obj];
    keys[i] = sl < 0 ? ~0ull : (((uint64_t)(uint32_t)sl << 7) | c.pid);
    idx[i] = (uint32_t)i;
    x_slot[i] = kNoGroupSlot;
}

// gidx[i] = groups that start before sorted call i (a group starts where the key changes),
// gidx[n] = the frame's groups; one workgroup (a window's calls: tens of thousands)
__global__ __launch_bounds__(1024) void k_scan_heads(const uint64_t* __restrict__ keys, int n, uint32_t* __restrict__ gidx) {
    __shared__ uint32_t s[1024];
    const int per = (n + 1023) / 1024, i0 = min(n, (int)threadIdx.x * per), i1 = min(n, i0 + per);
    auto head = [&](int i) -> uint32_t { return keys[i] != ~0ull && (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u; };
    uint32_t sum = 0;
    for (int i = i0; i < i1; i++) sum += head(i);
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t acc = s[threadIdx.x] - sum;
    for (int i = i0; i < i1; i++) {
        gidx[i] = acc;
        acc += head(i);
    }
    if (threadIdx.x == 1023) gidx[n] = s[1023];
}

// the groups (slot, property, first call), each slot's first group in ext_head, and the calls'
// values in sorted order
__global__ void k_xgroups(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                          const uint32_t* __restrict__ gidx, const XCall* __restrict__ x,
                          const uint64_t* __restrict__ x_h, int32_t n, uint32_t* __restrict__ x_slot,
                          uint32_t* __restrict__ x_pid, uint32_t* __restrict__ x_first, uint64_t* __restrict__ x_bits,
                          uint64_t* __restrict__ x_bits_h, uint32_t* __restrict__ ext_head, uint8_t* __restrict__ tile_work) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    if (k == ~0ull) return;
    const uint32_t j = idx[i];
    x_bits[i] = x[j].bits;
    if (x_bits_h) x_bits_h[i] = x_h[j];
    const uint64_t kp = i ? keys[i - 1] : ~0ull;
    const uint32_t sl = (uint32_t)(k >> 7);
    if (k != kp) {
        const uint32_t g = gidx[i];
        x_slot[g] = sl;
        x_pid[g] = (uint32_t)(k & 127);
        x_first[g] = (uint32_t)i;
        if (i == 0 || (uint32_t)(kp >> 7) != sl) {
            ext_head[sl] = g + 1;
            if (tile_work) tile_work[sl / kTile] = 1;
        }
    }
    if (i + 1 == n || keys[i + 1] == ~0ull) x_first[gidx[n]] = (uint32_t)i + 1;  // the last group's end
}

// The SetProperty* calls queued before this frame (NFCKernelModule::SetPropertyInt/Float,
// KM:323-347), one thread per (slot, property) group, in call order through the reference's
// change predicates: NFCProperty::SetInt stores only a different value (PR:254-293), SetFloat
// only when !IsZeroDouble(v - cur) with eps 1e-15 (PR:295-334, NFPlatform.h:362).  Calls on
// different properties never interact and every call precedes the frame's heartbeat scan, so the
// groups are independent.  The column gets the value after the group; x_old / x_new keep the
// frame-start value and that value for the frame's diff.
__global__ __launch_bounds__(kTPB) void k_sets(Dev d) {
    const int g = blockIdx.x * kTPB + threadIdx.x;
    if (g >= d.n_x || d.x_slot[g] == kNoGroupSlot) return;
    const uint32_t pid = d.x_pid[g];
    uint64_t* p = prop_ptr(d, pid, (int)d.x_slot[g]);
    const uint64_t start = *p;
    uint64_t cur = start;
    const uint32_t i1 = d.x_first[g + 1];
    if ((int)pid >= d.n_if) {
        // NFCProperty::SetObject (PR:377-416): the NFGUID changes when either half differs; the
        // column holds (data, head) side by side
        const uint64_t start_h = p[1];
        uint64_t cur_h = start_h;
        for (uint32_t i = d.x_first[g]; i < i1; i++) {
            const uint64_t b = d.x_bits[i], bh = d.x_bits_h[i];
            cur = b;
            cur_h = bh;
        }
        if (cur != start || cur_h != start_h) {
            p[0] = cur;
            p[1] = cur_h;
        }
        d.x_old[g] = start;
        d.x_new[g] = cur;
        d.x_old_h[g] = start_h;
        d.x_new_h[g] = cur_h;
        return;
    }
    const bool isint = (int)pid < d.n_int;
    for (uint32_t i = d.x_first[g]; i < i1; i++) {
        const uint64_t b = d.x_bits[i];
        const bool set = isint ? b != cur
                               : !(fabs(__longlong_as_double((long long)b) - __longlong_as_double((long long)cur)) <= 1e-15);
        cur = set ? b : cur;
    }
    if (cur != start) *p = cur;
    d.x_old[g] = start;
    d.x_new[g] = cur;
}


// ---------------------------------------------------------------------------------
// The window's schedule calls (AddSchedule / RemoveSchedule(self, name) / RemoveSchedule(self),
// SM:218-251) folded on the device into the pre-scan entries (k_pre_hostops) and the post-scan
// (slot, kind) entries (k_post_hostops), as NFCScheduleModule::Execute applies them:
//  * RemoveSchedule(self) erases the object's schedules at once (SM:240-243);
//  * RemoveSchedule(self, name) inserts into the std::map<NFGUID, name> remove list, so only the
//    object's first one in the window owns the key (SM:245-249), and it also blocks the scan's own
//    insert (SM:68);
//  * remove runs before add at the end of Execute (SM:83-119); AddSchedule keeps an existing name,
//    so of several adds of one (object, name) the first wins (SM:108-116).
// Keys slot << 5 | kind (kind 0 for RemoveSchedule(self) and a name without a device program), a
// stable radix sort (call order within a key), then one thread per slot walks its calls.
constexpr uint32_t kHNoKind = 0xFFFFFFFFu;  // a RemoveSchedule(self, name) of a name with no device program
struct HCall {  // (World::HOp's layout)
    int32_t code;
    uint32_t obj, kind;
    float interval;
    int32_t count;
    int64_t time;
};
// the schedule calls' post-scan entries (k_post_hostops): one array per field
struct HPost {
    uint32_t *slot, *kind, *op;
    float* interval;
    int32_t* count;
    int64_t* time;
};
__global__ void k_hkeys(const HCall* __restrict__ h, int32_t n, const int32_t* __restrict__ obj_slot,
                        uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const HCall c = h[i];
    const int32_t sl = obj_slot[c.obj];
    keys[i] = sl < 0 ? ~0ull : (((uint64_t)(uint32_t)sl << 5) | (c.code == 3 || c.kind == kHNoKind ? 0u : c.kind));
    idx[i] = (uint32_t)i;
}
// the slot whose calls start at sorted position i (else none): its pre and post entries counted
// (kEmit = false, into npre / npost at i) or written at the scanned positions opre[i] / opost[i]
template <bool kEmit>
__global__ void k_hfold(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                        const HCall* __restrict__ h, int32_t n, uint32_t* __restrict__ npre,
                        uint32_t* __restrict__ npost, const uint32_t* __restrict__ opre,
                        const uint32_t* __restrict__ opost, uint32_t* __restrict__ pre_slot,
                        uint32_t* __restrict__ pre_op, HPost post) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (!kEmit && a == n) {  // (the counts' last entry: the scans' totals land at [n])
        npre[n] = npost[n] = 0;
        return;
    }
    if (a >= n) return;
    const uint64_t ka = keys[a];
    const uint32_t slot = (uint32_t)(ka >> 5);
    if (ka == ~0ull || (a > 0 && (uint32_t)(keys[a - 1] >> 5) == slot && keys[a - 1] != ~0ull)) {
        if (!kEmit) npre[a] = npost[a] = 0;
        return;
    }
    int b = a;
    uint32_t owner_seq = 0xFFFFFFFFu, owner_kind = 0;
    bool erase_all = false;
    for (; b < n && keys[b] != ~0ull && (uint32_t)(keys[b] >> 5) == slot; b++) {
        const uint32_t seq = idx[b];
        const HCall& c = h[seq];
        if (c.code == 3) erase_all = true;
        if (c.code == 2 && seq < owner_seq) {
            owner_seq = seq;
            owner_kind = c.kind;
        }
    }
    uint32_t np = 0, nq = 0;
    const uint32_t p0 = kEmit ? opre[a] : 0u, q0 = kEmit ? opost[a] : 0u;
    auto put_pre = [&](uint32_t op) {
        if (kEmit) {
            pre_slot[p0 + np] = slot;
            pre_op[p0 + np] = op;
        }
        np++;
    };
    auto put_post = [&](uint32_t kind, uint32_t op, float iv, int32_t cnt, int64_t t) {
        if (kEmit) {
            post.slot[q0 + nq] = slot;
            post.kind[q0 + nq] = kind;
            post.op[q0 + nq] = op;
            post.interval[q0 + nq] = iv;
            post.count[q0 + nq] = cnt;
            post.time[q0 + nq] = t;
        }
        nq++;
    };
    if (erase_all) put_pre(2);
    if (owner_seq != 0xFFFFFFFFu) {
        put_pre(1);
        if (owner_kind == kHNoKind) put_post(0, 8, 0.f, 0, 0);  // release the key only
    }
    for (int c = a; c < b;) {
        const uint32_t kind = (uint32_t)(keys[c] & 31);
        uint32_t op = (owner_seq != 0xFFFFFFFFu && owner_kind == kind) ? 1u | 4u : 0u;
        float iv = 0.f;
        int32_t cnt = 0;
        int64_t t = 0;
        int e = c;
        for (; e < b && (uint32_t)(keys[e] & 31) == kind; e++) {
            const HCall& x = h[idx[e]];
            if (x.code == 1 && !(op & 2u)) {
                op |= 2u;
                iv = x.interval;
                cnt = x.count;
                t = x.time;
            }
        }
        if (op) put_post(kind, op, iv, cnt, t);
        c = e;
    }
    if (!kEmit) {
        npre[a] = np;
        npost[a] = nq;
    }
}

// op: 1 = RemoveSchedule(self, name) queued (owns the remove-list key), 2 = RemoveSchedule(self);
// n_dev: the entry count on the device (the device fold's), else n
__global__ void k_pre_hostops(const uint32_t* __restrict__ slot, const uint32_t* __restrict__ op, int32_t n,
                              uint8_t* __restrict__ e_flags, SchedHot* __restrict__ s_hot, int32_t n_kind,
                              int32_t kstr, const uint32_t* __restrict__ n_dev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (n_dev && (uint32_t)i >= *n_dev)) return;
    const uint32_t s = slot[i];
    if (op[i] == 1) e_flags[s] |= 1;
    if (op[i] == 2)
        for (int k = 0; k < n_kind; k++) s_hot[(size_t)k * kstr + s].state = 0;
}

// post-scan host ops, one entry per (slot, kind): bit0 remove, bit1 add (remove first), bit2 clear
// key, bit3 clear key only (a kind-less remove-list owner); added[i] = the add created the schedule
__global__ void k_post_hostops(const uint32_t* __restrict__ slot, const uint32_t* __restrict__ kind,
                               const uint32_t* __restrict__ op, const float* __restrict__ interval,
                               const int32_t* __restrict__ count, const int64_t* __restrict__ time, int32_t n,
                               uint8_t* __restrict__ added, Dev d, const uint32_t* __restrict__ n_dev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (n_dev && (uint32_t)i >= *n_dev)) return;
    const uint32_t s = slot[i];
    if (op[i] & 8) {
        d.e_flags[s] = 0;
        added[i] = 0;
        return;
    }
    const size_t at = (size_t)kind[i] * d.s_kstr + s;
    SchedHot h = d.s_hot[at];
    if (op[i] & 1) h.state = 0;
    if (op[i] & 4) d.e_flags[s] = 0;
    added[i] = (op[i] & 2) && !(h.state & 1);
    if ((op[i] & 2) && !(h.state & 1)) {  // AddSchedule (SM:218): an existing name wins
        const float f = interval[i];
        const int32_t c = count[i];
        const int64_t step = (int64_t)(f * 1000.0f);
        h.state = kStPresent | (c < 0 ? kStForever : 0u) | st_pack_step(step);
        h.next = time[i] + step;
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
    const Dev* dv;
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
        return *prop_ptr(*dv, p, e);
    }
    __device__ __forceinline__ int64_t geti(uint32_t p) { return (int64_t)getb(p); }
    __device__ __forceinline__ double getf(uint32_t p) { return __longlong_as_double((long long)getb(p)); }
    // a program destination whose queued Set group (k_sets) already ran: frame-start value and
    // the value the programs start from
    __device__ __forceinline__ void tinit(uint32_t p, uint64_t oldv, uint64_t curv) {
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++)
            if (j == n) {
                pid[j] = p;
                cur[j] = curv;
            }
        if (n < NFK_MAX_TOUCH) old[n * kTPB] = oldv;
        else ovf = true;
        n++;
    }
};

// One heartbeat callback = the kind's program.  Pass 1 issues every operand load of the
// program at once (independent loads, one memory round trip); pass 2 runs the ops in order,
// reading a property from the frame's written-property list when an earlier op (or kind, or
// queued SetProperty) wrote it, else from the prefetched column value.
// Log: called with (kind, op, property, old, new) for every Set the predicates accept (k_chain's
// per-Set log; k_tick_touch passes the empty one, which compiles away).
struct NoChainLog {
    __device__ __forceinline__ void operator()(int, int, uint32_t, uint64_t, uint64_t) const {}
};
template <class Log = NoChainLog>
__device__ __forceinline__ void run_program_chunk(Ent& en, const Tables* __restrict__ tab, int k, int i0, int n,
                                                  const Log& log = Log()) {
    uint64_t pre[4][6];  // dst, a, b, c, guard, the property the guard compares to (NFK_GUARD_PROP)
#pragma unroll
    for (int ii = 0; ii < 4; ii++) {
        const int i = i0 + ii;
        if (i >= n) break;
        const nfk_op op = tab->ops[k][i];
        if (op.code != NFK_OP_IADD_CLAMP && op.code != NFK_OP_FLERP && op.code != NFK_OP_FAFFINE &&
            op.code != NFK_OP_ISET && op.code != NFK_OP_FSET)
            continue;
        const uint32_t p0 = op.dst;
        const bool isf = op.code != NFK_OP_IADD_CLAMP;
        (void)isf;
        pre[ii][0] = *prop_ptr(*en.dv, p0, en.e);
        en.bytes += 8;
        if (op.flags & NFK_GUARD) {
            pre[ii][4] = *prop_ptr(*en.dv, op.guard & 0xFFFFu, en.e);
            en.bytes += 8;
            if (op.guard & NFK_GUARD_PROP) {
                pre[ii][5] = *prop_ptr(*en.dv, op.guard >> 19, en.e);
                en.bytes += 8;
            }
        }
        if (op.code == NFK_OP_FLERP || ((op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) && (op.flags & NFK_A_PROP))) {
            pre[ii][1] = *prop_ptr(*en.dv, (uint32_t)op.a, en.e);
            en.bytes += 8;
        } else if (op.code == NFK_OP_IADD_CLAMP) {
            if (op.flags & NFK_A_PROP) { pre[ii][1] = *prop_ptr(*en.dv, (uint32_t)op.a, en.e); en.bytes += 8; }
            if (op.flags & NFK_LO_PROP) { pre[ii][2] = *prop_ptr(*en.dv, (uint32_t)op.b, en.e); en.bytes += 8; }
            if (op.flags & NFK_HI_PROP) { pre[ii][3] = *prop_ptr(*en.dv, (uint32_t)op.c, en.e); en.bytes += 8; }
        }
    }
#pragma unroll
    for (int ii = 0; ii < 4; ii++) {
        const int i = i0 + ii;
        if (i >= n) break;
        const nfk_op op = tab->ops[k][i];
        if (op.flags & NFK_GUARD) {
            uint64_t t;
            const int64_t g = en.tget(op.guard & 0xFFFFu, t) ? (int64_t)t : (int64_t)pre[ii][4];
            const int64_t h = !(op.guard & NFK_GUARD_PROP) ? (int64_t)NFK_GUARD_KVAL(op.guard) : en.tget(op.guard >> 19, t) ? (int64_t)t : (int64_t)pre[ii][5];
            if (!guard_ok((op.guard >> 16) & 3u, g, h)) continue;
        }
        if (op.code == NFK_OP_IADD_CLAMP) {
            uint64_t t;
            const int64_t cur = en.tget(op.dst, t) ? (int64_t)t : (int64_t)pre[ii][0];
            const int64_t a = (op.flags & NFK_A_PROP) ? (en.tget((uint32_t)op.a, t) ? (int64_t)t : (int64_t)pre[ii][1]) : op.a;
            const int64_t lo = (op.flags & NFK_LO_PROP) ? (en.tget((uint32_t)op.b, t) ? (int64_t)t : (int64_t)pre[ii][2]) : op.b;
            const int64_t hi = (op.flags & NFK_HI_PROP) ? (en.tget((uint32_t)op.c, t) ? (int64_t)t : (int64_t)pre[ii][3]) : op.c;
            int64_t v = (int64_t)((uint64_t)cur + (uint64_t)a);
            v = v < lo ? lo : v;
            v = v > hi ? hi : v;
            if (v != cur) {  // NFCProperty::SetInt (PR:273)
                en.tput(op.dst, (uint64_t)cur, (uint64_t)v);
                log(k, i, op.dst, (uint64_t)cur, (uint64_t)v);
            }
        } else if (op.code == NFK_OP_FLERP || op.code == NFK_OP_FAFFINE) {
            uint64_t t;
            const double x = __longlong_as_double((long long)(en.tget(op.dst, t) ? t : pre[ii][0]));
            double v;
            if (op.code == NFK_OP_FLERP) {
                const double tg = __longlong_as_double((long long)(en.tget((uint32_t)op.a, t) ? t : pre[ii][1]));
                const double dd = tg - x;
                const double m = dd * __longlong_as_double(op.b);
                v = x + m;
            } else {
                const double m = x * __longlong_as_double(op.a);
                v = m + __longlong_as_double(op.b);
            }
            if (!(fabs(v - x) <= 1e-15)) {  // NFCProperty::SetFloat (PR:314): IsZeroDouble(v - cur)
                en.tput(op.dst, (uint64_t)__double_as_longlong(x), (uint64_t)__double_as_longlong(v));
                log(k, i, op.dst, (uint64_t)__double_as_longlong(x), (uint64_t)__double_as_longlong(v));
            }
        } else if (op.code == NFK_OP_ISET || op.code == NFK_OP_FSET) {
            uint64_t t;
            const uint64_t cur = en.tget(op.dst, t) ? t : pre[ii][0];
            const uint64_t r = (op.flags & NFK_A_PROP) ? (en.tget((uint32_t)op.a, t) ? t : pre[ii][1]) : (uint64_t)op.a;
            const bool set = op.code == NFK_OP_ISET
                                 ? r != cur  // NFCProperty::SetInt (PR:273)
                                 : !(fabs(__longlong_as_double((long long)r) - __longlong_as_double((long long)cur)) <= 1e-15);
            if (set) {
                en.tput(op.dst, cur, r);
                log(k, i, op.dst, cur, r);
            }
        }
        // record ops run in k_records
    }
}

template <class Log = NoChainLog>
__device__ __forceinline__ void run_program(Ent& en, const Tables* __restrict__ tab, int k, const Log& log = Log()) {
    const int n = tab->nops[k];
    // (ops in chunks of 4: an operand an earlier op wrote is read from the written list either way)
#pragma unroll 1
    for (int i0 = 0; i0 < n; i0 += 4)
        run_program_chunk(en, tab, k, i0, min(n, i0 + 4), log);
}

}  // namespace nfgpu

#include "nfgpu_tick.hpp"
namespace nfgpu {

// k_tick_touch: the general path, used when the programs' working set does not fit the U slots
// (see k_tick): a per-entity written-property list, one operand round trip per fired kind.  The
// list holds program destinations only (at most NFK_MAX_TOUCH, checked at commit); queued Sets
// of other properties are standalone events merged at emission.
__global__ __launch_bounds__(kTPB) void k_tick_touch(Dev d) {
    __shared__ unsigned long long s_w[kTPB / 64];
    __shared__ unsigned s_bytes;
    __shared__ uint64_t s_old[NFK_MAX_TOUCH * kTPB];
    __shared__ uint8_t s_pflags[NFK_MAX_CLASSES][kMaxProps];
    const int tile = blockIdx.x;
    const int e = tile * kTile + (int)threadIdx.x;
    uint64_t desc = kDeadDesc;
    unsigned dbytes = 0;
    if (e < d.N) {
        desc = d.fan_desc[e];
        dbytes = 8;
    }
    const bool live = !desc_dead(desc);
    if (threadIdx.x == 0) s_bytes = 0;
    {
        const int words = d.n_class * kMaxProps / 4;
        for (int i = threadIdx.x; i < words; i += kTPB)
            ((uint32_t*)s_pflags)[i] = ((const uint32_t*)d.tab->pflags)[i];
    }
    Ent en;
    en.n = 0;
    en.old = s_old + threadIdx.x;
    en.ovf = false;
    en.bytes = 0;
    en.dv = &d;
    en.cap = (size_t)d.cap;
    en.n_int = d.n_int;
    en.e = live ? e : 0;
    en.bytes = dbytes;
    uint32_t fired = 0;
    uint32_t xh = 0;
    int n_set = 0;
    if (live) {
        // 1. SetProperty* calls queued before this frame: k_sets applied them; a program
        //    destination enters the written-property list with its frame-start value
        if (d.n_x) {
            xh = d.ext_head[e];
            en.bytes += 4;
            if (xh)
                for (int g = (int)xh - 1; g < d.n_x && d.x_slot[g] == (uint32_t)e; g++) {
                    en.bytes += 8;
                    if (d.tab->w_slot[d.x_pid[g]] == kNoU) continue;  // standalone: merged at emission
                    en.tinit(d.x_pid[g], d.x_old[g], d.x_new[g]);
                    en.bytes += 16;
                }
            n_set = en.n;
        }
        // 2. NFCScheduleModule::Execute (SM:51-81)
        fired = sched_scan(d, e, en.bytes, desc);
        // 3. the fired heartbeats' effect programs, in schedule-name order
        if (!(d.ablate & kAblPrograms) && fired) {
            for (int k = 0; k < d.n_kind; k++)
                if ((fired >> k) & 1) run_program(en, d.tab, k);
        }
    }
    __syncthreads();  // s_pflags
    // 4. dirty diff: written properties whose bits changed since the frame began, and the
    //    fan-out message count of each dirty event
    uint32_t dmask = 0;
    unsigned nmsg = 0;
    const unsigned cls = (unsigned)(desc >> 60);
#pragma unroll
    for (int j = 0; j < NFK_MAX_TOUCH; j++)
        if (j < en.n && en.cur[j] != en.old[j * kTPB]) {
            dmask |= 1u << j;
            nmsg += event_msgs(desc, s_pflags[cls][en.pid[j]]);
        }
    // standalone Set events (properties no program writes)
    unsigned nd = __builtin_popcount(dmask);
    if (xh)
        for (int g = next_standalone(d, (int)xh - 1, e); g < d.n_x; g = next_standalone(d, g + 1, e)) {
            nd++;
            nmsg += event_msgs(desc, s_pflags[cls][d.x_pid[g]]);
            en.bytes += 8;
        }
    const unsigned nf = __builtin_popcount(fired);
    if (en.ovf) dev_error(d, kErrTouch);

    // 5. tile-local compaction: one block scan of (fired:16 | events:16 | messages:32)
    unsigned long long tot;
    const unsigned long long excl =
        block_excl_scan(((unsigned long long)nf << 48) | ((unsigned long long)nd << 32) | nmsg, s_w, tot);
    unsigned pev = (unsigned)((excl >> 32) & 0xFFFF);
    unsigned pfi = (unsigned)(excl >> 48);
    unsigned pmsg = (unsigned)excl;
    const size_t ev0 = (size_t)tile * d.ev_tcap, fi0 = (size_t)tile * d.fi_tcap;

    if (live) {
        // write back changed columns, and every Set program destination (k_sets changed its
        // column; the list's first n_set entries)
#pragma unroll
        for (int j = 0; j < NFK_MAX_TOUCH; j++) {
            if (!((dmask >> j) & 1) && j >= n_set) continue;
            const uint32_t pid = en.pid[j];
            *prop_ptr(d, pid, e) = en.cur[j];
            en.bytes += 8;
        }
        // events in property-id order: the written-property list merged with the standalone groups
        uint32_t left = dmask;
        int g = xh ? next_standalone(d, (int)xh - 1, e) : d.n_x;
        for (unsigned q = 0; q < nd; q++) {
            uint32_t best = 0xFFFFFFFFu;
            int bj = 0;
#pragma unroll
            for (int j = 0; j < NFK_MAX_TOUCH; j++)
                if (((left >> j) & 1) && en.pid[j] < best) {
                    best = en.pid[j];
                    bj = j;
                }
            uint64_t nv = 0, ov;
            if (g < d.n_x && d.x_pid[g] < best) {
                best = d.x_pid[g];
                ov = d.x_old[g];
                nv = d.x_new[g];
                if ((int)best >= d.n_if) {  // an object property: its head halves beside
                    d.ev_old_h[ev0 + pev] = d.x_old_h[g];
                    d.ev_new_h[ev0 + pev] = d.x_new_h[g];
                    en.bytes += 16;
                }
                g = next_standalone(d, g + 1, e);
            } else {
#pragma unroll
                for (int j = 0; j < NFK_MAX_TOUCH; j++)
                    if (j == bj) nv = en.cur[j];
                ov = en.old[bj * kTPB];
                left &= ~(1u << bj);
            }
            const size_t at = ev0 + pev;
            d.ev_slot[at] = (uint32_t)e;
            d.ev_pid[at] = best;
            d.ev_old[at] = ov;
            d.ev_new[at] = nv;
            d.ev_moff[at] = pmsg;  // tile-local; k_fanout adds the tile's message base
            pmsg += event_msgs(desc, s_pflags[cls][best]);
            pev++;
            en.bytes += 28;
        }
        uint32_t fl = fired;
        while (fl) {
            const int k = __builtin_ctz(fl);
            fl &= fl - 1;
            const size_t at = fi0 + pfi;
            d.fi_slot[at] = (uint32_t)e;
            d.fi_kind[at] = (uint32_t)k;
            d.fi_remain[at] = d.s_hot[(size_t)k * d.s_kstr + e].remain;
            pfi++;
            en.bytes += 12;
        }
        if (xh) d.ext_head[e] = 0;
    }
    if (d.has_recops && e < d.N) {  // slack slots too: a slot's previous occupant left a mask
        d.fired_mask[e] = fired;
        en.bytes += 4;
    }
    // tile counts and algorithmic-byte tally
    const unsigned wb = (unsigned)wave_sum(en.bytes);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_bytes, wb);
    __syncthreads();
    if (threadIdx.x == 0) {
        d.t_ev[tile] = (unsigned)((tot >> 32) & 0xFFFF);
        d.t_fi[tile] = (unsigned)(tot >> 48);
        d.t_msg[tile] = (unsigned)tot;
        tally_add(d, kTallyTick, (unsigned long long)(s_bytes + 12));
    }
}

// ---------------------------------------------------------------------------------
// Per-Set chains of watched properties (nfk_watch_props).  The frame's events are coalesced per
// (entity, property); the reference fires a property's per-object callbacks once per accepted Set
// (NFCProperty::SetInt / SetFloat, PR:254-334), in the order NFCScheduleModule::Execute runs the
// functors (SM:52-80).  For the watched properties k_chain re-runs the frame's fire test and
// heartbeat programs READ-ONLY, before k_tick, on the values k_sets left — k_tick_touch's own code
// (sched_scan without its stores, run_program) — and logs every accepted Set of a watched property
// as (slot, kind, op, property, old, new).  Off (not launched) while nothing is watched.
// The log is tile-staged like the frame's other outputs: tile t's entries at t * tcap (tcap = the
// tile's slots x the (kind, op) pairs whose destination is watched), in (slot, kind, op) order — a
// thread's own in program order, the threads' placed by a block scan of their counts (the programs
// run twice: count, then write) — and t_cnt[t] of them; no atomics, so the log is deterministic.
// nfk_read_chain compacts it and sorts it into the walk's (NFGUID, kind, op) order on the device.
// (ChainEnt: nfgpu_tick.hpp)
__global__ __launch_bounds__(kTPB) void k_chain(Dev d, ChainEnt* __restrict__ out, uint32_t* __restrict__ t_cnt,
                                                uint32_t tcap, uint32_t kinds, uint64_t watch0, uint64_t watch1) {
    __shared__ uint64_t s_old[NFK_MAX_TOUCH * kTPB];  // (Ent's frame-start list; unused here)
    __shared__ unsigned long long s_w[kTPB / 64];
    const int e = blockIdx.x * kTPB + (int)threadIdx.x;
    uint32_t fired = 0;
    if (e < d.N) {
        unsigned bytes = 0;
        uint64_t desc = kDeadDesc;
        fired = sched_scan<DynSchema, false>(d, e, bytes, desc) & kinds;
        if (desc_dead(desc)) fired = 0;
    }
    Ent en;
    auto run = [&](auto&& log) {
        en.n = 0;
        en.old = s_old + threadIdx.x;
        en.ovf = false;
        en.bytes = 0;
        en.dv = &d;
        en.cap = (size_t)d.cap;
        en.n_int = d.n_int;
        en.e = e;
        for (int k = 0; k < d.n_kind; k++)
            if ((fired >> k) & 1) run_program(en, d.tab, k, log);
    };
    auto watched = [&](uint32_t p) { return ((p < 64 ? watch0 >> p : watch1 >> (p - 64)) & 1ull) != 0; };
    uint32_t cnt = 0;
    bool ovf = false;
    if (fired) {
        run([&](int, int, uint32_t p, uint64_t, uint64_t) { cnt += watched(p) ? 1u : 0u; });
        ovf = en.ovf;  // (a program touching more than NFK_MAX_TOUCH properties: k_tick raises it too)
    }
    unsigned long long tot;
    uint32_t at = (uint32_t)block_excl_scan(cnt, s_w, tot);
    if (cnt) {
        ChainEnt* t_out = out + (size_t)blockIdx.x * tcap;
        run([&](int k, int i, uint32_t p, uint64_t o, uint64_t n) {
            if (watched(p) && at < tcap) t_out[at++] = ChainEnt{(uint32_t)e, (uint16_t)p, (uint8_t)k, (uint8_t)i, o, n};
        });
    }
    if (threadIdx.x == 0) t_cnt[blockIdx.x] = (uint32_t)tot;
    if (ovf) dev_error(d, kErrTouch);  // (the log of an overflowing entity is not the frame's)
}
// nfk_read_chain: the staged log -> sort keys (rank of the object's NFGUID, kind, op) and the staged
// index of each entry, in dense order (db: the tiles' exclusive scan)
__global__ __launch_bounds__(kTPB) void k_chain_keys(const ChainEnt* __restrict__ src, const uint32_t* __restrict__ db,
                                                     int n_tiles, uint32_t tcap, const int32_t* __restrict__ slot_obj,
                                                     const int32_t* __restrict__ rank, uint64_t* __restrict__ keys,
                                                     uint32_t* __restrict__ idx) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = db[t], n = db[t + 1] - b;
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) {
            const size_t s = (size_t)t * tcap + i;
            const ChainEnt c = src[s];
            keys[b + i] = ((uint64_t)(uint32_t)rank[slot_obj[c.slot]] << 8) | ((uint64_t)c.kind << 3) | (uint64_t)c.op;
            idx[b + i] = (uint32_t)s;
        }
    }
}
// the sorted log as object-index columns (obj, kind, op, pid as int32; old, new) for one copy back
__global__ __launch_bounds__(kTPB) void k_chain_gather(const ChainEnt* __restrict__ src, const uint32_t* __restrict__ idx,
                                                       int n, const int32_t* __restrict__ slot_obj,
                                                       int32_t* __restrict__ i32, uint64_t* __restrict__ u64) {
    const int j = blockIdx.x * kTPB + threadIdx.x;
    if (j >= n) return;
    const ChainEnt c = src[idx[j]];
    i32[j] = slot_obj[c.slot];
    i32[(size_t)n + j] = c.kind;
    i32[2 * (size_t)n + j] = c.op;
    i32[3 * (size_t)n + j] = c.pid;
    u64[j] = c.old_bits;
    u64[(size_t)n + j] = c.new_bits;
}

// ---------------------------------------------------------------------------------
// NFIKernelModule::SetRecordInt / SetRecordFloat (KM:505 / KM:545) between frames: one thread per
// (slot, cell) group applies the group's calls in call order through NFCRecord::SetInt / SetFloat
// (RC:182 / RC:243): refused on a row that is not used (RC:194); an int cell changes when the bits
// differ, an f64 cell unless |new - cur| < 0.001 (TData::operator==, NFIDataList.h:106-113).
__global__ void k_rs_scatter(const uint32_t* __restrict__ rss_slot, int32_t n, uint32_t* __restrict__ rs_head) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rs_head[rss_slot[i]] = (uint32_t)i + 1;  // 1 + the slot's index among the SetRecord slots
}

__global__ __launch_bounds__(kTPB) void k_rsets(Dev d) {
    const int g = blockIdx.x * kTPB + threadIdx.x;
    if (g >= d.n_rs) return;
    const uint32_t e = d.rs_slot[g], rrc = d.rs_rrc[g];
    d.rs_has[g] = 0;
    if (rrc >> 31) return;  // a row-operation list's cell: k_rrows applies its calls in call order
    const int r = (int)(rrc >> 16), row = (int)((rrc >> 8) & 0xFF), col = (int)(rrc & 0xFF);
    const int rows = d.tab->rec_rows[r], cols = d.tab->rec_cols[r];
    uint64_t* cells = nullptr;
    const uint64_t* usedp = nullptr;
#pragma unroll
    for (int q = 0; q < NFK_MAX_RECORDS; q++)
        if (q == r) {
            cells = d.rcells[q];
            usedp = d.rused[q];
        }
    const uint64_t used = usedp[e];
    uint64_t* cell = cells + ((size_t)e * cols + col) * rows + rec_pos(used, rec_rowm(rows), row);
    const uint64_t c0 = *cell;
    uint64_t v = c0;
    if ((used >> row) & 1) {
        const bool f64 = d.tab->rec_ctype[r][col] != 0;
        bool logged = false;
        for (uint32_t k = d.rs_first[g]; k < d.rs_first[g + 1]; k++) {
            const uint64_t x = d.rs_bits[k];
            if (f64) {
                const double df = __longlong_as_double((long long)x) - __longlong_as_double((long long)v);
                if (!(df < 0.001 && df > -0.001)) {
                    v = x;
                    logged = true;
                }
            } else if (x != v) {
                v = x;
                logged = true;
            }
        }
        if (v != c0) *cell = v;
        d.rs_has[g] = logged ? 1 : 0;
    }
    d.rs_old[g] = c0;
    d.rs_new[g] = v;
}

// Record row operations between frames, one thread per (slot, record) list, every call of the
// list in call order on the cells and the used-row mask:
//   SetRecordInt / Float (RC:182 / RC:243): as k_rsets, on the row's used state at that call;
//       the cell's group keeps the first logged old value and the last logged new one;
//   AddRow(row, values) (RC:111-180): row -1 takes the first unused row (none: nothing); a used
//       row is covered; the cells are written without Update events; one Add / Cover event;
//   Remove(row) (RC:1086-1107): a used row's Del event, then the row is unused (cells kept);
//   ClearRecord (KM:492 -> RC:1109): Remove from the last row to the first.
// one slot's record vectors [cols][rows] moved from the places of mask `from` to those of `to`
__device__ void rec_repack(uint64_t* cells, int rows, int cols, uint64_t rowm, uint64_t from, uint64_t to) {
    if (from == to) return;
    for (int c = 0; c < cols; c++) {
        uint64_t* v = cells + (size_t)c * rows;
        uint64_t t[64];
        for (int r = 0; r < rows; r++) t[r] = v[rec_pos(from, rowm, r)];
        for (int r = 0; r < rows; r++) v[rec_pos(to, rowm, r)] = t[r];
    }
}

__global__ __launch_bounds__(kTPB) void k_rrows(Dev d) {
    const int l = blockIdx.x * kTPB + threadIdx.x;
    if (l >= d.n_rl) return;
    const uint32_t e = d.rl_slot[l];
    const int r = (int)d.rl_rec[l];
    const int rows = d.tab->rec_rows[r], cols = d.tab->rec_cols[r];
    uint64_t* cells = nullptr;
    uint64_t* usedp = nullptr;
#pragma unroll
    for (int q = 0; q < NFK_MAX_RECORDS; q++)
        if (q == r) {
            cells = d.rcells[q];
            usedp = d.rused[q];
        }
    cells += (size_t)e * cols * rows;
    const uint64_t rowm = rec_rowm(rows);
    uint64_t used = usedp[e];
    // the calls run on the cells in row order (rec_pos with an empty mask) and the vectors are
    // packed again by the final mask (row operations are rare; one private vector per column)
    rec_repack(cells, rows, cols, rowm, used, 0ull);
    uint32_t* ev = d.rl_ev + d.rl_ev0[l];
    unsigned nev = 0;
    for (uint32_t k = d.rl_c0[l]; k < d.rl_c0[l + 1]; k++) {
        const uint32_t code = d.rc_code[k];
        const uint32_t op = code & 0xFF, row = (code >> 8) & 0xFF, col = (code >> 16) & 0xFF;
        if (op == 0) {
            if (!((used >> row) & 1)) continue;  // RC:194
            const uint32_t g = d.rc_aux[k];
            uint64_t* c = cells + (size_t)col * rows + row;
            const uint64_t cur = *c, x = d.rc_bits[k];
            bool changed;
            if (d.tab->rec_ctype[r][col]) {
                const double df = __longlong_as_double((long long)x) - __longlong_as_double((long long)cur);
                changed = !(df < 0.001 && df > -0.001);
            } else {
                changed = x != cur;
            }
            if (!changed) continue;
            if (!d.rs_has[g]) {
                d.rs_old[g] = cur;
                d.rs_has[g] = 1;
            }
            d.rs_new[g] = x;
            *c = x;
        } else if (op == 1) {
            int rr = (int)row;
            bool cover = false;
            if (row == 0xFF) {
                const uint64_t fr = ~used & rowm;
                if (!fr) continue;  // no unused row: AddRow returns -1
                rr = __builtin_ctzll(fr);
            } else {
                cover = (used >> rr) & 1;
            }
            used |= 1ull << rr;
            const uint32_t vi = d.rc_aux[k];
            for (int c = 0; c < cols; c++)
                cells[(size_t)c * rows + rr] = vi == 0xFFFFFFFFu ? 0ull : d.rvals[(size_t)vi * NFK_MAX_REC_COLS + c];
            ev[nev++] = ((cover ? 3u : 1u) << 8) | (uint32_t)rr;
        } else if (op == 2) {
            if (!((used >> row) & 1)) continue;
            ev[nev++] = (2u << 8) | row;
            used &= ~(1ull << row);
        } else {
            for (int q = rows - 1; q >= 0; q--)
                if ((used >> q) & 1) {
                    ev[nev++] = (2u << 8) | (uint32_t)q;
                    used &= ~(1ull << q);
                }
        }
    }
    rec_repack(cells, rows, cols, rowm, 0ull, used);
    usedp[e] = used;
    d.rl_cnt[l] = nev;
}

// The slots with SetRecord groups this window, one wave each (lane = row), every record of the
// slot, every column in order: a cell's event runs from its frame-start value (the group's rs_old,
// else the cell) to its value after the slot's fired record ops, which apply to the value the Sets
// left (RC:182 / RC:243); it is dropped when the bits are equal.  Events in (rec, row, col) order,
// as k_records' own.  kEmit = false: count the slot's events and messages (rss_ev, rss_msg) before
// k_records, which reserves their room in the slot's place in its tile (rss_pos, rss_pmsg); kEmit:
// write them there, with the cells' write-back and the fused fan-out, after it.
template <bool kEmit>
__global__ __launch_bounds__(kTPB) void k_rset_slots(Dev d) {
    __shared__ uint8_t s_rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    for (int i = threadIdx.x; i < (int)sizeof(s_rflags) / 4; i += kTPB)
        ((uint32_t*)s_rflags)[i] = ((const uint32_t*)d.tab->rflags)[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int si = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
    if (si >= d.n_rss) return;  // wave-uniform
    const int e = (int)d.rss_slot[si], g0 = (int)d.rss_g0[si];
    int g1 = g0;
    while (g1 < d.n_rs && d.rs_slot[g1] == (uint32_t)e) g1++;
    int li = d.n_rl ? (int)d.rss_l0[si] : 0;  // the slot's row-operation lists (by record)
    const uint32_t fmask = d.has_recops ? d.fired_mask[e] & d.rop_kinds : 0u;
    const uint64_t desc = d.fan_desc[e];
    const unsigned cls = (unsigned)(desc >> 60);
    const int nro = d.n_rops;
    const int rt = e / kRTile;
    const size_t re0 = (size_t)rt * d.re_tcap;
    const uint32_t sit = (uint32_t)(e - rt * kRTile) << kRrcSitShift;  // (the event word's slot field)
    const uint32_t mrb = d.fuse_rec ? d.msg_rb0 + (uint32_t)rt * d.msg_rtcap : 0u;
    unsigned pos = kEmit ? d.rss_pos[si] : 0u, pmsg = kEmit ? d.rss_pmsg[si] : 0u;
    unsigned bytes = 0;
    for (int r = 0; r < d.n_rec; r++) {
        const int rows = d.tab->rec_rows[r], cols = d.tab->rec_cols[r];
        if (rows <= 0) continue;
        // record r's arrays by a select over compile-time indices (a run-time index into the
        // kernel-argument arrays would put them in scratch)
        uint64_t* cells = nullptr;
        const uint64_t* usedp = nullptr;
#pragma unroll
        for (int q = 0; q < NFK_MAX_RECORDS; q++)
            if (q == r) {
                cells = d.rcells[q];
                usedp = d.rused[q];
            }
        const uint8_t rfl = s_rflags[cls][r];
        const unsigned per = event_msgs(desc, rfl);
        const uint64_t used = usedp[e];
        const bool act = lane < rows;
        const uint32_t lp = act ? rec_pos(used, rec_rowm(rows), lane) : 0u;  // this lane's row's place
        // GetBroadCastObject (AOI:531-593) of one record event into its run at lmo
        auto fan = [&](uint32_t lmo) {
            uint32_t* out = d.msg_rcpt + mrb + lmo;
            if (!(rfl & NFK_PUBLIC)) {
                out[0] = (uint32_t)e;  // private & !upload: the entity itself
                bytes += 4;
            } else {  // every player of the group but self
                const uint32_t np = (uint32_t)((desc >> 32) & 0x3FFF);
                const uint32_t r1 = (uint32_t)((desc >> 46) & 0x3FFF);
                uint32_t q = 0;
                for (uint32_t u = 0; u < np; u++) {
                    if (u + 1 == r1) continue;
                    out[q++] = (uint32_t)d.pl_slot[(uint32_t)desc + u];
                }
                bytes += 4 * (per + np);
            }
        };
        // the record's row events first (AddRow / Remove / Clear, in call order: k_rrows)
        if (li < d.n_rl && d.rl_slot[li] == (uint32_t)e && d.rl_rec[li] == (uint32_t)r) {
            const unsigned nrow = d.rl_cnt[li];
            if constexpr (kEmit) {
                const uint32_t* rev = d.rl_ev + d.rl_ev0[li];
                for (unsigned q = (unsigned)lane; q < nrow; q += 64) {
                    const uint32_t x = rev[q];
                    const unsigned at = pos + q;
                    const uint32_t lmo = pmsg + per * q;
                    d.re_rrc[re0 + at] = sit | ((x >> 8) << 24) | ((uint32_t)r << 16) | ((x & 0xFF) << 8);
                    d.re_old[re0 + at] = 0;
                    d.re_new[re0 + at] = 0;
                    if (!d.fuse_rec) d.re_moff[re0 + at] = lmo;  // (fused: the readers count, k_counted_moff)
                    bytes += d.fuse_rec ? 24 : 28;
                    if (d.fuse_rec && per) fan(lmo);
                }
            }
            pos += nrow;
            pmsg += per * nrow;
            li++;
        }
        // cell (r, lane, c): its event (old, new) if any, and whether a record op writes nb back
        auto eval = [&](int c, uint64_t& ob, uint64_t& nb, bool& wb) -> bool {
            bool op = false;
            int code = 0;
            int64_t oa = 0, obb = 0, oc = 0;
#pragma unroll
            for (int j = 0; j < NFK_MAX_REC_OPS; j++)
                if (j < nro && d.rops[j].rec == r && d.rops[j].col == c && ((fmask >> d.rops[j].kind) & 1)) {
                    op = true;
                    code = d.rops[j].code;
                    oa = d.rops[j].a;
                    obb = d.rops[j].b;
                    oc = d.rops[j].c;
                }
            int gi = -1;
            const uint32_t key = ((uint32_t)r << 16) | ((uint32_t)lane << 8) | (uint32_t)c;
            for (int g = g0; g < g1; g++)
                if ((d.rs_rrc[g] & 0x7FFFFFFFu) == key) gi = g;
            wb = false;
            if (!act || (!op && gi < 0)) return false;
            const bool has = gi >= 0 && d.rs_has[gi];
            const uint64_t cur = cells[((size_t)e * cols + c) * rows + lp];
            nb = cur;
            if (op && ((used >> lane) & 1)) {
                if (code == NFK_OP_RIADD_CLAMP) {
                    int64_t v = (int64_t)(cur + (uint64_t)oa);
                    v = v < obb ? obb : v;
                    v = v > oc ? oc : v;
                    if (v != (int64_t)cur) {  // TData::operator== (NFIDataList.h:98)
                        nb = (uint64_t)v;
                        wb = true;
                    }
                } else {
                    const double x = __longlong_as_double((long long)cur);
                    const double m = x * __longlong_as_double(oa);
                    const double v = m + __longlong_as_double(obb);
                    const double df = v - x;
                    if (!(df < 0.001 && df > -0.001)) {  // NFIDataList.h:106-113
                        nb = (uint64_t)__double_as_longlong(v);
                        wb = true;
                    }
                }
            }
            // coalesced (first logged old, last logged new): a cell AddRow rewrote after its Sets
            // keeps the Sets' last value as the event's new one unless a record op changed it
            ob = has ? d.rs_old[gi] : cur;
            if (!wb && has) nb = d.rs_new[gi];
            return ob != nb;
        };
        unsigned cnt = 0;
        for (int c = 0; c < cols; c++) {
            uint64_t ob, nb;
            bool wb;
            cnt += eval(c, ob, nb, wb) ? 1u : 0u;
        }
        const unsigned incl = wave_incl_scan_u32(cnt);
        const unsigned total = (unsigned)__builtin_amdgcn_readlane((int)incl, 63);
        if constexpr (kEmit) {
            unsigned k = incl - cnt;
            for (int c = 0; c < cols; c++) {
                uint64_t ob, nb;
                bool wb;
                const bool ev = eval(c, ob, nb, wb);
                if (wb) {
                    __builtin_nontemporal_store(nb, cells + ((size_t)e * cols + c) * rows + lp);
                    bytes += 8;
                }
                if (!ev) continue;
                const unsigned at = pos + k;
                const uint32_t lmo = pmsg + per * k;
                d.re_rrc[re0 + at] = sit | ((uint32_t)r << 16) | ((uint32_t)lane << 8) | (uint32_t)c;
                d.re_old[re0 + at] = ob;
                d.re_new[re0 + at] = nb;
                if (!d.fuse_rec) d.re_moff[re0 + at] = lmo;  // tile-local: k_fanout adds the base
                bytes += d.fuse_rec ? 20 : 24;
                if (d.fuse_rec && per) fan(lmo);  // GetBroadCastObject (AOI:531-593)
                k++;
            }
            if (act) bytes += 8u * (unsigned)cols;  // the row's cells read
        }
        pos += total;
        pmsg += per * total;
    }
    if constexpr (kEmit) {
        const unsigned wb = (unsigned)wave_sum(bytes);
        if (lane == 0 && wb) tally_add(d, kTallyRec, (unsigned long long)wb + 16u * (unsigned)(g1 - g0));
    } else if (lane == 0) {
        d.rss_ev[si] = pos;
        d.rss_msg[si] = pmsg;
    }
}

// ---------------------------------------------------------------------------------
// Record effects: one wave per 64-slot record tile, lane = row; the wave walks its slots in
// order, kGroup at a time with every cell load of the group issued before any is consumed and
// the next group's loads issued before this group's stores.  A record span's events are staged
// in the wave's LDS rows and stored dense; changed cells are written back non-temporally.
// Cells [cap][cols][rows] with the used rows packed first (rec_pos), so a wave reads one (slot,
// col) run of popcount(used) cells contiguously and no line of unused rows.

// x held in a vector register from here on (uniform values the compiler would otherwise keep in
// scalar registers: k_records' per-op constants and used masks overflow the 102 SGPRs and were
// spilled to VGPR lanes, one v_readlane per reload, a third of the kernel's VALU instructions)
template <class T>
__device__ __forceinline__ T in_vgpr(T x) {
    asm volatile("" : "+v"(x));
    return x;
}

// lane l's value in every lane (l wave-uniform): v_readlane into a scalar register
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}

// kOps: register slots for the record ops (>= n_rops), kGroup: slots whose cells are in flight
// together; instantiated so that a frame's op count does not pay for NFK_MAX_REC_OPS registers.
template <int kOps, int kGroup>
struct RecGrp {  // one group of slots with record work: their ops and cells
    int js[kGroup];
    uint32_t masks[kGroup];  // bit j: op j runs on the slot
    uint32_t rsg[kGroup];  // 1 + the slot's index among the SetRecord slots (0: none)
    uint64_t cur[kGroup][kOps];
};

// kSets: the frame has SetRecord slots (k_rset_slots writes theirs; here their room is reserved)
// kCodes: per op j, bits 2j..2j+1 = 1 (RIADD_CLAMP) / 2 (RFAFFINE) when the launch knows it (the
// common two-op shape: no per-op code branch or its masks), 0 = read from d.rops
template <int kOps, int kGroup, bool kSets, bool kFuse, unsigned kCodes = 0>
__global__ __launch_bounds__(kTPB) void k_records(Dev d) {
    __shared__ uint8_t s_rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    __shared__ uint64_t s_eold[kTPB / 64][kOps * 64], s_enew[kTPB / 64][kOps * 64];  // a span's events,
    __shared__ uint32_t s_errc[kTPB / 64][kOps * 64];                                // per wave
    for (int i = threadIdx.x; i < (int)sizeof(s_rflags) / 4; i += kTPB)
        ((uint32_t*)s_rflags)[i] = ((const uint32_t*)d.tab->rflags)[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rt = blockIdx.x * (kTPB / 64) + w;
    if (rt >= d.n_rtiles) return;  // wave-uniform; no barrier follows
    const int nro = d.n_rops;
    // popcount of a mask's bits below this lane: the lane's row's place among the used rows
    const auto below = [&](uint64_t m) -> uint32_t {
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    };
    const int s0 = rt * kRTile;
    unsigned bytes = 0;    // per lane
    unsigned sbytes = 0;   // per wave (wave-uniform)
    // lane j holds slot s0 + j's fired mask and fan-out descriptor
    uint32_t my_mask = 0, my_rs = 0;
    uint64_t my_desc = 0;
    if (lane < kRTile && s0 + lane < d.N) {
        my_mask = d.fired_mask[s0 + lane] & d.rop_kinds;
        bytes += 4;
        if (kSets) {
            my_rs = d.rs_head[s0 + lane];
            bytes += 4;
        }
        if (my_mask || my_rs) {
            my_desc = d.fan_desc[s0 + lane];
            bytes += 8;
        }
    }
    // lane j: slot s0 + j's used-row mask of each op's record, loaded with the descriptors, so a
    // group's cell addresses (the used rows' places, rec_pos) need no further round trip
    uint64_t my_used[kOps];
    uint32_t my_ops = 0;  // bit j: op j's kind fired on slot s0 + lane
#pragma unroll
    for (int j = 0; j < kOps; j++) {
        if (j < nro) my_ops |= ((my_mask >> d.rops[j].kind) & 1u) << j;
        my_used[j] = 0;
        if (j < nro && !(kSets && my_rs) && ((my_mask >> d.rops[j].kind) & 1))
            my_used[j] = d.rops[j].used[s0 + lane] & rec_rowm(d.rops[j].rows);
    }
    // per op: its column's vector of slot 0 (bytes), the slot stride (bytes) and the op's
    // operands, in vector registers (in_vgpr)
    uint64_t op_base[kOps], op_a[kOps], op_b[kOps], op_c[kOps];
    uint32_t op_stride[kOps];
#pragma unroll
    for (int j = 0; j < kOps; j++) {
        const bool on = j < nro;
        op_base[j] = in_vgpr(on ? (uint64_t)(uintptr_t)(d.rops[j].cells + (size_t)d.rops[j].col * d.rops[j].rows) : 0ull);
        op_stride[j] = in_vgpr(on ? (uint32_t)(d.rops[j].cols * d.rops[j].rows * 8) : 0u);
        op_a[j] = in_vgpr(on ? (uint64_t)d.rops[j].a : 0ull);
        op_b[j] = in_vgpr(on ? (uint64_t)d.rops[j].b : 0ull);
        op_c[j] = in_vgpr(on ? (uint64_t)d.rops[j].c : 0ull);
    }
    unsigned long long work = __ballot(my_mask != 0 || my_rs != 0);
    unsigned pos = 0, pmsg = 0;  // tile-local
    // this tile's output runs as wave-uniform base pointers, indexed by 32-bit tile-local offsets
    const size_t re0 = (size_t)rt * d.re_tcap;
    uint32_t* const t_rrc = d.re_rrc + re0;
    uint64_t* const t_old = d.re_old + re0;
    uint64_t* const t_new = d.re_new + re0;
    uint32_t* const t_moff = d.re_moff + re0;
    const uint32_t mrb = kFuse ? d.msg_rb0 + (uint32_t)rt * d.msg_rtcap : 0u;  // fused: this tile's run
    // Two groups in flight: the next group's cell loads are issued before the current group's
    // stores, so its wait covers the stores' acknowledgements (vmcnt counts loads and stores in
    // issue order) instead of a full HBM round trip after them.
    auto pick_load = [&](RecGrp<kOps, kGroup>& G) {
        // next group of up to kGroup slots with record work, in slot order; every cell load of
        // the group is issued before any is consumed
#pragma unroll
        for (int g = 0; g < kGroup; g++) {
            G.js[g] = work ? __builtin_ctzll(work) : -1;
            if (work) work &= work - 1;
            // (js is wave-uniform: lane reads into scalar registers, no LDS permute)
            G.masks[g] = G.js[g] >= 0 ? rl32(my_ops, G.js[g]) : 0u;  // (bit j: op j runs on the slot)
            G.rsg[g] = (kSets && G.js[g] >= 0) ? rl32(my_rs, G.js[g]) : 0u;
        }
#pragma unroll
        for (int g = 0; g < kGroup; g++)
#pragma unroll
            for (int j = 0; j < kOps; j++) {
                G.cur[g][j] = 0;
                if (j < nro && G.js[g] >= 0 && !(kSets && G.rsg[g]) && ((G.masks[g] >> j) & 1)) {
                    const int e = s0 + G.js[g];
                    // only the used rows: one dense run at the vector's start (rec_pos), lane p
                    // holding the p-th used row, so every load is lane-aligned
                    if (lane < __builtin_popcountll(rl64(my_used[j], G.js[g])))
                        G.cur[g][j] = ((const uint64_t*)(op_base[j] + (uint64_t)e * op_stride[j]))[lane];
                }
            }
    };
    auto process = [&](RecGrp<kOps, kGroup>& G) {
#pragma unroll
        for (int g = 0; g < kGroup; g++) {
            if (G.js[g] < 0) break;
            const int e = s0 + G.js[g];
            const uint64_t desc = rl64(my_desc, G.js[g]);
            const unsigned cls = (unsigned)(desc >> 60);
            if (kSets && G.rsg[g]) {  // (wave-uniform) a slot with SetRecord calls: k_rset_slots writes its
                             // events into the room reserved here
                const int i = (int)G.rsg[g] - 1;
                if (lane == 0) {
                    d.rss_pos[i] = pos;
                    d.rss_pmsg[i] = pmsg;
                }
                pos += d.rss_ev[i];
                pmsg += d.rss_msg[i];
                continue;
            }
            bool ch[kOps], wr[kOps];
            uint64_t nv[kOps];
#pragma unroll
            for (int j = 0; j < kOps; j++) {
                ch[j] = wr[j] = false;
                nv[j] = 0;
                if (j >= nro || !((G.masks[g] >> j) & 1)) continue;
                const RecOpX& ro = d.rops[j];
                // algorithmic bytes, counted per wave: the used mask and the used rows' cells
                const int nu = __builtin_popcountll(rl64(my_used[j], G.js[g]));
                sbytes += 8u + 8u * (unsigned)nu;
                if (lane >= nu) continue;  // lane p: the p-th used row
                const uint64_t c = G.cur[g][j];
                uint64_t nb;
                bool changed;
                const unsigned cc = (kCodes >> (2 * j)) & 3u;  // (j unrolled: a constant)
                if (cc ? cc == 1u : ro.code == NFK_OP_RIADD_CLAMP) {
                    int64_t v = (int64_t)(c + op_a[j]);
                    v = v < (int64_t)op_b[j] ? (int64_t)op_b[j] : v;
                    v = v > (int64_t)op_c[j] ? (int64_t)op_c[j] : v;
                    nb = (uint64_t)v;
                    changed = v != (int64_t)c;  // TData::operator== (NFIDataList.h:98)
                } else {
                    const double x = __longlong_as_double((long long)c);
                    const double m = x * __longlong_as_double((long long)op_a[j]);
                    const double v = m + __longlong_as_double((long long)op_b[j]);
                    const double df = v - x;
                    changed = !(df < 0.001 && df > -0.001);  // NFIDataList.h:106-113
                    nb = (uint64_t)__double_as_longlong(v);
                }
                if (changed) {
                    // (non-temporal: the cell is not read again this frame; measured -7 % of k_records,
                    // while non-temporal event stores cost +30 %: profiles/r01zzf_*)
                    __builtin_nontemporal_store(nb, (uint64_t*)(op_base[j] + (uint64_t)e * op_stride[j]) + lane);
                    wr[j] = true;
                    ch[j] = nb != c;  // coalesced diff: bits must differ
                    nv[j] = nb;
                }
            }
#pragma unroll
            for (int j = 0; j < kOps; j++)
                if (j < nro) sbytes += 8u * (unsigned)__builtin_popcountll(__ballot(wr[j]));  // cells written
            // per-slot event order (rec, row, col): records outer, lanes (rows), cols inner
#pragma unroll
            for (int j0 = 0; j0 < kOps; j0++) {
                if (j0 >= nro || d.rops[j0].gfirst != j0) continue;  // j0 opens a record's op span
                const int j1 = d.rops[j0].glast;
                // lane p's row (lane p holds the p-th used row): every lane sends its lane number to
                // its row's place (rec_pos: a permutation of the lanes, rows past the record's
                // rows in place), so lane p receives the row placed at p
                uint64_t um = 0;
#pragma unroll
                for (int j = 0; j < kOps; j++)
                    if (j >= j0 && j <= j1) um |= rl64(my_used[j], G.js[g]);  // (one record: one mask or 0)
                const uint32_t place = ((um >> lane) & 1) ? below(um)
                                       : lane < d.rops[j0].rows ? (uint32_t)__builtin_popcountll(um) + below(~um & rec_rowm(d.rops[j0].rows))
                                                      : (uint32_t)lane;
                const uint32_t row_at = (uint32_t)__builtin_amdgcn_ds_permute((int)(place * 4), lane);
                // the span's events before this lane's (rows below it, every column) and in total:
                // one ballot + lane-mask count per op instead of a wave scan
                unsigned below = 0, n = 0;
#pragma unroll
                for (int j = 0; j < kOps; j++) {
                    if (!(j >= j0 && j <= j1)) continue;
                    const unsigned long long b = __ballot(ch[j]);
                    below += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
                    n += (unsigned)__builtin_popcountll(b);
                }
                if (n == 0) continue;  // wave-uniform
                unsigned p = pos + below;
                const uint8_t rfl = s_rflags[cls][d.rops[j0].rec];
                const unsigned per = event_msgs(desc, rfl);
                // stage the span's events in this wave's LDS rows at their span index, then write
                // them back dense: lane q stores event q of every output array (full, contiguous
                // runs instead of one sparse store per op and array)
                unsigned q = p - pos;
#pragma unroll
                for (int j = 0; j < kOps; j++) {
                    if (!(j >= j0 && j <= j1 && ch[j])) continue;
                    s_eold[w][q] = G.cur[g][j];
                    s_enew[w][q] = nv[j];
                    s_errc[w][q] = ((uint32_t)G.js[g] << kRrcSitShift) | ((uint32_t)d.rops[j].rec << 16) |
                                   (row_at << 8) | (uint32_t)d.rops[j].col;
                    q++;
                }
                __builtin_amdgcn_wave_barrier();  // (one wave's LDS operations complete in order)
                for (unsigned q0 = 0; q0 < n; q0 += 64) {
                    const unsigned qq = q0 + (unsigned)lane;
                    if (qq >= n) break;
                    const unsigned at = pos + qq;
                    const uint32_t lmo = pmsg + per * qq;
                    t_rrc[at] = s_errc[w][qq];
                    t_old[at] = s_eold[w][qq];
                    t_new[at] = s_enew[w][qq];
                    // unfused: the tile-local offset k_fanout expands the event at; fused, the run is
                    // dense in event order and the readers count their way through it (k_counted_moff)
                    if (!kFuse) t_moff[at] = lmo;
                    if (kFuse && per) {
                        // GetBroadCastObject (AOI:531-593) for the record event, into the tile's run
                        uint32_t* out = d.msg_rcpt + mrb + lmo;
                        if (!(rfl & NFK_PUBLIC)) {
                            out[0] = (uint32_t)e;  // private & !upload: the entity itself
                        } else {  // every player of the group but self
                            const uint32_t np = (uint32_t)((desc >> 32) & 0x3FFF);
                            const uint32_t r1 = (uint32_t)((desc >> 46) & 0x3FFF);
                            uint32_t k = 0;
                            for (uint32_t u = 0; u < np; u++) {
                                if (u + 1 == r1) continue;
                                out[k++] = (uint32_t)d.pl_slot[(uint32_t)desc + u];
                            }
                        }
                    }
                }
                // event records, their recipient words and (public) the player run read per event
                sbytes += n * ((kFuse ? 20u : 24u) + ((kFuse && per) ? 4u * per : 0u) +
                               ((kFuse && per && (rfl & NFK_PUBLIC)) ? 4u * (uint32_t)((desc >> 32) & 0x3FFF) : 0u));
                __builtin_amdgcn_wave_barrier();
                pos += n;
                pmsg += per * n;
            }
        }
    };
    RecGrp<kOps, kGroup> A, B;
    pick_load(A);
    while (A.js[0] >= 0) {
        pick_load(B);
        process(A);
        if (B.js[0] < 0) break;
        pick_load(A);
        process(B);
    }
    if (kSets && my_rs) d.rs_head[s0 + lane] = 0;  // (the groups are consumed)
    if (lane == 0) {
        d.t_re[rt] = pos;
        d.t_msg[d.n_tiles + rt] = pmsg;
    }
    const unsigned wb = (unsigned)wave_sum(bytes) + sbytes;
    if (lane == 0 && wb) tally_add(d, kTallyRec, (unsigned long long)wb + 8);
}

// ---------------------------------------------------------------------------------
// Exclusive scans of the four per-tile count arrays (events, fired, record events, messages) in
// one workgroup of 1024 threads: every thread loads kScanPer consecutive counts of all four
// arrays at once (one memory round trip per pass), then four block scans share each barrier.
// Writes bases[n+1] (bases[n] = total) and the frame totals.
#ifndef NFGPU_SCANPER
#define NFGPU_SCANPER 8
#endif
constexpr int kScanTPB = 1024, kScanPer = NFGPU_SCANPER;

struct ScanArr {
    uint32_t v[kScanPer];
    unsigned long long sum, inc;
};

__device__ __forceinline__ void scan_load(ScanArr& x, const uint32_t* __restrict__ cnt, int len, int i0) {
    x.sum = 0;
    if (i0 + kScanPer <= len) {  // 16-byte loads (cnt is 16-byte aligned, i0 a multiple of kScanPer)
#pragma unroll
        for (int q = 0; q < kScanPer / 4; q++) {
            const uint4 a = ((const uint4*)(cnt + i0))[q];
            x.v[4 * q] = a.x; x.v[4 * q + 1] = a.y; x.v[4 * q + 2] = a.z; x.v[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < kScanPer; q++) x.v[q] = (i0 + q < len) ? cnt[i0 + q] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kScanPer; q++) x.sum += x.v[q];
}
static_assert(kScanPer % 4 == 0, "scan_load's vector path loads 4 counts at a time");

// block-scan step of one array (s_pre = exclusive prefix of the wave totals); returns the pass total
__device__ __forceinline__ unsigned long long scan_store(ScanArr& x, const unsigned long long* s_pre,
                                                         unsigned long long carry, uint32_t* __restrict__ base,
                                                         int len, int i0) {
    unsigned long long run = carry + s_pre[threadIdx.x >> 6] + x.inc - x.sum;
#pragma unroll
    for (int q = 0; q < kScanPer; q++) {
        if (i0 + q < len) base[i0 + q] = (uint32_t)run;
        run += x.v[q];
    }
    return s_pre[kScanTPB / 64];
}

// One workgroup per count array (blockIdx.x: 0 events, 1 fired, 2 record events, 3 message runs;
// block 3 also sums the messages of the tiles fanned out at a fixed stride).
__global__ __launch_bounds__(kScanTPB) void k_scan_tiles(Dev d) {
    __shared__ unsigned long long s_w[kScanTPB / 64 + 1];  // wave totals -> exclusive prefixes, [16] = total
    __shared__ unsigned long long s_real[kScanTPB / 64];  // (block 3) messages of the fixed-stride tiles
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nrt = d.has_recops ? d.n_rtiles : 0;
    const int a = blockIdx.x;
    const uint32_t* cnt = a == 0 ? d.t_ev : a == 1 ? d.t_fi : a == 2 ? d.t_re : d.t_msg;
    uint32_t* base = a == 0 ? d.ev_base : a == 1 ? d.fi_base : a == 2 ? d.re_base : d.msg_base;
    const int len = a < 2 ? d.n_tiles : a == 2 ? nrt : d.n_tiles + nrt;
    // message runs: property tiles fanned out by k_tick take msg_tcap each, record tiles fanned
    // out by k_records msg_rtcap each
    const int fixed = (a == 3 && d.msg_tcap) ? d.n_tiles : 0;
    const int rfixed = (a == 3 && d.fuse_rec) ? nrt : 0;
    unsigned long long carry = 0, real = 0;
    for (int c0 = 0; c0 < len; c0 += kScanTPB * kScanPer) {
        const int i0 = c0 + tid * kScanPer;
        ScanArr x;
        scan_load(x, cnt, len, i0);
        if (a == 3 && (fixed || rfixed)) {  // a fixed-stride tile's run is its reservation
            x.sum = 0;
#pragma unroll
            for (int q = 0; q < kScanPer; q++) {
                if (i0 + q < fixed) {
                    real += x.v[q];
                    x.v[q] = d.msg_tcap;
                } else if (i0 + q >= d.n_tiles && i0 + q < d.n_tiles + rfixed) {
                    real += x.v[q];
                    x.v[q] = d.msg_rtcap;
                }
                x.sum += x.v[q];
            }
        }
        x.inc = wave_incl_scan(x.sum);
        if (lane == 63) s_w[w] = x.inc;
        __syncthreads();
        if (w == 0 && lane < kScanTPB / 64) {
            const unsigned long long v = s_w[lane];
            unsigned long long y = v;
#pragma unroll
            for (int dd = 1; dd < kScanTPB / 64; dd <<= 1) {
                const unsigned long long t = shfl_up_u64(y, dd);
                if (lane >= dd) y += t;
            }
            s_w[lane] = y - v;
            if (lane == kScanTPB / 64 - 1) s_w[kScanTPB / 64] = y;
        }
        __syncthreads();
        carry += scan_store(x, s_w, carry, base, len, i0);
        __syncthreads();
    }
    if (tid == 0) {
        base[len] = (uint32_t)carry;
        if (a == 0) d.ctrl->n_ev = carry;
        if (a == 1) d.ctrl->n_fi = carry;
        if (a == 2) d.ctrl->n_re = carry;
        if (a == 3) {
            d.ctrl->msg_extent = carry;
            if (carry > (unsigned long long)d.msg_cap || (d.ablate & kAblForceMsgCap)) dev_error(d, kErrMsgCap);
        }
    }
    if (a == 3) {  // sum of the fixed-stride tiles' messages
        real = wave_sum(real);
        if (lane == 0) s_real[w] = real;
        __syncthreads();
        if (tid == 0) {
            unsigned long long t = 0;
            for (int i = 0; i < kScanTPB / 64; i++) t += s_real[i];
            d.ctrl->n_msgs_ptiles = t;
        }
    }
}

// ---------------------------------------------------------------------------------
// Fan-out: GetBroadCastObject recipient lists (AOI:531-593) for every dirty event, one workgroup
// per tile (property tiles, then record tiles; blockIdx.x + blk0 is the tile).  When k_tick
// writes its own tiles' fan-out this runs for the record tiles only.  Each tile's messages are
// one contiguous run at msg_base[tile] (k_scan_tiles).  A pass takes up to kTPB * kFanPer
// events: their (first message, first player | slot, count | rank | public) triples go to LDS,
// and each event is then expanded by a group of L lanes (L = the pass's largest recipient count
// rounded up to a power of two, at most 64), so a group of 32 players fills half a wave per event
// and a 2-player group an eighth.  Slots are in (scene, group, guid) order, so the players of
// every group the pass touches form one contiguous run of pl_slot, staged in LDS when it fits;
// messages are staged in LDS and stored coalesced when the pass's run fits, else stored by the
// lane groups directly (each group's stores are contiguous).  Also rewrites each event's
// tile-local message offset as a global one.  Does nothing (and sets no output) when the frame's
// message runs exceed msg_cap: the host grows the buffer and re-runs it.
constexpr int kFanLds = 2048, kFanPer = 4, kFanMsgLds = 4096;

__global__ __launch_bounds__(kTPB) void k_fanout(Dev d, int32_t blk0) {
    __shared__ uint32_t s_pl[kFanLds];
    __shared__ __align__(16) uint32_t s_msg[kFanMsgLds];  // a pass's messages, stored to HBM coalesced
    __shared__ uint32_t s_ev[3 * kTPB * kFanPer];       // a pass's event triples
    __shared__ uint32_t s_pb[3], s_m[2];                // player run [lo, hi), largest count
    __shared__ unsigned s_bytes;
    __shared__ uint8_t s_pflags[NFK_MAX_CLASSES][kMaxProps];
    __shared__ uint8_t s_rflags[NFK_MAX_CLASSES][NFK_MAX_RECORDS];
    if (d.ctrl->msg_extent > (unsigned long long)d.msg_cap) return;  // uniform: host re-runs
    const int tg = (int)blockIdx.x + blk0;  // tile: property tiles, then record tiles
    const bool rec = tg >= d.n_tiles;
    const int t = rec ? tg - d.n_tiles : tg;
    const uint32_t* base = rec ? d.re_base : d.ev_base;
    const unsigned tcap = (unsigned)(rec ? d.re_tcap : d.ev_tcap);
    const size_t off0 = (size_t)t * tcap;
    const uint32_t* slots = rec ? d.re_rrc : d.ev_slot;  // (a record event's slot is in its word)
    const uint32_t s_base = (uint32_t)t * (uint32_t)kRTile;
    uint32_t* moff = rec ? d.re_moff : d.ev_moff;
    // one round trip: the tile's counts, its message range and (speculatively, inside the tile's
    // staging capacity) the first pass's events
    const uint32_t b0 = base[t], b1 = base[t + 1];
    const uint32_t tmsg = d.t_msg[tg], mbase = d.msg_base[tg];
    uint32_t slot[kFanPer], key[kFanPer], lm[kFanPer];
#pragma unroll
    for (int q = 0; q < kFanPer; q++) {
        const unsigned i = q * kTPB + threadIdx.x;
        slot[q] = key[q] = lm[q] = 0;
        if (i < tcap) {
            const uint32_t x = slots[off0 + i];
            slot[q] = rec ? s_base + (x >> kRrcSitShift) : x;
            key[q] = rec ? ((x >> 16) & 0xFF) : d.ev_pid[off0 + i];
            lm[q] = moff[off0 + i];
        }
    }
    const unsigned cnt = b1 - b0;
    if (cnt == 0) return;  // uniform
    if (threadIdx.x == 0) s_bytes = 0;
    if (rec) {
        for (int i = threadIdx.x; i < (int)sizeof(s_rflags) / 4; i += kTPB)
            ((uint32_t*)s_rflags)[i] = ((const uint32_t*)d.tab->rflags)[i];
    } else {
        const int words = d.n_class * kMaxProps / 4;
        for (int i = threadIdx.x; i < words; i += kTPB)
            ((uint32_t*)s_pflags)[i] = ((const uint32_t*)d.tab->pflags)[i];
    }
    unsigned bytes = threadIdx.x == 0 ? 16u : 0u;
    const int lane = threadIdx.x & 63;
    for (unsigned c0 = 0; c0 < cnt; c0 += kTPB * kFanPer) {
        const unsigned c_end = min(cnt, c0 + kTPB * kFanPer);
        if (c0) {
#pragma unroll
            for (int q = 0; q < kFanPer; q++) {
                const unsigned i = c0 + q * kTPB + threadIdx.x;
                if (i < cnt) {
                    const uint32_t x = slots[off0 + i];
                    slot[q] = rec ? s_base + (x >> kRrcSitShift) : x;
                    key[q] = rec ? ((x >> 16) & 0xFF) : d.ev_pid[off0 + i];
                    lm[q] = moff[off0 + i];
                }
            }
        }
        if (threadIdx.x == 0) {
            s_pb[0] = 0xFFFFFFFFu;
            s_pb[1] = 0;
            s_pb[2] = 1;
        }
        __syncthreads();  // s_pflags / s_rflags; s_pb reset; the previous pass is done with s_ev
        // second round trip: the events' fan-out descriptors -> LDS triples, global offsets
        uint32_t lo = 0xFFFFFFFFu, hi = 0, nmax = 0;
#pragma unroll
        for (int q = 0; q < kFanPer; q++) {
            const unsigned i = c0 + q * kTPB + threadIdx.x;
            if (i < c_end) {
                const uint64_t desc = d.fan_desc[slot[q]];
                const unsigned cls = (unsigned)(desc >> 60);
                const uint8_t fl = rec ? s_rflags[cls][key[q]] : s_pflags[cls][key[q]];
                const uint32_t n = event_msgs(desc, fl);
                const bool pub = fl & NFK_PUBLIC;
                const uint32_t src = (uint32_t)desc, np = (uint32_t)((desc >> 32) & 0x3FFF);
                uint32_t* x = s_ev + 3 * (i - c0);
                x[0] = lm[q];
                x[1] = pub ? src : slot[q];
                x[2] = n | ((uint32_t)((desc >> 46) & 0x3FFF) << 14) | (pub ? 0x80000000u : 0u);
                moff[off0 + i] = mbase + lm[q];
                bytes += 4 + 4 + 4 + 8 + 4 + 4 * n;
                nmax = max(nmax, n);
                if (pub && n) {
                    lo = min(lo, src);
                    hi = max(hi, src + np);
                }
            }
            if (i == c0) s_m[0] = lm[q];
        }
        if (threadIdx.x == 0) s_m[1] = c_end < cnt ? moff[off0 + c_end] : tmsg;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, m, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, m, 64));
            nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, m, 64));
        }
        if (lane == 0) {
            if (hi) {
                atomicMin(&s_pb[0], lo);
                atomicMax(&s_pb[1], hi);
            }
            atomicMax(&s_pb[2], nmax);
        }
        __syncthreads();
        const uint32_t p0 = s_m[0], pn = s_m[1] - s_m[0];
        const bool lds_out = pn <= (uint32_t)kFanMsgLds;
        const uint32_t pb_lo = s_pb[0], npl = s_pb[1] > s_pb[0] ? s_pb[1] - s_pb[0] : 0u;
        const bool staged = npl <= (uint32_t)kFanLds;
        const uint32_t nm = s_pb[2];
        const uint32_t L = nm <= 1 ? 1u : nm >= 64 ? 64u : 1u << (32 - __builtin_clz(nm - 1));
        if (staged) {  // third round trip: the players, NFGUID order (pl_slot is in slot order)
            for (uint32_t i = threadIdx.x; i < npl; i += kTPB) s_pl[i] = (uint32_t)d.pl_slot[pb_lo + i];
            bytes += 4 * ((npl + kTPB - 1 - threadIdx.x) / kTPB);
            __syncthreads();
        }
        // expansion: lane group g = threadIdx.x / L takes events g, g + kTPB / L, ...
        uint32_t* out = lds_out ? s_msg : d.msg_rcpt + mbase + p0;
        const uint32_t sub = threadIdx.x & (L - 1);
        for (uint32_t i = threadIdx.x / L; i < c_end - c0; i += kTPB / L) {
            const uint32_t ms = s_ev[3 * i] - p0, a = s_ev[3 * i + 1], b = s_ev[3 * i + 2];
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
        if (lds_out) {
            __syncthreads();
            uint32_t* dst = d.msg_rcpt + mbase + p0;
            if (((mbase + p0) & 3u) == 0) {
                const uint32_t n4 = pn >> 2;
                for (uint32_t i = threadIdx.x; i < n4; i += kTPB) ((uint4*)dst)[i] = ((const uint4*)s_msg)[i];
                if (threadIdx.x < (pn & 3u)) dst[4 * n4 + threadIdx.x] = s_msg[4 * n4 + threadIdx.x];
            } else {
                for (uint32_t i = threadIdx.x; i < pn; i += kTPB) dst[i] = s_msg[i];
            }
        }
        __syncthreads();
    }
    const unsigned wb = (unsigned)wave_sum(bytes);
    if ((threadIdx.x & 63) == 0 && wb) atomicAdd(&s_bytes, wb);
    __syncthreads();
    if (threadIdx.x == 0) tally_add(d, kTallyFan, (unsigned long long)s_bytes);
}

// ---------------------------------------------------------------------------------
// Membership changes (SwitchScene / DestroyObject / cross-shard migration): an entity's state
// travels as a ROW of 64-bit words — its properties, its schedule records (hot 2 words + cold 2
// words per kind) and its record cells + used mask per record.  k_pack gathers rows from slots,
// k_unpack scatters rows (or zeros: a slack slot) into slots, k_meta rewrites the per-slot
// membership metadata of the scene-group segments that changed.  Thread t handles word
// t / n of row t % n, so a wave reads one column across consecutive slots.
__device__ __forceinline__ uint64_t* row_word(const Dev& d, int32_t s, int w) {
    if (w < d.n_if) return prop_ptr(d, (uint32_t)w, s);
    w -= d.n_if;
    if (w < 2 * d.n_obj) return prop_ptr(d, (uint32_t)(d.n_if + (w >> 1)), s) + (w & 1);  // (data, head)
    w -= 2 * d.n_obj;
    if (w < 4 * d.n_kind) {
        const int k = w >> 2, q = w & 3;
        return q < 2 ? (uint64_t*)&d.s_hot[(size_t)k * d.s_kstr + s] + q
                     : (uint64_t*)&d.s_cold[(size_t)k * d.s_kstr + s] + (q - 2);
    }
    w -= 4 * d.n_kind;
    for (int r = 0; r < d.n_rec; r++) {
        const int per = d.tab->rec_rows[r] * d.tab->rec_cols[r];
        if (w < per) return d.rcells[r] + (size_t)s * per + w;
        if (w == per) return d.rused[r] + s;
        w -= per + 1;
    }
    return nullptr;  // unreachable for w < row words
}

__global__ __launch_bounds__(kTPB) void k_pack(Dev d, const int32_t* __restrict__ src, int32_t n, int32_t rw,
                                               uint64_t* __restrict__ rows) {
    const size_t total = (size_t)n * rw;
    for (size_t t = (size_t)blockIdx.x * kTPB + threadIdx.x; t < total; t += (size_t)gridDim.x * kTPB) {
        const int32_t i = (int32_t)(t % (size_t)n), w = (int32_t)(t / (size_t)n);
        if (src[i] >= 0) rows[(size_t)i * rw + w] = *row_word(d, src[i], w);  // (-1: a row nobody reads)
    }
}

// src[i] >= 0: row src[i] of mv; kZeroRow: zeros (a slack slot); kKeepRow: the slot keeps its row;
// else row -1 - src[i] of ins
constexpr int64_t kZeroRow = INT64_MIN, kKeepRow = INT64_MIN + 1;
__global__ __launch_bounds__(kTPB) void k_unpack(Dev d, const int32_t* __restrict__ dst,
                                                 const int64_t* __restrict__ src, int32_t n, int32_t rw,
                                                 const uint64_t* __restrict__ mv, const uint64_t* __restrict__ ins) {
    const size_t total = (size_t)n * rw;
    for (size_t t = (size_t)blockIdx.x * kTPB + threadIdx.x; t < total; t += (size_t)gridDim.x * kTPB) {
        const int32_t i = (int32_t)(t % (size_t)n), w = (int32_t)(t / (size_t)n);
        const int64_t r = src[i];
        if (r == kKeepRow) continue;
        const uint64_t x = r == kZeroRow ? 0ull : (r >= 0 ? mv[(size_t)r * rw + w] : ins[(size_t)(-1 - r) * rw + w]);
        *row_word(d, dst[i], w) = x;
    }
}

// Full re-layout of the segments whose members did not change (only their slot range moves:
// slack recomputed, segments inserted or dropped before them): their pack / unpack / metadata
// lists are generated here from the segment table instead of on the host.  Reads the old
// slot_obj / fan_desc / pl_slot (before k_meta rewrites them), rebasing descriptors and player
// runs from ob to nb.
struct SegMove {
    int32_t ob, nb, n, nc;  // old base, new base, members, new slot count
    int32_t np;             // players (the player run pl_slot[base, base + np))
    int32_t po, lo, pad;    // first pack row, first list entry
};

__global__ __launch_bounds__(kTPB) void k_seg_lists(const SegMove* __restrict__ mv, int32_t n_mv,
                                                    const int32_t* __restrict__ slot_obj,
                                                    const uint64_t* __restrict__ fan_desc,
                                                    const int32_t* __restrict__ pl_slot, int32_t* __restrict__ pack_src,
                                                    int32_t* __restrict__ un_dst, int64_t* __restrict__ un_src,
                                                    int32_t* __restrict__ m_slot, int32_t* __restrict__ m_obj,
                                                    uint64_t* __restrict__ m_desc, int32_t* __restrict__ m_pl) {
    for (int32_t g = blockIdx.x; g < n_mv; g += gridDim.x) {
        const SegMove s = mv[g];
        for (int32_t i = threadIdx.x; i < s.nc; i += kTPB) {
            const int32_t at = s.lo + i, ns = s.nb + i;
            un_dst[at] = ns;
            m_slot[at] = ns;
            if (i < s.n) {
                const int32_t os = s.ob + i;
                un_src[at] = s.po + i;
                pack_src[s.po + i] = os;
                m_obj[at] = slot_obj[os];
                const uint64_t dsc = fan_desc[os];
                m_desc[at] = (dsc & ~0xFFFFFFFFull) | (uint64_t)(uint32_t)s.nb;
            } else {
                un_src[at] = kZeroRow;  // a slack slot
                m_obj[at] = -1;
                m_desc[at] = kDeadDesc;
            }
            m_pl[at] = i < s.np ? pl_slot[s.ob + i] - s.ob + s.nb : 0;
        }
    }
}

// The segments whose member lists changed (SwitchScene, CreateObject, DestroyObject): each new
// member list is the old one with some members removed and some inserted, all in NFGUID order,
// i.e. a MERGE of the old members that stay (their slots in order) with the inserted objects at
// their new ranks, which the host found by binary search in the NFGUID-ordered list.  The slot
// lists are generated here per new slot: a member at new rank i is inserted object a if
// ins_rank[a] == i (a = inserted objects ranked below i), else the (i - a)-th member that stays,
// whose old rank follows from the removed ranks by a binary search; players are ranked by a
// block scan.  (ob < 0: a new (scene, group) pair, all members inserted.)
struct SegEdit {
    int32_t ob, nb, on, nn;  // old base (-1: new segment), new base, old / new members
    int32_t nc, np;          // new slot count, players among the new members
    int32_t ni, io;          // inserted objects [io, io + ni) of the ins_* arrays
    int32_t nr, ro;          // removed old ranks [ro, ro + nr) of rem_rank
    int32_t po, lo;          // first pack row (nn rows), first list entry (nc entries)
    int32_t all, pad;        // all: every member moves (a full re-layout), else only the ones whose slot changes
};

__global__ __launch_bounds__(kTPB) void k_seg_edit(const SegEdit* __restrict__ ed, int32_t n_ed,
                                                   const int32_t* __restrict__ ins_rank,
                                                   const int32_t* __restrict__ ins_obj,
                                                   const uint64_t* __restrict__ ins_meta,  // cls << 60 | player
                                                   const int64_t* __restrict__ ins_src,    // old slot, or -1 - import row
                                                   const int32_t* __restrict__ rem_rank,
                                                   const int32_t* __restrict__ slot_obj,
                                                   const uint64_t* __restrict__ fan_desc, int32_t* __restrict__ pack_src,
                                                   int32_t* __restrict__ un_dst, int64_t* __restrict__ un_src,
                                                   int32_t* __restrict__ m_slot, int32_t* __restrict__ m_obj,
                                                   uint64_t* __restrict__ m_desc, int32_t* __restrict__ m_pl) {
    __shared__ int32_t s_w[kTPB / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int32_t g = blockIdx.x; g < n_ed; g += gridDim.x) {
        const SegEdit s = ed[g];
        const int32_t* ir = ins_rank + s.io;
        const int32_t* rr = rem_rank + s.ro;
        int32_t carry = 0;  // players at new ranks below the chunk
        for (int32_t c0 = 0; c0 < s.nc; c0 += kTPB) {  // (block-uniform)
            const int32_t i = c0 + (int32_t)threadIdx.x;
            const int32_t at = s.lo + i, ns = s.nb + i;
            bool pl = false;
            int32_t obj = -1;
            uint64_t meta = 0;  // cls << 60
            int64_t src = kKeepRow;
            int32_t psrc = -1;  // the old slot packed into row po + i (-1: none)
            if (i < s.nn) {
                // inserted objects ranked below i
                int32_t lo = 0, hi = s.ni;
                while (lo < hi) {
                    const int32_t mid = (lo + hi) >> 1;
                    if (ir[mid] < i) lo = mid + 1;
                    else hi = mid;
                }
                if (lo < s.ni && ir[lo] == i) {
                    obj = ins_obj[s.io + lo];
                    meta = ins_meta[s.io + lo];
                    pl = meta & 1;
                    meta &= 0xFull << 60;
                    const int64_t sr = ins_src[s.io + lo];
                    if (sr < 0) {
                        src = sr;  // an imported row
                    } else {
                        psrc = (int32_t)sr;
                        src = s.po + i;
                    }
                } else {
                    // the k-th member that stays (k = i - lo) has old rank k + j, j = removed ranks below it:
                    // the largest j with rr[j - 1] - (j - 1) <= k
                    const int32_t k = i - lo;
                    int32_t a = 0, b = s.nr;
                    while (a < b) {
                        const int32_t mid = (a + b) >> 1;
                        if (rr[mid] - mid <= k) a = mid + 1;
                        else b = mid;
                    }
                    const int32_t os = s.ob + k + a;
                    obj = slot_obj[os];
                    const uint64_t od = fan_desc[os];
                    meta = od & (0xFull << 60);
                    pl = ((od >> 46) & 0x3FFF) != 0;
                    if (s.all || os != ns) {
                        psrc = os;
                        src = s.po + i;
                    }
                }
            } else if (i < s.nc) {
                // slack: cleared if an entity occupied the slot before
                src = (s.all || (s.ob == s.nb && i < s.on)) ? kZeroRow : kKeepRow;
            }
            // player rank: block scan of the player flags, carried across chunks
            const unsigned long long bal = __ballot(pl && i < s.nn);
            const int32_t below_w = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (lane == 0) s_w[wv] = (int32_t)__builtin_popcountll(bal);
            __syncthreads();
            int32_t before = carry, tot = 0;
#pragma unroll
            for (int q = 0; q < kTPB / 64; q++) {
                before += q < wv ? s_w[q] : 0;
                tot += s_w[q];
            }
            __syncthreads();
            carry += tot;
            if (i < s.nc) {
                const int32_t prank = before + below_w;
                un_dst[at] = ns;
                un_src[at] = src;
                m_slot[at] = ns;
                if (i < s.nn) {
                    m_obj[at] = obj;
                    m_desc[at] = (uint64_t)(uint32_t)s.nb | ((uint64_t)s.np << 32) |
                                 ((uint64_t)(pl ? prank + 1 : 0) << 46) | meta;
                    if (pl) m_pl[s.lo + prank] = ns;
                } else {
                    m_obj[at] = -1;
                    m_desc[at] = kDeadDesc;
                }
                if (i >= s.np) m_pl[at] = 0;
            }
            if (i < s.nn) pack_src[s.po + i] = psrc;
        }
    }
}

__global__ __launch_bounds__(kTPB) void k_meta(const int32_t* __restrict__ slot, const int32_t* __restrict__ obj,
                                               const uint64_t* __restrict__ desc, const int32_t* __restrict__ pl,
                                               int32_t n, int32_t* __restrict__ slot_obj,
                                               uint64_t* __restrict__ fan_desc, int32_t* __restrict__ pl_slot) {
    const int32_t i = blockIdx.x * kTPB + threadIdx.x;
    if (i >= n) return;
    const int32_t s = slot[i];
    slot_obj[s] = obj[i];
    fan_desc[s] = desc[i];
    pl_slot[s] = pl[i];
}

// ---------------------------------------------------------------------------------
// Leaderboards (NFIRankRedisModule::GetRange, a Redis ZREVRANGE over a property's score): the
// score is the property as a double (SetRankValue takes a double); keys are the scores' bits
// mapped to an unsigned order.  A radix select finds the score of the k-th entity (8-bit digits,
// most significant first), then every entity at or above it is collected; the host orders that
// small set by (score desc, NFGUID string desc) and keeps k.
__device__ __forceinline__ uint64_t rank_key(const Dev& d, int32_t pid, int e) {
    const uint64_t raw = *prop_ptr(d, (uint32_t)pid, e);
    const double sc = pid < d.n_int ? (double)(int64_t)raw : __longlong_as_double((long long)raw);
    const uint64_t b = (uint64_t)__double_as_longlong(sc == 0.0 ? 0.0 : sc);  // -0 == +0
    return (b >> 63) ? ~b : (b | (1ull << 63));
}

__global__ __launch_bounds__(kTPB) void k_rank_hist(Dev d, int32_t pid, uint64_t prefix, uint64_t pmask, int shift,
                                                    unsigned* __restrict__ hist) {
    __shared__ unsigned s_h[256];
    for (int i = threadIdx.x; i < 256; i += kTPB) s_h[i] = 0;
    __syncthreads();
    for (int e = blockIdx.x * kTPB + threadIdx.x; e < d.N; e += gridDim.x * kTPB) {
        if (desc_dead(d.fan_desc[e])) continue;
        const uint64_t k = rank_key(d, pid, e);
        if ((k & pmask) == prefix) atomicAdd(&s_h[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += kTPB)
        if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

__global__ __launch_bounds__(kTPB) void k_rank_collect(Dev d, int32_t pid, uint64_t thr, unsigned* __restrict__ n,
                                                       int64_t* __restrict__ out, unsigned cap) {
    for (int e = blockIdx.x * kTPB + threadIdx.x; e < d.N; e += gridDim.x * kTPB) {
        if (desc_dead(d.fan_desc[e])) continue;
        if (rank_key(d, pid, e) >= thr) {
            const unsigned i = atomicAdd(n, 1u);
            if (i < cap) {
                out[2 * (size_t)i] = e;  // (slot, raw property word)
                out[2 * (size_t)i + 1] = (int64_t)*prop_ptr(d, (uint32_t)pid, e);
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// GetProperty* reads (nfk_get_props): word src[i] of the property memory, or (bit 63) of the rows of
// entities imported in this window
__global__ __launch_bounds__(kTPB) void k_gather_words(const uint64_t* __restrict__ src, int32_t n,
                                                       const uint64_t* __restrict__ pmem,
                                                       const uint64_t* __restrict__ ins, uint64_t* __restrict__ out) {
    const int i = blockIdx.x * kTPB + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = src[i];
    out[i] = (s >> 63) ? ins[s & ~(1ull << 63)] : pmem[s];
}

// GetRecord* reads (nfk_get_records): 8-byte words at device addresses (used masks and cells)
__global__ __launch_bounds__(kTPB) void k_gather_abs(const uint64_t* __restrict__ addr, int32_t n,
                                                     uint64_t* __restrict__ out) {
    const int i = blockIdx.x * kTPB + threadIdx.x;
    if (i >= n) return;
    out[i] = *(const uint64_t*)(uintptr_t)addr[i];
}

// ---------------------------------------------------------------------------------
// Readback only (not part of a frame): tile-staged array -> dense array in global order.
template <typename T>
__global__ __launch_bounds__(kTPB) void k_compact(const T* __restrict__ src, T* __restrict__ dst,
                                                  const uint32_t* __restrict__ base, int n_tiles, int tcap) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b;
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) dst[b + i] = src[(size_t)t * tcap + i];
    }
}

// ---------------------------------------------------------------------------------
// nfk_read_frame: the frame's outputs as dense host-ready arrays, in object-index terms.
// tile-staged slots -> dense object indices
__global__ __launch_bounds__(kTPB) void k_compact_obj(const uint32_t* __restrict__ src, int32_t* __restrict__ dst,
                                                      const uint32_t* __restrict__ base, int n_tiles, int tcap,
                                                      const int32_t* __restrict__ slot_obj) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b;
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) dst[b + i] = slot_obj[src[(size_t)t * tcap + i]];
    }
}
// the property tiles' events (object, property, old, new) and fired heartbeats (object, kind, remain)
// in one launch: what four k_compact / k_compact_obj launches and three more do one array each
// (a small world's read-back is launch-bound: config[0]).  A null destination skips its list.
__global__ __launch_bounds__(kTPB) void k_compact_frame(Dev d, const int32_t* __restrict__ slot_obj,
                                                        int32_t* __restrict__ eo, uint32_t* __restrict__ ep,
                                                        uint64_t* __restrict__ eold, uint64_t* __restrict__ enew,
                                                        int32_t* __restrict__ fo, uint32_t* __restrict__ fk,
                                                        int32_t* __restrict__ fr) {
    for (int t = blockIdx.x; t < d.n_tiles; t += gridDim.x) {
        if (eo) {
            const uint32_t b = d.ev_base[t], n = d.ev_base[t + 1] - b;
            const size_t s0 = (size_t)t * d.ev_tcap;
            for (uint32_t i = threadIdx.x; i < n; i += kTPB) {
                eo[b + i] = slot_obj[d.ev_slot[s0 + i]];
                ep[b + i] = d.ev_pid[s0 + i];
                eold[b + i] = d.ev_old[s0 + i];
                enew[b + i] = d.ev_new[s0 + i];
            }
        }
        if (fo) {
            const uint32_t b = d.fi_base[t], n = d.fi_base[t + 1] - b;
            const size_t s0 = (size_t)t * d.fi_tcap;
            for (uint32_t i = threadIdx.x; i < n; i += kTPB) {
                fo[b + i] = slot_obj[d.fi_slot[s0 + i]];
                fk[b + i] = d.fi_kind[s0 + i];
                fr[b + i] = d.fi_remain[s0 + i];
            }
        }
    }
}
// record events: the slot from the event word and its tile, the word in the host format
__global__ __launch_bounds__(kTPB) void k_compact_rec(const uint32_t* __restrict__ src, int32_t* __restrict__ obj,
                                                      uint32_t* __restrict__ rrc, const uint32_t* __restrict__ base,
                                                      int n_tiles, int tcap, const int32_t* __restrict__ slot_obj) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b;
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) {
            const uint32_t x = src[(size_t)t * tcap + i];
            obj[b + i] = slot_obj[(uint32_t)t * (uint32_t)kRTile + (x >> kRrcSitShift)];
            rrc[b + i] = x & kRrcHost;
        }
    }
}
// Tiles whose fan-out k_tick (property tiles) or k_records (record tiles) wrote itself store no
// per-event message offsets: a tile's run holds its events' recipients in event order, so an
// event's dense CSR offset is the tile's dense base (db) plus the recipient counts (event_msgs of
// the event's property / record flags for the entity's class, as the frame counted them) of the
// events before it in its tile.  rec: the record tiles, else the property tiles.
__global__ __launch_bounds__(kTPB) void k_counted_moff(Dev d, int rec, uint32_t* __restrict__ dst,
                                                       const uint32_t* __restrict__ db) {
    __shared__ uint8_t s_fl[NFK_MAX_CLASSES * kMaxProps];  // pflags, or rflags (NFK_MAX_RECORDS per class)
    __shared__ uint32_t s_w[kTPB / 64 + 1];
    const int fw = rec ? NFK_MAX_RECORDS : kMaxProps;  // flags per class
    const uint8_t* fl = rec ? &d.tab->rflags[0][0] : &d.tab->pflags[0][0];
    for (int i = threadIdx.x; i < NFK_MAX_CLASSES * fw; i += kTPB) s_fl[i] = fl[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nt = rec ? d.n_rtiles : d.n_tiles;
    const uint32_t* base = rec ? d.re_base : d.ev_base;
    const size_t tcap = (size_t)(rec ? d.re_tcap : d.ev_tcap);
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b;
        uint32_t carry = db[(rec ? d.n_tiles : 0) + t];
        for (uint32_t c0 = 0; c0 < n; c0 += kTPB) {  // uniform
            const uint32_t i = c0 + threadIdx.x;
            uint32_t per = 0;
            if (i < n) {
                uint32_t slot, key;
                if (rec) {
                    const uint32_t x = d.re_rrc[(size_t)t * tcap + i];
                    slot = (uint32_t)t * (uint32_t)kRTile + (x >> kRrcSitShift);
                    key = (x >> 16) & 0xFF;
                } else {
                    slot = d.ev_slot[(size_t)t * tcap + i];
                    key = d.ev_pid[(size_t)t * tcap + i];
                }
                const uint64_t desc = d.fan_desc[slot];
                per = event_msgs(desc, s_fl[(uint32_t)(desc >> 60) * (uint32_t)fw + key]);
            }
            const uint32_t incl = wave_incl_scan_u32(per);
            if (lane == 63) s_w[w] = incl;
            __syncthreads();
            if (threadIdx.x == 0) {
                uint32_t a = 0;
                for (int q = 0; q < kTPB / 64; q++) {
                    const uint32_t v = s_w[q];
                    s_w[q] = a;
                    a += v;
                }
                s_w[kTPB / 64] = a;
            }
            __syncthreads();
            if (i < n) dst[b + i] = carry + s_w[w] + incl - per;
            carry += s_w[kTPB / 64];
            __syncthreads();  // (s_w is rewritten by the next chunk)
        }
    }
}
// object-property head halves: 0 for the other events (their entries are unwritten)
__global__ __launch_bounds__(kTPB) void k_compact_h(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                    const uint32_t* __restrict__ pid, const uint32_t* __restrict__ base,
                                                    int n_tiles, int tcap, int n_if) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b;
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) {
            const size_t s = (size_t)t * tcap + i;
            dst[b + i] = (int)pid[s] >= n_if ? src[s] : 0ull;
        }
    }
}
// exclusive scan of n counts (one workgroup of 1024: a contiguous chunk per thread)
__global__ __launch_bounds__(1024) void k_scan_counts(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ out,
                                                      int n) {
    __shared__ uint32_t s[1024];
    const int per = (n + 1023) / 1024, i0 = min(n, (int)threadIdx.x * per), i1 = min(n, i0 + per);
    uint32_t sum = 0;
    for (int i = i0; i < i1; i++) sum += cnt[i];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the chunk sums
        const uint32_t v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t acc = s[threadIdx.x] - sum;
    for (int i = i0; i < i1; i++) {
        out[i] = acc;
        acc += cnt[i];
    }
    if (threadIdx.x == 1023) out[n] = s[1023];
}
// message offsets of tile-staged events: the tile's run start mb[t] -> its dense start db[t]
__global__ __launch_bounds__(kTPB) void k_compact_moff(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                       const uint32_t* __restrict__ base, int n_tiles, int tcap,
                                                       const uint32_t* __restrict__ mb, const uint32_t* __restrict__ db) {
    for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const uint32_t b = base[t], n = base[t + 1] - b, d0 = db[t] - mb[t];
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) dst[b + i] = src[(size_t)t * tcap + i] + d0;
    }
}
// every tile's recipient run, mb[t] -> db[t], slots -> objects
__global__ __launch_bounds__(kTPB) void k_runs_obj(const uint32_t* __restrict__ rcpt, int32_t* __restrict__ dst,
                                                   const uint32_t* __restrict__ mb, const uint32_t* __restrict__ mc,
                                                   const uint32_t* __restrict__ db, int ntt,
                                                   const int32_t* __restrict__ slot_obj) {
    for (int t = blockIdx.x; t < ntt; t += gridDim.x) {
        const uint32_t s0 = mb[t], n = mc[t], d0 = db[t];
        for (uint32_t i = threadIdx.x; i < n; i += kTPB) dst[d0 + i] = slot_obj[rcpt[(size_t)s0 + i]];
    }
}
// fired entries' sort keys: (rank of the object's NFGUID, kind) and their dense index
__global__ __launch_bounds__(kTPB) void k_fired_keys(const int32_t* __restrict__ fobj, const int32_t* __restrict__ fkind,
                                                     const int32_t* __restrict__ rank, uint64_t* __restrict__ keys,
                                                     uint32_t* __restrict__ idx, int n) {
    const int i = blockIdx.x * kTPB + threadIdx.x;
    if (i >= n) return;
    keys[i] = ((uint64_t)(uint32_t)rank[fobj[i]] << 5) | (uint64_t)fkind[i];
    idx[i] = (uint32_t)i;
}
// A stable sort of n <= 2 * kSmallSort (key, value) pairs in one launch: each pair's place is the count
// of pairs with a smaller key, or an equal key and a smaller index — the order rocPRIM's stable radix
// sort of the same keys gives, without its passes' launches (a window's few hundred SetProperty or
// schedule calls, a small per-Set log: config[0], the migration frames' SwitchScene writes)
// One workgroup per 256 pairs (each loads every key into LDS), so the n^2 compares spread over n / 256
// CUs.  Used up to kSmallPairs pairs: at 1536 (a migration frame's SwitchScene writes) the compares cost
// more than rocPRIM's passes (aux 34.5 -> 60.8 us; one workgroup of 1024 threads: 110 us,
// profiles/r17o_selfmig_trace.txt, r17p_selfmig_trace.txt); at a hundred (config[0]) one launch wins.
constexpr int kSmallPairs = 512;
__global__ __launch_bounds__(kTPB) void k_sort_small_pairs(const uint64_t* __restrict__ k1, uint64_t* __restrict__ k2,
                                                           const uint32_t* __restrict__ v1, uint32_t* __restrict__ v2,
                                                           int n) {
    __shared__ uint64_t sk[kSmallPairs];  // (n <= kSmallPairs)
    for (int i = threadIdx.x; i < n; i += kTPB) sk[i] = k1[i];
    __syncthreads();
    const int i = blockIdx.x * kTPB + (int)threadIdx.x;
    if (i >= n) return;
    const uint64_t k = sk[i];
    int at = 0;
    for (int j = 0; j < n; j++) at += (sk[j] < k || (sk[j] == k && j < i)) ? 1 : 0;
    k2[at] = k;
    v2[at] = v1[i];
}
// a small frame's fired list (n <= kSmallSort) into the walk's order in one launch: the keys are unique
// ((object, kind) fires once a frame), so each entry's place is the count of smaller keys (what the
// radix sort of k_fired_keys' keys and k_permute3 give, without their launches: config[0])
constexpr int kSmallSort = 1024;
__global__ __launch_bounds__(kTPB) void k_fired_small(const int32_t* __restrict__ fobj,
                                                      const int32_t* __restrict__ fkind,
                                                      const int32_t* __restrict__ frem,
                                                      const int32_t* __restrict__ rank, int32_t* __restrict__ ao,
                                                      int32_t* __restrict__ bo, int32_t* __restrict__ co, int n) {
    __shared__ uint64_t sk[kSmallSort];  // (every key, in each of the n / 256 workgroups)
    for (int j = threadIdx.x; j < n; j += kTPB) sk[j] = ((uint64_t)(uint32_t)rank[fobj[j]] << 5) | (uint64_t)fkind[j];
    __syncthreads();
    const int i = blockIdx.x * kTPB + (int)threadIdx.x;
    if (i >= n) return;
    const uint64_t k = sk[i];
    int at = 0;
    for (int j = 0; j < n; j++) at += sk[j] < k ? 1 : 0;
    ao[at] = fobj[i];
    bo[at] = fkind[i];
    co[at] = frem[i];
}
__global__ __launch_bounds__(kTPB) void k_permute3(const uint32_t* __restrict__ idx, const int32_t* __restrict__ a,
                                                   const int32_t* __restrict__ b, const int32_t* __restrict__ c,
                                                   int32_t* __restrict__ ao, int32_t* __restrict__ bo,
                                                   int32_t* __restrict__ co, int n) {
    const int i = blockIdx.x * kTPB + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = idx[i];
    ao[i] = a[j];
    bo[i] = b[j];
    co[i] = c[j];
}

}  // namespace nfgpu
