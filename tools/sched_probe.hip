// Schedule-scan probe (measurement tool, not on the product path): k_tick's heartbeat scan in
// isolation on config[1]'s shape — 1M slots, 5 kinds of 16-byte schedule records in [kind][slot]
// arrays (kColPad apart), an 8-byte descriptor per slot — with progressively less of the scan's
// work, to find what its ~127 MB per frame costs beyond streaming those bytes:
//   full     fire test, reschedule and store of the fired records, remains to LDS, a block scan of
//            the fired counts, the fired list (slot, kind, remain) at the tile's fixed-stride run
//   nolist   the same without the block scan and the fired list
//   noscan   the fired list at per-thread fixed slots (no block scan, no barrier)
//   loads    the loads and the fire test only (one word per thread written)
//   stream   the same bytes as 'full' as a grid-stride stream of 16-byte loads and stores
// Prints one JSON line per case (best and median us of 20 launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                       \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                               \
        }                                                           \
    } while (0)

struct alignas(16) Rec {
    int64_t next;
    int32_t remain;
    uint32_t state;
};
constexpr int kTPB = 256, kK = 5;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct P {
    Rec* hot;
    Rec* shadow;
    int64_t kstr;
    const uint64_t* desc;
    uint32_t* fi_slot;
    uint32_t* fi_kind;
    int32_t* fi_rem;
    uint32_t* t_fi;
    uint32_t* sink;
    int64_t now;
    int fi_tcap;
};

// kLd: non-temporal schedule loads; kSt: 0 plain record stores, 1 non-temporal, 2 to a second
// (shadow) copy of the records instead of in place, 3 only the dense kind's (Move) stores, 4 every
// record of every kind stored (whole lines), fired or not
// kLay: 0 records in [kind][slot] arrays (k_tick's layout), 1 one [slot][kind] block of every kind
// (80 B per slot), 2 the dense kind (Move) in its own array and the four sparse kinds in one
// [slot][4] block (64 B per slot)
__host__ __device__ __forceinline__ size_t rec_at(int lay, int64_t kstr, int k, uint32_t e) {
    if (lay == 1) return (size_t)e * kK + k;
    if (lay == 2) return k == 2 ? (size_t)e : (size_t)kstr + (size_t)e * 4 + (k < 2 ? k : k - 1);
    return (size_t)k * kstr + e;
}
template <int kMode, bool kLd = true, int kSt = 0, int kLay = 0>  // kMode 0 full, 1 nolist, 2 noscan, 3 loads
__global__ __launch_bounds__(kTPB) void scan(P p) {
    __shared__ int32_t s_rem[kK * kTPB];
    __shared__ uint32_t s_w[4];
    const uint32_t e = blockIdx.x * kTPB + threadIdx.x;
    Rec h[kK];
#pragma unroll
    for (int k = 0; k < kK; k++) {  // (non-temporal, as k_tick's schedule loads)
        const u32x4* a = (const u32x4*)(p.hot + rec_at(kLay, p.kstr, k, e));
        const u32x4 x = kLd ? __builtin_nontemporal_load(a) : *a;
        __builtin_memcpy(&h[k], &x, 16);
    }
    const uint64_t desc = __builtin_nontemporal_load(p.desc + e);
    uint32_t fired = 0;
#pragma unroll
    for (int k = 0; k < kK; k++) {
        if ((desc >> 63) || !(h[k].state & 1) || !(p.now > h[k].next)) continue;
        h[k].remain -= 1;
        fired |= 1u << k;
        h[k].next += (int64_t)((int32_t)h[k].state >> 4);
        if (kMode <= 2 && kSt >= 5) continue;  // (stored below, by lane groups)
        if (kMode <= 2 && kSt != 4 && !(kSt == 3 && k != 2)) {
            Rec* d = (kSt == 2 ? p.shadow : p.hot) + rec_at(kLay, p.kstr, k, e);
            u32x4 x;
            __builtin_memcpy(&x, &h[k], 16);
            if (kSt == 1)
                __builtin_nontemporal_store(x, (u32x4*)d);
            else
                *(u32x4*)d = x;
        }
        s_rem[k * kTPB + threadIdx.x] = h[k].remain;
    }
    if (kSt >= 5) {  // a record is stored when any lane of its group of 2 / 4 / 8 fired that kind:
                     // whole 32 / 64 / 128-byte sectors (the unchanged neighbours rewrite their own)
        constexpr int g = kSt == 5 ? 2 : kSt == 6 ? 4 : 8;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < kK; k++) {
            const uint64_t m = __ballot((fired >> k) & 1);
            if ((m >> (lane & ~(g - 1))) & ((1ull << g) - 1)) {
                u32x4 x;
                __builtin_memcpy(&x, &h[k], 16);
                *(u32x4*)(p.hot + k * p.kstr + e) = x;
            }
        }
    }
    if (kSt == 4)
#pragma unroll
        for (int k = 0; k < kK; k++) {
            u32x4 x;
            __builtin_memcpy(&x, &h[k], 16);
            *(u32x4*)(p.hot + k * p.kstr + e) = x;
        }
    if (kMode == 3) {
        if (fired == 0xFFFFFFFFu) p.sink[e] = fired;
        return;
    }
    if (kMode == 1) return;
    const uint32_t nf = __builtin_popcount(fired);
    uint32_t pos;
    if (kMode == 0) {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t inc = nf;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (int i = 0; i < 4; i++) {
            before += i < w ? s_w[i] : 0u;
            tot += s_w[i];
        }
        pos = before + inc - nf;
        if (threadIdx.x == 0) p.t_fi[blockIdx.x] = tot;
    } else {
        pos = threadIdx.x * kK;
    }
    const size_t b = (size_t)blockIdx.x * p.fi_tcap;
    uint32_t f = fired;
    while (f) {
        const int k = __builtin_ctz(f);
        f &= f - 1;
        p.fi_slot[b + pos] = e;
        p.fi_kind[b + pos] = k;
        p.fi_rem[b + pos] = s_rem[k * kTPB + threadIdx.x];
        pos++;
    }
}

__global__ __launch_bounds__(256) void stream(const u32x4* __restrict__ r, size_t nr, u32x4* __restrict__ w, size_t nw) {
    const size_t stride = (size_t)gridDim.x * 256;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nr; i += stride) {
        const u32x4 x = __builtin_nontemporal_load(r + i);
        acc ^= x.x ^ x.w;
    }
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += stride) w[i] = u32x4{(uint32_t)i, acc, 0, 0};
}

int main() {
    const int N = 1 << 20, T = N / kTPB;
    const int64_t kstr = N + 2304 / 16;
    std::vector<Rec> hot((size_t)kK * kstr);
    std::vector<uint64_t> desc(N, 0);
    // Move (kind 2) due every frame; kinds 0, 1, 3, 4 due for ~10 / 5 / 3 / 14 % of the slots
    const int pct[kK] = {10, 5, 100, 3, 14};
    uint32_t seed = 7;
    std::vector<Rec> hot_lay[3];
    for (int lay = 0; lay < 3; lay++) hot_lay[lay].assign(hot.size(), Rec{(int64_t)1 << 60, -1, 0u});
    for (int k = 0; k < kK; k++)
        for (int i = 0; i < N; i++) {
            seed = seed * 1664525u + 1013904223u;
            const bool due = (int)((seed >> 8) % 100) < pct[k];
            const Rec r{due ? 0 : (int64_t)1 << 60, -1, 1u | 2u | (0u << 4)};
            hot[(size_t)k * kstr + i] = r;
            for (int lay = 0; lay < 3; lay++) hot_lay[lay][rec_at(lay, kstr, k, (uint32_t)i)] = r;
        }
    P p;
    CK(hipMalloc(&p.hot, hot.size() * sizeof(Rec)));
    CK(hipMemcpy(p.hot, hot.data(), hot.size() * sizeof(Rec), hipMemcpyHostToDevice));
    CK(hipMalloc(&p.shadow, hot.size() * sizeof(Rec)));
    uint64_t* dd;
    CK(hipMalloc(&dd, (size_t)N * 8));
    CK(hipMemcpy(dd, desc.data(), (size_t)N * 8, hipMemcpyHostToDevice));
    p.desc = dd;
    p.kstr = kstr;
    p.fi_tcap = kK * kTPB;
    CK(hipMalloc(&p.fi_slot, (size_t)T * p.fi_tcap * 4));
    CK(hipMalloc(&p.fi_kind, (size_t)T * p.fi_tcap * 4));
    CK(hipMalloc(&p.fi_rem, (size_t)T * p.fi_tcap * 4));
    CK(hipMalloc(&p.t_fi, (size_t)T * 4));
    CK(hipMalloc(&p.sink, (size_t)N * 4));
    p.now = 1;
    // fired per slot ~1.32: bytes read 5*16+8, written 16*fired + 12*fired
    const double rd = (double)N * (kK * 16 + 8), wr = (double)N * 1.32 * (16 + 12);
    u32x4 *sr, *sw;
    CK(hipMalloc(&sr, (size_t)rd + 64));
    CK(hipMalloc(&sw, (size_t)wr + 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[21] = {"full", "nolist", "noscan", "loads", "stream", "nolist_plainld", "nolist_ntst",
                             "nolist_shadow", "nolist_plainld_ntst", "nolist_dense_kind_only", "nolist_all_records",
                             "nolist_all_records_plainld", "nolist_sector32", "nolist_sector64", "nolist_line128",
                             "aos5_nolist", "aos5_loads", "aos5_full", "hyb_nolist", "hyb_loads", "hyb_full"};
    for (int m = 0; m < 21; m++) {
        const int lay = m >= 18 ? 2 : m >= 15 ? 1 : 0;  // the records in the case's layout
        CK(hipMemcpy(p.hot, hot_lay[lay].data(), hot.size() * sizeof(Rec), hipMemcpyHostToDevice));
        std::vector<float> t;
        for (int it = 0; it < 22; it++) {
            CK(hipEventRecord(a));
            if (m == 0) scan<0><<<T, kTPB>>>(p);
            if (m == 1) scan<1><<<T, kTPB>>>(p);
            if (m == 2) scan<2><<<T, kTPB>>>(p);
            if (m == 3) scan<3><<<T, kTPB>>>(p);
            if (m == 4) stream<<<256 * 8, 256>>>(sr, (size_t)rd / 16, sw, (size_t)wr / 16);
            if (m == 5) scan<1, false, 0><<<T, kTPB>>>(p);
            if (m == 6) scan<1, true, 1><<<T, kTPB>>>(p);
            if (m == 7) scan<1, true, 2><<<T, kTPB>>>(p);
            if (m == 8) scan<1, false, 1><<<T, kTPB>>>(p);
            if (m == 9) scan<1, true, 3><<<T, kTPB>>>(p);
            if (m == 10) scan<1, true, 4><<<T, kTPB>>>(p);
            if (m == 11) scan<1, false, 4><<<T, kTPB>>>(p);
            if (m == 12) scan<1, true, 5><<<T, kTPB>>>(p);
            if (m == 13) scan<1, true, 6><<<T, kTPB>>>(p);
            if (m == 14) scan<1, true, 7><<<T, kTPB>>>(p);
            if (m == 15) scan<1, true, 0, 1><<<T, kTPB>>>(p);
            if (m == 16) scan<3, true, 0, 1><<<T, kTPB>>>(p);
            if (m == 17) scan<0, true, 0, 1><<<T, kTPB>>>(p);
            if (m == 18) scan<1, true, 0, 2><<<T, kTPB>>>(p);
            if (m == 19) scan<3, true, 0, 2><<<T, kTPB>>>(p);
            if (m == 20) scan<0, true, 0, 2><<<T, kTPB>>>(p);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it >= 2) t.push_back(ms * 1000);
        }
        std::sort(t.begin(), t.end());
        printf("{\"case\": \"%s\", \"best_us\": %.1f, \"median_us\": %.1f, \"MB\": %.0f}\n", names[m], t[0], t[t.size() / 2],
               (rd + wr) / 1e6);
    }
    return 0;
}
