// Store-pattern probe for k_tick's event emission (measurement tool, not on the product path).
// One thread per entity, 256-entity tiles at a fixed output stride, each entity with nd events
// (2 or 3: k_tick's config[1] mix, 2.4 per entity) in property order at tile-local rank pev0 (a
// block scan): slot (u32), pid (u32), old (u64), new (u64) per event, plus the write-back of the
// changed columns (u64, one column per event slot).  Cases:
//   slot    one store per (event slot, array) across the wave, as k_tick emits (lanes ~2.4 apart)
//   pair    each thread's events two at a time (8-byte stores for the u32 arrays, 16-byte for the
//           u64 ones, at any dword), then the odd one
//   dense   the same bytes written lane = event (the floor for this volume)
//   wb      only the column write-backs
// Prints one JSON line per case (best and median us of 20 launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
constexpr int kTPB = 256, kSlots = 6;

struct Out {
    uint32_t* slot;
    uint32_t* pid;
    uint64_t* old_;
    uint64_t* new_;
    uint64_t* col[kSlots];
    const uint8_t* dm;  // per entity: its dirty event slots (bit j)
    int tcap;           // events per tile reserved
};

__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* s_w, uint32_t& tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    tot = 0;
    for (int i = 0; i < kTPB / 64; i++) {
        before += i < w ? s_w[i] : 0u;
        tot += s_w[i];
    }
    return before + inc - v;
}

template <int kMode>
__global__ __launch_bounds__(kTPB) void emit(Out o) {
    __shared__ uint32_t s_w[4];
    const uint32_t e = blockIdx.x * kTPB + threadIdx.x;
    const uint32_t dm = o.dm[e];
    uint64_t v[kSlots];
#pragma unroll
    for (int j = 0; j < kSlots; j++) v[j] = (uint64_t)e * 31 + j;
    uint32_t tot;
    const uint32_t nd = __builtin_popcount(dm);
    const uint32_t pev0 = block_excl(nd, s_w, tot);
    const size_t base = (size_t)blockIdx.x * o.tcap;
    uint32_t* ts = o.slot + base;
    uint32_t* tp = o.pid + base;
    uint64_t* to = o.old_ + base;
    uint64_t* tn = o.new_ + base;
    if (kMode == 0 || kMode == 3) {  // slot / wb
#pragma unroll
        for (int j = 0; j < kSlots; j++) {
            if (!((dm >> j) & 1)) continue;
            o.col[j][e] = v[j];
            if (kMode == 3) continue;
            const uint32_t at = pev0 + __builtin_popcount(dm & ((1u << j) - 1));
            ts[at] = e;
            tp[at] = (uint32_t)j;
            to[at] = v[j] ^ 1;
            tn[at] = v[j];
        }
    } else if (kMode == 1) {  // pair
        uint32_t p[kSlots];
        uint64_t a[kSlots];
        int n = 0;
#pragma unroll
        for (int j = 0; j < kSlots; j++)
            if ((dm >> j) & 1) {
                o.col[j][e] = v[j];
                p[n < kSlots ? n : 0] = j;
                a[n < kSlots ? n : 0] = v[j];
                n++;
            }
        for (int q = 0; q + 1 < n; q += 2) {
            *(u32x2_a4*)(ts + pev0 + q) = u32x2_a4{e, e};
            *(u32x2_a4*)(tp + pev0 + q) = u32x2_a4{p[q], p[q + 1]};
            *(u32x4_a4*)(to + pev0 + q) = u32x4_a4{(uint32_t)(a[q] ^ 1), (uint32_t)(a[q] >> 32), (uint32_t)(a[q + 1] ^ 1),
                                                   (uint32_t)(a[q + 1] >> 32)};
            *(u32x4_a4*)(tn + pev0 + q) =
                u32x4_a4{(uint32_t)a[q], (uint32_t)(a[q] >> 32), (uint32_t)a[q + 1], (uint32_t)(a[q + 1] >> 32)};
        }
        if (n & 1) {
            const int q = n - 1;
            ts[pev0 + q] = e;
            tp[pev0 + q] = p[q];
            to[pev0 + q] = a[q] ^ 1;
            tn[pev0 + q] = a[q];
        }
    } else {  // dense: lane = event over the tile's run
#pragma unroll
        for (int j = 0; j < kSlots; j++)
            if ((dm >> j) & 1) o.col[j][e] = v[j];
        for (uint32_t q = threadIdx.x; q < tot; q += kTPB) {
            ts[q] = e;
            tp[q] = q;
            to[q] = q ^ 1;
            tn[q] = q;
        }
    }
}

int main() {
    const int N = 1 << 20, T = N / kTPB, tcap = 6 * kTPB;
    std::vector<uint8_t> dm(N);
    uint32_t seed = 12345;
    size_t nev = 0;
    for (int i = 0; i < N; i++) {  // X, Y (slots 2, 3) always; HP (slot 0) 40 %
        seed = seed * 1664525u + 1013904223u;
        dm[i] = 0xC | (((seed >> 8) % 100) < 40 ? 1 : 0);
        nev += __builtin_popcount(dm[i]);
    }
    Out o;
    CK(hipMalloc(&o.slot, (size_t)T * tcap * 4));
    CK(hipMalloc(&o.pid, (size_t)T * tcap * 4));
    CK(hipMalloc(&o.old_, (size_t)T * tcap * 8));
    CK(hipMalloc(&o.new_, (size_t)T * tcap * 8));
    for (int j = 0; j < kSlots; j++) CK(hipMalloc(&o.col[j], (size_t)N * 8 + 2304));
    uint8_t* dmd;
    CK(hipMalloc(&dmd, N));
    CK(hipMemcpy(dmd, dm.data(), N, hipMemcpyHostToDevice));
    o.dm = dmd;
    o.tcap = tcap;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[4] = {"slot", "pair", "dense", "wb"};
    for (int m = 0; m < 4; m++) {
        std::vector<float> t;
        for (int it = 0; it < 22; it++) {
            CK(hipEventRecord(a));
            if (m == 0) emit<0><<<T, kTPB>>>(o);
            if (m == 1) emit<1><<<T, kTPB>>>(o);
            if (m == 2) emit<2><<<T, kTPB>>>(o);
            if (m == 3) emit<3><<<T, kTPB>>>(o);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it >= 2) t.push_back(ms * 1000);
        }
        std::sort(t.begin(), t.end());
        const double bytes = (m == 3 ? 0.0 : nev * 24.0) + nev * 8.0 + N;
        printf("{\"case\": \"%s\", \"events\": %zu, \"best_us\": %.1f, \"median_us\": %.1f, \"GBps_best\": %.0f}\n", names[m],
               nev, t[0], t[t.size() / 2], bytes / (t[0] * 1e3));
    }
    return 0;
}
