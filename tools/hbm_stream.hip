// hbm_stream.hip — a tuned HBM streaming probe: how close to the 8 TB/s spec a read / write / copy
// / k_tick-shaped read+write mix gets on this box, so k_tick's roofline fraction can be read
// against a measured ceiling.  Every footprint is >= 1 GiB (4x the 256 MiB Infinity Cache), each
// array is streamed once per launch, 16 B per lane, every line used whole.  Variants:
//   oneshot     one thread per 16-B element (the shape k_tick has: one thread per entity slot)
//   persist     a persistent grid (CUs x waves-per-CU workgroups) striding over the arrays, 4
//               elements in flight per thread
//   +nt         non-temporal stores (__builtin_nontemporal_store) / loads
// The guide's reference point is 6.29 TB/s for a float4 copy (MI355X_MICROARCH.md:36).
//
//   hbm_stream      one JSON line per case: streams, bytes per launch, best / median us, TB/s
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int kMaxArr = 24;
struct Arrs {
    uint4* a[kMaxArr];
};

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
    if constexpr (NT) {
        uint4 v;
        v.x = __builtin_nontemporal_load(&p->x);
        v.y = __builtin_nontemporal_load(&p->y);
        v.z = __builtin_nontemporal_load(&p->z);
        v.w = __builtin_nontemporal_load(&p->w);
        return v;
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void st(uint4* p, uint4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}

// one thread per element: R loads then W stores
template <int R, int W, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void oneshot(Arrs s, size_t n, uint32_t* __restrict__ sink) {
    const size_t e = blockIdx.x * 256ull + threadIdx.x;
    if (e >= n) return;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < R; i++) {
        const uint4 v = ld<NTL>(s.a[i] + e);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
#pragma unroll
    for (int i = 0; i < W; i++) st<NTS>(s.a[R + i] + e, make_uint4(acc + i, (uint32_t)e, 0u, 1u));
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// persistent grid-stride: each thread keeps U elements in flight per array
template <int R, int W, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void persist(Arrs s, size_t n, uint32_t* __restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    uint32_t acc = 0;
    for (size_t base = blockIdx.x * 256ull * U + threadIdx.x; base < n; base += stride) {
        uint32_t a[U];
#pragma unroll
        for (int u = 0; u < U; u++) a[u] = 0;
#pragma unroll
        for (int i = 0; i < R; i++) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const size_t e = base + (size_t)u * 256;
                v[u] = e < n ? ld<NTL>(s.a[i] + e) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; u++) a[u] ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
#pragma unroll
        for (int i = 0; i < W; i++)
#pragma unroll
            for (int u = 0; u < U; u++) {
                const size_t e = base + (size_t)u * 256;
                if (e < n) st<NTS>(s.a[R + i] + e, make_uint4(a[u] + i, (uint32_t)e, 0u, 1u));
            }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= a[u];
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <typename K>
int timeit(K launch, double bytes, const char* name, int R, int W, size_t n, int grid) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    std::vector<float> t;
    for (int rep = 0; rep < 10; rep++) {
        CHK(hipEventRecord(a));
        launch();
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) t.push_back(ms);
    }
    CHK(hipGetLastError());
    std::sort(t.begin(), t.end());
    printf("{\"case\": \"%s\", \"read_arrays\": %d, \"write_arrays\": %d, \"elems\": %zu, \"grid\": %d, "
           "\"bytes_per_launch\": %.0f, \"best_us\": %.1f, \"median_us\": %.1f, \"TBps_best\": %.3f, \"TBps_median\": %.3f}\n",
           name, R, W, n, grid, bytes, 1000.0 * t.front(), 1000.0 * t[t.size() / 2], bytes / (t.front() * 1e-3) / 1e12,
           bytes / (t[t.size() / 2] * 1e-3) / 1e12);
    fflush(stdout);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

template <int R, int W>
int cases(const Arrs& s, uint32_t* sink, int cus, const char* tag) {
    // >= 1 GiB per launch over all arrays, >= 64 MiB per array
    const size_t n = std::max<size_t>((1ull << 30) / (16ull * (R + W)), (64ull << 20) / 16);
    const double bytes = 16.0 * (R + W) * (double)n;
    char nm[96];
    int r = 0;
    const int g1 = (int)((n + 255) / 256);
    snprintf(nm, sizeof nm, "%s/oneshot", tag);
    r |= timeit([&] { oneshot<R, W, false, false><<<g1, 256>>>(s, n, sink); }, bytes, nm, R, W, n, g1);
    snprintf(nm, sizeof nm, "%s/oneshot+ntstore", tag);
    r |= timeit([&] { oneshot<R, W, false, true><<<g1, 256>>>(s, n, sink); }, bytes, nm, R, W, n, g1);
    for (int wpc : {4, 8, 16}) {  // 256-thread workgroups per CU
        const int g = cus * wpc / 4;
        snprintf(nm, sizeof nm, "%s/persist%d", tag, wpc);
        r |= timeit([&] { persist<R, W, 4, false, false><<<g, 256>>>(s, n, sink); }, bytes, nm, R, W, n, g);
        snprintf(nm, sizeof nm, "%s/persist%d+ntstore", tag, wpc);
        r |= timeit([&] { persist<R, W, 4, false, true><<<g, 256>>>(s, n, sink); }, bytes, nm, R, W, n, g);
        snprintf(nm, sizeof nm, "%s/persist%d+nt", tag, wpc);
        r |= timeit([&] { persist<R, W, 4, true, true><<<g, 256>>>(s, n, sink); }, bytes, nm, R, W, n, g);
    }
    return r;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    // arrays sized for the largest per-array footprint (read_only / write_only / copy: 1 GiB over
    // 1 or 2 arrays)
    Arrs s;
    const size_t cap = 1ull << 30;
    for (int i = 0; i < kMaxArr; i++) {
        const size_t bytes = i < 2 ? cap : (256ull << 20);
        CHK(hipMalloc(&s.a[i], bytes + 4096));
        CHK(hipMemset(s.a[i], i + 1, bytes));
    }
    uint32_t* sink;
    CHK(hipMalloc(&sink, 64));
    printf("{\"device\": \"%s\", \"cus\": %d}\n", p.name, cus);
    int r = 0;
    r |= cases<1, 0>(s, sink, cus, "read_only");
    r |= cases<0, 1>(s, sink, cus, "write_only");
    r |= cases<1, 1>(s, sink, cus, "copy_1_1");
    r |= cases<10, 13>(s, sink, cus, "mix_10_13_ktick");
    r |= cases<4, 9>(s, sink, cus, "mix_4_9_krecords");
    CHK(hipDeviceSynchronize());
    return r;
}
