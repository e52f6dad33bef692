// hbm_mix.hip — what HBM bandwidth a read/write MIX of many concurrent streams reaches on this
// box, for reading k_tick's roofline fraction against something achievable rather than the 8 TB/s
// spec.  Every kernel is the ideal form of such a mix: one thread per entity slot (256-slot
// workgroups, as k_tick; 2M slots), each thread reading R and writing W separate
// arrays of 16 B per slot (fully coalesced, every line used whole), all arrays far beyond the
// 256 MiB Infinity Cache.  k_tick's real traffic per launch is 175 MB read + 226 MB written
// (profiles/r02u_pmc.json): R:W = 10:13 is that ratio.
//
//   hbm_mix            one JSON line per kernel: streams, bytes per launch, best/median us, TB/s
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

constexpr int kMaxArr = 32;
struct Arrs {
    uint4* a[kMaxArr];  // array i holds n slots of 16 B
};

// R arrays read, W arrays written, one 16-byte value per slot each; all loads issued before any
// store (as k_tick issues its schedule records together)
template <int R, int W>
__global__ __launch_bounds__(256) void mix(Arrs s, size_t n, uint32_t* __restrict__ sink) {
    const size_t e = blockIdx.x * 256ull + threadIdx.x;
    if (e >= n) return;
    uint32_t acc = 0;
    uint4 v[R > 0 ? R : 1];
#pragma unroll
    for (int i = 0; i < R; i++) v[i] = s.a[i][e];
#pragma unroll
    for (int i = 0; i < R; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
#pragma unroll
    for (int i = 0; i < W; i++) s.a[R + i][e] = make_uint4(acc + i, (uint32_t)e, 0u, 1u);
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads live
}

template <int R, int W>
int run(const Arrs& s, size_t n, uint32_t* sink, const char* name) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    std::vector<float> t;
    for (int rep = 0; rep < 12; rep++) {
        CHK(hipEventRecord(a));
        mix<R, W><<<grid, block>>>(s, n, sink);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double bytes = 16.0 * (R + W) * (double)n;
    printf("{\"kernel\": \"%s\", \"read_arrays\": %d, \"write_arrays\": %d, \"slots\": %zu, \"bytes_per_launch\": %.0f, "
           "\"best_us\": %.2f, \"median_us\": %.2f, \"TBps_best\": %.3f, \"TBps_median\": %.3f}\n",
           name, R, W, n, bytes, 1000.0 * t.front(), 1000.0 * t[t.size() / 2], bytes / (t.front() * 1e-3) / 1e12,
           bytes / (t[t.size() / 2] * 1e-3) / 1e12);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

int main() {
    const size_t n = 1ull << 21;  // 2M slots: each array 32 MiB, 23 arrays 736 MiB (> Infinity Cache)
    Arrs s;
    for (int i = 0; i < kMaxArr; i++) {
        CHK(hipMalloc(&s.a[i], n * 16 + 4096));
        CHK(hipMemset(s.a[i], i + 1, n * 16));
    }
    uint32_t* sink;
    CHK(hipMalloc(&sink, 64));
    int r = 0;
    r |= run<23, 0>(s, n, sink, "read_only");
    r |= run<0, 23>(s, n, sink, "write_only");
    r |= run<1, 1>(s, n, sink, "copy_1_1");
    r |= run<12, 11>(s, n, sink, "mix_12_11");
    r |= run<10, 13>(s, n, sink, "mix_10_13_ktick_ratio");
    r |= run<5, 5>(s, n, sink, "mix_5_5");
    r |= run<4, 9>(s, n, sink, "mix_4_9_krecords_ratio");
    CHK(hipDeviceSynchronize());
    return r;
}
