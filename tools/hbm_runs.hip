// Write-bandwidth probe for k_tick's fan-out pattern (measurement tool, not on the product path).
// k_tick's fused fan-out has every workgroup write its tile's recipient run (tens of KB) into its
// own fixed-stride region of the message buffer while ~2000 other workgroups do the same.  This
// probe times that pattern against a grid-stride stream of the same bytes:
//   stream      persistent grid-stride 16-byte stores over one contiguous buffer
//   runs R/S    one workgroup per run: run w of R bytes at w * S, 256 threads x 16-byte stores
//               (S = R: the runs are adjacent; S > R: fixed-stride regions as in k_tick)
//   +4          the same runs starting 4 bytes into their region (k_tick's runs start at any dword)
// Prints one JSON line per case (best and median GB/s of 10 launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                 \
            return 1;                                                                               \
        }                                                                                           \
    } while (0)

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

__global__ __launch_bounds__(256) void stream_write(uint4* __restrict__ p, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// run blockIdx.x: [base + blockIdx.x * S, + R) in 16-byte stores at a dword-aligned start
__global__ __launch_bounds__(256) void runs_write(uint32_t* __restrict__ base, size_t S, size_t R, uint32_t off) {
    uint32_t* run = base + (size_t)blockIdx.x * (S / 4) + off;
    const size_t n16 = R / 16;
    for (size_t i = threadIdx.x; i < n16; i += 256)
        *(u32x4_a4*)(run + 4 * i) = u32x4_a4{(uint32_t)i, blockIdx.x, 2u, 3u};
}

static void report(const char* name, size_t bytes, std::vector<float>& ms) {
    std::sort(ms.begin(), ms.end());
    printf("{\"case\": \"%s\", \"bytes\": %zu, \"best_GBps\": %.0f, \"median_GBps\": %.0f}\n", name, bytes,
           bytes / (ms[0] * 1e-3) / 1e9, bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const size_t total = (size_t)768 << 20;  // bytes written per launch (config[3]: ~0.74 GB)
    const size_t maxS = (size_t)448 << 10;
    const size_t cap = std::max(total, (total / (16 << 10)) * maxS) + 4096;  // room for the widest case
    uint32_t* buf = nullptr;
    CK(hipMalloc(&buf, cap));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        std::vector<float> ms;
        launch();
        (void)hipDeviceSynchronize();
        for (int r = 0; r < 10; r++) {
            (void)hipEventRecord(a);
            launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float t = 0;
            (void)hipEventElapsedTime(&t, a, b);
            ms.push_back(t);
        }
        return ms;
    };
    {
        auto ms = timeit([&] { hipLaunchKernelGGL(stream_write, dim3(cus * 8), dim3(256), 0, 0, (uint4*)buf, total / 16); });
        report("stream", total, ms);
    }
    const size_t Rs[] = {(size_t)16 << 10, (size_t)64 << 10};
    const size_t Ss[] = {0, (size_t)128 << 10, (size_t)426 << 10};  // 0: S = R
    for (size_t R : Rs)
        for (size_t S0 : Ss)
            for (uint32_t off : {0u, 1u}) {
                const size_t S = S0 ? S0 : R + (off ? 64 : 0);
                const unsigned g = (unsigned)(total / R);
                if ((size_t)g * S + R + 16 > cap) continue;
                auto ms = timeit([&] { hipLaunchKernelGGL(runs_write, dim3(g), dim3(256), 0, 0, buf, S, R, off); });
                char nm[96];
                snprintf(nm, sizeof nm, "runs R=%zuK S=%zuK%s", R >> 10, S >> 10, off ? " +4" : "");
                report(nm, (size_t)g * R, ms);
            }
    CK(hipFree(buf));
    return 0;
}
