// Copy-kernel rate against launch size (not product code): does a copy of S bytes in + S bytes out
// reach the same HBM rate at 100 MB as at 6.4 GB?  Each size timed two ways: launches queued back to
// back (the GPU never idles), and one launch per host round trip with a short host gap between (the
// shape of a decode step).  Prints one JSON line per size.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/size_probe tools/size_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void __launch_bounds__(256) k_copy(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    for (; i + step < n16; i += 2 * step) {
        const uint4 a = in[i], b = in[i + step];
        out[i] = a;
        out[i + step] = b;
    }
    if (i < n16) out[i] = in[i];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t max_b = 6400ull << 20;
    void *in, *out;
    CK(hipMalloc(&in, max_b));
    CK(hipMalloc(&out, max_b));
    CK(hipMemset(in, 1, max_b));
    CK(hipMemset(out, 0, max_b));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t grid = cus * 8;
    for (uint64_t mb = 100; mb <= 6400; mb *= 2) {
        const uint64_t b = mb << 20, n16 = b / 16;
        // back to back
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n16);
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n16);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms_b2b = 0;
        CK(hipEventElapsedTime(&ms_b2b, e0, e1));
        ms_b2b /= reps;
        // one launch per round trip, 60 us host gap
        float best = 1e9, sum = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n16);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            sum += ms;
            if (ms < best) best = ms;
            std::this_thread::sleep_for(std::chrono::microseconds(60));
        }
        printf("{\"mb\": %llu, \"b2b_ms\": %.4f, \"b2b_tbs\": %.3f, \"gap_avg_ms\": %.4f, \"gap_tbs\": %.3f, "
               "\"gap_best_tbs\": %.3f}\n",
               (unsigned long long)mb, ms_b2b, 2.0 * b / ms_b2b / 1e9, sum / reps, 2.0 * b / (sum / reps) / 1e9,
               2.0 * b / best / 1e9);
        fflush(stdout);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
