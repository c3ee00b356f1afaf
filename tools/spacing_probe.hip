// Column-spacing probe (not product code): the T20 decode's memory pattern without the parsing --
// 1024-row windows of 64-byte records read into LDS, written back as 20 column pieces at
// column_base(c) = cap * offset(c) -- timed against the column stride `cap`, to see how the rate of
// the same traffic depends on where the column streams sit relative to each other.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/spacing_probe tools/spacing_probe.hip
// usage: tools/spacing_probe ROWS PAD0 PAD1 STEP [reps]   (pads in 1024-row windows; one JSON line each)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int NC = 20;
__constant__ int kW[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
__constant__ int kOff[NC];  // byte offset of each column inside a record = its column offset (row-bytes units)

constexpr int ROWS = 1024, REC = 64;

__global__ void __launch_bounds__(256) k_window(const uint4 *__restrict__ in, uint8_t *__restrict__ out, uint64_t cap,
                                                uint32_t nwin) {
    __shared__ uint4 lds[ROWS * REC / 16];  // 64 KiB
    const uint32_t G = gridDim.x, X = 8, x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X, start = x * per, end = min(nwin, start + per);
    for (uint32_t W = start + l; W < end; W += G / X) {
        const uint4 *src = in + (uint64_t)W * (ROWS * REC / 16);
#pragma unroll 4
        for (int i = threadIdx.x; i < ROWS * REC / 16; i += 256) lds[i] = src[i];
        __syncthreads();
        // column c of the window: 1024 * w bytes, 16 bytes per thread store (the content is LDS data,
        // not the transposed column: only the memory pattern matters here)
        for (int c = 0; c < NC; ++c) {
            const int w = kW[c], o = kOff[c];
            uint4 *dst = (uint4 *)(out + cap * o + (uint64_t)W * ROWS * w);
            const int pieces = ROWS * w / 16;
            for (int p = threadIdx.x; p < pieces; p += 256) dst[p] = lds[(c * 64 + p) & (ROWS * REC / 16 - 1)];
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s ROWS PAD0 PAD1 STEP [reps]\n", argv[0]);
        return 1;
    }
    const uint64_t rows = strtoull(argv[1], 0, 10);
    const long pad0 = atol(argv[2]), pad1 = atol(argv[3]), step = atol(argv[4]);
    const int reps = argc > 5 ? atoi(argv[5]) : 5;
    const uint32_t nwin = (uint32_t)((rows + ROWS - 1) / ROWS);
    int off[NC], acc = 0, W[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
    for (int c = 0; c < NC; ++c) {
        off[c] = acc;
        acc += W[c];
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(kOff), off, sizeof off));
    const uint64_t in_b = (uint64_t)nwin * ROWS * REC;
    const uint64_t cap_max = ((uint64_t)nwin + pad1) * ROWS;
    void *in, *out;
    CK(hipMalloc(&in, in_b));
    CK(hipMalloc(&out, cap_max * REC + 4096));
    CK(hipMemset(in, 3, in_b));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t grid = cus * 8;
    for (long pad = pad0; pad <= pad1; pad += step) {
        const uint64_t cap = ((uint64_t)nwin + pad) * ROWS;
        hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint8_t *)out, cap, nwin);
        float best = 1e9, sum = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint8_t *)out, cap, nwin);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            sum += ms;
            if (ms < best) best = ms;
        }
        printf("{\"rows\": %llu, \"pad\": %ld, \"cap\": %llu, \"ms\": %.4f, \"best_ms\": %.4f, \"tbs\": %.3f}\n",
               (unsigned long long)rows, pad, (unsigned long long)cap, sum / reps, best,
               2.0 * nwin * ROWS * REC / (sum / reps) / 1e9);
        fflush(stdout);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
