// HBM placement map (not product code): allocate N chunks of S MiB one after the other (the VRAM
// allocator hands them out in address order, mostly) and time, per chunk, a read-only pass, a
// write-only pass and the decode's pattern (1024-row windows of 64-byte records read from the first
// half, 20 column streams written to the second half) -- do some allocations run slower than others,
// and is it the memory or the access pattern?
// build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_map_probe tools/hbm_map_probe.hip
// usage: tools/hbm_map_probe [chunks 128] [MiB 512]     one JSON line per chunk
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int NC = 20, ROWS = 1024, REC = 64;
__constant__ int kW[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
__constant__ int kOff[NC] = {0, 4, 8, 12, 16, 20, 28, 36, 40, 44, 46, 48, 50, 51, 52, 53, 54, 58, 62, 63};

__global__ void __launch_bounds__(256) k_read(const uint4 *__restrict__ in, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_write(uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void __launch_bounds__(256) k_window(const uint4 *__restrict__ in, uint8_t *__restrict__ out, uint64_t cap,
                                                uint32_t nwin) {
    __shared__ uint4 lds[ROWS * REC / 16];
    const uint32_t G = gridDim.x, X = 8, x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X, start = x * per, end = min(nwin, start + per);
    for (uint32_t W = start + l; W < end; W += G / X) {
        const uint4 *src = in + (uint64_t)W * (ROWS * REC / 16);
        for (int i = threadIdx.x; i < ROWS * REC / 16; i += 256) lds[i] = src[i];
        __syncthreads();
        for (int c = 0; c < NC; ++c) {
            const int w = kW[c], o = kOff[c];
            uint4 *dst = (uint4 *)(out + cap * o + (uint64_t)W * ROWS * w);
            for (int p = threadIdx.x; p < ROWS * w / 16; p += 256) dst[p] = lds[(c * 64 + p) & (ROWS * REC / 16 - 1)];
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int chunks = argc > 1 ? atoi(argv[1]) : 128;
    const uint64_t bytes = (uint64_t)(argc > 2 ? atoi(argv[2]) : 512) << 20;
    std::vector<void *> p(chunks);
    for (int i = 0; i < chunks; ++i) CK(hipMalloc(&p[i], bytes));
    uint32_t *sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t grid = cus * 8;
    const uint64_t n16 = bytes / 16;
    const uint32_t nwin = (uint32_t)(bytes / 2 / (ROWS * REC));
    const uint64_t cap = (uint64_t)nwin * ROWS;
    auto timed = [&](auto fn) {
        fn();
        float best = 1e9;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, 0));
            fn();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        return best;
    };
    for (int i = 0; i < chunks; ++i) {
        uint8_t *c = (uint8_t *)p[i];
        const float tr = timed([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const uint4 *)c, n16, sink); });
        const float tw = timed([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (uint4 *)c, n16); });
        const float td = timed([&] {
            hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)c, c + bytes / 2, cap, nwin);
        });
        printf("{\"chunk\": %d, \"va\": \"%p\", \"read_tbs\": %.3f, \"write_tbs\": %.3f, \"window_tbs\": %.3f}\n", i,
               (void *)c, bytes / tr / 1e9, bytes / tw / 1e9, bytes / td / 1e9);
        fflush(stdout);
    }
    for (int i = 0; i < chunks; ++i) CK(hipFree(p[i]));
    return 0;
}
