// Random-access ceilings of the HBM for the aggregation table (one lane per record, its
// group row at a random place in a table far larger than the caches): lines read, lines
// read and written back, and device-scope atomics, per second.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mixr(uint64_t x) {
    x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull; return x ^ (x >> 33);
}

// MODE 0: read L lines of the row; 1: read + plain write of one dword per line; 2: A atomics (u64 add)
// on the row; 3: read the row's first line, then A atomics; 4: read L lines, write them back whole
// (16-byte stores over every byte); 5: write L lines whole, no read
template <int MODE>
__global__ __launch_bounds__(256) void k_probe(uint32_t *buf, uint64_t rows, uint32_t row_words, uint64_t n, int L, int A,
                                               uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = mixr(i * 0x9E3779B97F4A7C15ull + 1) % rows;
        uint32_t *R = buf + r * row_words;
        if (MODE == 0 || MODE == 1) {
            uint32_t v[4];
            for (int l = 0; l < L && l < 4; ++l) v[l] = R[l * 32];
            for (int l = 0; l < L && l < 4; ++l) acc += v[l];
            if (MODE == 1)
                for (int l = 0; l < L && l < 4; ++l) R[l * 32 + 1] = v[l] + 1;
        } else if (MODE == 4 || MODE == 5) {
            for (int l = 0; l < L && l < 2; ++l) {
                uint4 *q = (uint4 *)(R + l * 32);
                uint4 v[8];
                for (int j = 0; j < 8; ++j) v[j] = MODE == 4 ? q[j] : make_uint4(i, j, l, 1);
                for (int j = 0; j < 8; ++j) { v[j].x += 1; q[j] = v[j]; }
            }
        } else {
            if (MODE == 3) acc += R[0];
            for (int a = 0; a < A; ++a) atomicAdd((unsigned long long *)(R + 2 + 2 * a), 1ull);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Record-kernel shape: the row index comes from a per-record array (rec_g), the row's owner
// word is read and compared
__global__ __launch_bounds__(256) void k_owner(uint32_t *buf, uint64_t rows, uint32_t row_words, uint64_t n, int, int,
                                               uint32_t *sink) {
    const uint32_t *idx = sink + 64;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = idx[i];
        acc += buf[(uint64_t)r * row_words + 22] == (uint32_t)i;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_fill_idx(uint32_t *idx, uint64_t n, uint64_t rows) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        idx[i] = (uint32_t)(mixr(i * 0x9E3779B97F4A7C15ull + 7) % rows);
}

// Row-cooperative: 8 lanes per record, each a 16-byte piece of each of the row's L lines
// (one wave instruction touches 8 rows); W: write the pieces back
template <bool W>
__global__ __launch_bounds__(256) void k_coop(uint32_t *buf, uint64_t rows, uint32_t row_words, uint64_t n, int L, int,
                                              uint32_t *sink) {
    uint32_t acc = 0;
    const uint32_t piece = threadIdx.x & 7;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; i < n;
         i += ((uint64_t)gridDim.x * blockDim.x) >> 3) {
        const uint64_t r = mixr(i * 0x9E3779B97F4A7C15ull + 1) % rows;
        uint4 *q = (uint4 *)(buf + r * row_words) + piece;
        uint4 v[2];
        for (int l = 0; l < L && l < 2; ++l) v[l] = q[l * 8];
        for (int l = 0; l < L && l < 2; ++l) {
            acc += v[l].x;
            if (W) { v[l].y += 1; q[l * 8] = v[l]; }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t bytes = 40ull << 30;
    uint32_t *buf, *sink;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&sink, 64 * 4 + 100000000ull * 4));
    CHK(hipMemset(buf, 0, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const uint64_t n = 100000000;
    const uint32_t row_bytes = 256;
    const uint64_t rows = bytes / row_bytes;
    auto run = [&](const char *name, auto kern, int L, int A, int grid) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, rows, row_bytes / 4, n, L, A, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s L=%d A=%d grid=%7d  %8.2f ms  %6.2f ns/rec  %7.1f Mrec/s  lines %.2f G/s\n", name, L, A, grid, ms,
               ms * 1e6 / n, n / (ms * 1e3), (double)n * (L ? L : 1) / (ms * 1e6));
        fflush(stdout);
    };
    hipLaunchKernelGGL(k_fill_idx, dim3(4096), dim3(256), 0, 0, sink + 64, n, rows);
    for (int grid : {4096, 65536, 390625}) run("owner (idx array)", k_owner, 1, 0, grid);
    for (int grid : {65536}) {
        run("read", k_probe<0>, 1, 0, grid);
        run("read", k_probe<0>, 2, 0, grid);
        run("read+write", k_probe<1>, 1, 0, grid);
        run("read+write", k_probe<1>, 2, 0, grid);
        run("atomics", k_probe<2>, 0, 1, grid);
        run("atomics", k_probe<2>, 0, 2, grid);
        run("atomics", k_probe<2>, 0, 7, grid);
        run("read+atomics", k_probe<3>, 1, 7, grid);
        run("read+write whole lines", k_probe<4>, 1, 0, grid);
        run("read+write whole lines", k_probe<4>, 2, 0, grid);
        run("write whole lines", k_probe<5>, 1, 0, grid);
        run("write whole lines", k_probe<5>, 2, 0, grid);
        run("coop read", k_coop<false>, 1, 0, grid);
        run("coop read", k_coop<false>, 2, 0, grid);
        run("coop read+write", k_coop<true>, 1, 0, grid);
        run("coop read+write", k_coop<true>, 2, 0, grid);
    }
    return 0;
}
