// Output-layout probe (not product code): is the decode's bimodal rate a
// property of the column-major (SoA) layout's ~170 concurrent write streams, or of the memory?
// The T20 decode's memory pattern without the parsing -- 1024-row windows of 64-byte records
// read into LDS (64 KiB) and written back as 20 column pieces -- in two output layouts:
//   soa   column c of the whole batch at out + cap * off(c)   (the product layout: each workgroup
//         writes 20 pieces, each XCD advances 20 column regions at once)
//   tile  row-group tiles of T rows: tile t at out + t * T * 64, column c of the tile at
//         + T * off(c)  (a window writes one contiguous span; an XCD advances one region)
// Each trial allocates fresh input and output buffers (new physical pages; the previous pair is
// freed only after the next is allocated), so the trials sample the placement lottery.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/tile_probe tools/tile_probe.hip
// usage: tools/tile_probe ROWS TRIALS [tile_rows ...]    one JSON line per (trial, layout)
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

constexpr int NC = 20;
__constant__ int kW[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
__constant__ int kOff[NC];

constexpr int ROWS = 1024, REC = 64;

// tile_rows == 0: SoA with column stride cap; else tiles of tile_rows rows (a multiple of 1024)
__global__ void __launch_bounds__(256) k_window(const uint4 *__restrict__ in, uint8_t *__restrict__ out, uint64_t cap,
                                                uint32_t nwin, uint32_t tile_rows) {
    __shared__ uint4 lds[ROWS * REC / 16];  // 64 KiB
    const uint32_t G = gridDim.x, X = 8, x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X, start = x * per, end = min(nwin, start + per);
    for (uint32_t W = start + l; W < end; W += G / X) {
        const uint4 *src = in + (uint64_t)W * (ROWS * REC / 16);
#pragma unroll 4
        for (int i = threadIdx.x; i < ROWS * REC / 16; i += 256) lds[i] = src[i];
        __syncthreads();
        const uint64_t row0 = (uint64_t)W * ROWS;
        for (int c = 0; c < NC; ++c) {
            const int w = kW[c], o = kOff[c];
            uint8_t *base;
            if (tile_rows) {
                const uint64_t t = row0 / tile_rows, r = row0 % tile_rows;
                base = out + t * (uint64_t)tile_rows * REC + (uint64_t)tile_rows * o + r * w;
            } else {
                base = out + cap * o + row0 * w;
            }
            uint4 *dst = (uint4 *)base;
            const int pieces = ROWS * w / 16;
            for (int p = threadIdx.x; p < pieces; p += 256) dst[p] = lds[(c * 64 + p) & (ROWS * REC / 16 - 1)];
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s ROWS TRIALS [tile_rows ...]\n", argv[0]);
        return 1;
    }
    const uint64_t rows = strtoull(argv[1], 0, 10);
    const int trials = atoi(argv[2]);
    std::vector<uint32_t> layouts{0};
    for (int i = 3; i < argc; ++i) layouts.push_back((uint32_t)atoi(argv[i]));
    const uint32_t nwin = (uint32_t)((rows + ROWS - 1) / ROWS);
    int off[NC], acc = 0, Wd[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
    for (int c = 0; c < NC; ++c) {
        off[c] = acc;
        acc += Wd[c];
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(kOff), off, sizeof off));
    const uint64_t in_b = (uint64_t)nwin * ROWS * REC, out_b = (uint64_t)nwin * ROWS * REC + (1 << 20);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t grid = cus * 8;
    void *prev_in = nullptr, *prev_out = nullptr;
    for (int t = 0; t < trials; ++t) {
        void *in, *out;
        CK(hipMalloc(&in, in_b));
        CK(hipMalloc(&out, out_b));
        if (prev_in) CK(hipFree(prev_in));
        if (prev_out) CK(hipFree(prev_out));
        prev_in = in;
        prev_out = out;
        CK(hipMemset(in, 3, in_b));
        CK(hipMemset(out, 0, out_b));
        for (uint32_t tile : layouts) {
            const uint64_t cap = (uint64_t)nwin * ROWS;
            hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint8_t *)out, cap, nwin, tile);
            float sum = 0, best = 1e9;
            const int reps = 5;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, (uint8_t *)out, cap, nwin,
                                   tile);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                sum += ms;
                best = ms < best ? ms : best;
            }
            printf("{\"trial\": %d, \"layout\": \"%s\", \"tile_rows\": %u, \"rows\": %llu, \"ms\": %.4f, "
                   "\"best_ms\": %.4f, \"tbs\": %.3f}\n",
                   t, tile ? "tile" : "soa", tile, (unsigned long long)rows, sum / reps, best,
                   2.0 * nwin * ROWS * REC / (sum / reps) / 1e9);
            fflush(stdout);
        }
    }
    CK(hipFree(prev_in));
    CK(hipFree(prev_out));
    return 0;
}
