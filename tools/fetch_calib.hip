// Round 6: calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE for the aggregation's access
// shapes on a known byte count.  MI355X_MICROARCH.md calibrates the gfx950 FETCH_SIZE x2 correction
// only for wide coalesced streaming reads; the 5-tuple's owner kernel reads and writes 256-byte rows
// at random places, eight lanes per row, 16 bytes each.  Each kernel below is one dispatch (run under
// separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes); the known bytes are printed:
//   stream_read    n16 x 16 B coalesced loads                      (the guide's calibrated case)
//   rand_line      N rows, 8 lanes read one 128-B line             (N x 128 B)
//   rand_row       N rows, 8 lanes read a 256-B row (two lines)    (N x 256 B)
//   rand_row_rw    N rows, 8 lanes read a 256-B row and write it   (N x 256 B each way)
//   rand_dword     N rows, one lane reads one dword of its line    (N x 128 B if whole lines move)
// Table: 8 GiB (far past the 256 MB MALL), N = 10^7 random rows.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mixr(uint64_t x) {
    x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull; return x ^ (x >> 33);
}

__global__ __launch_bounds__(256) void stream_read(const uint4 *buf, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// 8 lanes per row, piece = lane & 7; L lines (128 B each); W: write the pieces back
template <int L, bool W>
__global__ __launch_bounds__(256) void rand_rows(uint4 *buf, uint64_t rows, uint64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    const uint32_t piece = threadIdx.x & 7;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; i < n;
         i += ((uint64_t)gridDim.x * blockDim.x) >> 3) {
        const uint64_t r = mixr(i * 0x9E3779B97F4A7C15ull + 1) % rows;
        uint4 *q = buf + r * 16 + piece;  // rows of 256 B = 16 pieces
        uint4 v[L];
#pragma unroll
        for (int l = 0; l < L; ++l) v[l] = q[l * 8];
#pragma unroll
        for (int l = 0; l < L; ++l) {
            acc += v[l].x;
            if (W) {
                v[l].y += 1;
                q[l * 8] = v[l];
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void rand_dword(const uint32_t *buf, uint64_t rows, uint64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = mixr(i * 0x9E3779B97F4A7C15ull + 1) % rows;
        acc += buf[r * 64];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t bytes = 8ull << 30, rows = bytes / 256, n = 10000000, n16 = (1ull << 30) / 16;
    uint4 *buf;
    uint32_t *sink;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(buf, 0, bytes));
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto timed = [&](const char *name, double rd, double wr, auto launch) {
        CHK(hipEventRecord(e0));
        launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-12s known_read_bytes %.6e known_write_bytes %.6e  %.3f ms\n", name, rd, wr, ms);
        fflush(stdout);
        return 0;
    };
    const dim3 g(65536), b(256);
    timed("stream_read", (double)n16 * 16, 0, [&] { hipLaunchKernelGGL(stream_read, g, b, 0, 0, buf, n16, sink); });
    timed("rand_line", (double)n * 128, 0, [&] { hipLaunchKernelGGL((rand_rows<1, false>), g, b, 0, 0, buf, rows, n, sink); });
    timed("rand_row", (double)n * 256, 0, [&] { hipLaunchKernelGGL((rand_rows<2, false>), g, b, 0, 0, buf, rows, n, sink); });
    timed("rand_row_rw", (double)n * 256, (double)n * 256,
          [&] { hipLaunchKernelGGL((rand_rows<2, true>), g, b, 0, 0, buf, rows, n, sink); });
    timed("rand_dword", (double)n * 128, 0,
          [&] { hipLaunchKernelGGL(rand_dword, g, b, 0, 0, (const uint32_t *)buf, rows, n, sink); });
    CHK(hipFree(buf));
    CHK(hipFree(sink));
    return 0;
}
