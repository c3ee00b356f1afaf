// HBM ceiling probe for the T20 decode shape (not product code): how fast can
// MI355X move 10^8 x 64-byte records in and 63 bytes/record of columns out
// under different access shapes.  Build: hipcc -O3 --offload-arch=gfx950
// tools/hbm_probe.hip -o /tmp/hbm_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr uint64_t N = 100000000ull;  // records
__constant__ int kW[20] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 1, 1, 1, 1, 1, 4, 4, 1, 1};

__global__ void __launch_bounds__(256) k_copy16(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}

__global__ void __launch_bounds__(256) k_copy16_nt(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        uint4 v;
        v.x = __builtin_nontemporal_load(&in[i].x);
        v.y = __builtin_nontemporal_load(&in[i].y);
        v.z = __builtin_nontemporal_load(&in[i].z);
        v.w = __builtin_nontemporal_load(&in[i].w);
        __builtin_nontemporal_store(v.x, &out[i].x);
        __builtin_nontemporal_store(v.y, &out[i].y);
        __builtin_nontemporal_store(v.z, &out[i].z);
        __builtin_nontemporal_store(v.w, &out[i].w);
    }
}

__global__ void __launch_bounds__(256) k_copy16_ntst(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = in[i];
        __builtin_nontemporal_store(v.x, &out[i].x);
        __builtin_nontemporal_store(v.y, &out[i].y);
        __builtin_nontemporal_store(v.z, &out[i].z);
        __builtin_nontemporal_store(v.w, &out[i].w);
    }
}

__global__ void __launch_bounds__(256) k_write16(uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void __launch_bounds__(256) k_read16(const uint4 *__restrict__ in, uint32_t *__restrict__ out, uint64_t n16) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// one record per lane: 4 x 16-byte loads at a 64-byte lane stride
__global__ void __launch_bounds__(256) k_rec_read(const uint4 *__restrict__ in, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t r = blockIdx.x * 256ull + threadIdx.x; r < N; r += (uint64_t)gridDim.x * 256) {
        const uint4 *p = in + 4 * r;
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc ^= a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ d.x;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// one record per lane, T20-shaped column stores (20 columns, 63 B/record)
template <bool NARROW, bool NT = false>
__global__ void __launch_bounds__(256) k_rec_cols(const uint4 *__restrict__ in, uint8_t *__restrict__ cols) {
    for (uint64_t r = blockIdx.x * 256ull + threadIdx.x; r < N; r += (uint64_t)gridDim.x * 256) {
        const uint4 *p = in + 4 * r;
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        const uint32_t w[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
        uint64_t coff = 0;
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            const uint32_t v = w[f % 16] ^ (uint32_t)f;
            const int wd = NARROW ? kW[f] : 4;
            uint8_t *col = cols + coff;
            if (NT) {
                if (wd == 1) __builtin_nontemporal_store((uint8_t)v, &col[r]);
                else if (wd == 2) __builtin_nontemporal_store((uint16_t)v, &((uint16_t *)col)[r]);
                else if (wd == 4) __builtin_nontemporal_store(v, &((uint32_t *)col)[r]);
                else __builtin_nontemporal_store(((uint64_t)w[(f + 1) % 16] << 32) | v, &((uint64_t *)col)[r]);
            } else if (wd == 1) col[r] = (uint8_t)v;
            else if (wd == 2) ((uint16_t *)col)[r] = (uint16_t)v;
            else if (wd == 4) ((uint32_t *)col)[r] = v;
            else ((uint2 *)col)[r] = make_uint2(v, w[(f + 1) % 16]);
            coff += (uint64_t)wd * N;
            if (!NARROW && f == 15) break;  // 16 x 4 B = 64 B/record
        }
    }
}

// coalesced 16-byte loads, then T20-shaped column stores from them (4 lanes per record)
__global__ void __launch_bounds__(256) k_coal_cols(const uint4 *__restrict__ in, uint8_t *__restrict__ cols) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < 4 * N; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = in[i];
        const uint64_t r = i >> 2;
        const int q = i & 3;  // quarter of the record this lane holds: 5 columns each
        uint64_t coff = 0;
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            const int wd = kW[f];
            if (f / 5 == q) {
                uint8_t *col = cols + coff;
                const uint32_t x = (f & 1) ? v.x : v.y;
                if (wd == 1) col[r] = (uint8_t)x;
                else if (wd == 2) ((uint16_t *)col)[r] = (uint16_t)x;
                else if (wd == 4) ((uint32_t *)col)[r] = x;
                else ((uint2 *)col)[r] = make_uint2(x, v.z);
            }
            coff += (uint64_t)wd * N;
        }
    }
}

template <class F>
float timeit(F &&f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < 10; ++i) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t in_b = 64 * N, out_b = 64 * N;
    uint4 *in;
    uint8_t *out;
    uint32_t *sink;
    CK(hipMalloc(&in, in_b));
    CK(hipMalloc(&out, out_b + 4096));
    CK(hipMalloc(&sink, 4u << 20));
    CK(hipMemset(in, 0x5A, in_b));
    for (int g : {cus * 2, cus * 4, cus * 8}) {
        const float w = timeit([&] { k_write16<<<g, 256>>>((uint4 *)out, in_b / 16); });
        const float cnt = timeit([&] { k_copy16_nt<<<g, 256>>>(in, (uint4 *)out, in_b / 16); });
        const float cst = timeit([&] { k_copy16_ntst<<<g, 256>>>(in, (uint4 *)out, in_b / 16); });
        const float cn2 = timeit([&] { k_rec_cols<true, true><<<g, 256>>>(in, out); });
        printf("grid %5d | write16 %.3f ms %.0f GB/s | copy16_nt %.3f ms %.0f GB/s | copy16_ntstore %.3f ms %.0f GB/s | "
               "rec_cols(T20, nt stores) %.3f ms %.0f GB/s\n",
               g, w, in_b / w / 1e6, cnt, 2 * in_b / cnt / 1e6, cst, 2 * in_b / cst / 1e6, cn2, (in_b + 63 * N) / cn2 / 1e6);
        const float c = timeit([&] { k_copy16<<<g, 256>>>(in, (uint4 *)out, in_b / 16); });
        const float r = timeit([&] { k_read16<<<g, 256>>>(in, sink, in_b / 16); });
        const float rr = timeit([&] { k_rec_read<<<g, 256>>>(in, sink); });
        const float cn = timeit([&] { k_rec_cols<true><<<g, 256>>>(in, out); });
        const float cw = timeit([&] { k_rec_cols<false><<<g, 256>>>(in, out); });
        const float cc = timeit([&] { k_coal_cols<<<g, 256>>>(in, out); });
        printf("grid %5d | copy16 %.3f ms %.0f GB/s | read16 %.3f ms %.0f GB/s | rec_read %.3f ms %.0f GB/s | "
               "rec_cols(T20) %.3f ms %.0f GB/s | rec_cols(16xu32) %.3f ms %.0f GB/s | coal_cols(T20) %.3f ms %.0f GB/s\n",
               g, c, 2 * in_b / c / 1e6, r, in_b / r / 1e6, rr, in_b / rr / 1e6, cn, (in_b + 63 * N) / cn / 1e6, cw,
               (in_b + 64 * N) / cw / 1e6, cc, (in_b + 63 * N) / cc / 1e6);
    }
    return 0;
}
