// HBM probe 2 (not product code): T20 decode shapes with packed multi-row
// column stores.  Which store granularity reaches the copy ceiling?
//   cC   : lane owns C consecutive records (C=4: 256 rows/wave, C=8: 512)
//   lds  : 256-thread workgroup decodes 1024 rows into LDS (column-major),
//          then writes each column's 1024*width bytes with 16-B stores
//   *_w  : the same stores with no loads (values from the row index)
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_probe2.hip -o /tmp/hbm_probe2
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr uint64_t N = 99999744ull;  // 97656 x 1024 records
struct Fld {
    int off, len, w;
};
constexpr Fld T[20] = {{0, 4, 4},  {4, 4, 4},  {8, 4, 4},  {12, 4, 4}, {16, 4, 4}, {20, 8, 8}, {28, 8, 8},
                       {36, 4, 4}, {40, 4, 4}, {44, 2, 2}, {46, 2, 2}, {48, 2, 1}, {50, 1, 1}, {51, 1, 1},
                       {52, 1, 1}, {53, 1, 1}, {54, 4, 4}, {58, 4, 4}, {62, 1, 1}, {63, 1, 1}};
__host__ __device__ constexpr int coff(int f) {
    int s = 0;
    for (int i = 0; i < f; ++i) s += T[i].w;
    return s;
}
constexpr int ROWB = coff(20);  // 63

__device__ __forceinline__ uint32_t dw(const uint32_t *R, int o) {
    const int q = o >> 2;
    return (o & 3) ? __builtin_amdgcn_alignbyte(R[q + 1], R[q], o & 3) : R[q];
}
__device__ __forceinline__ uint64_t val(const uint32_t *R, int f) {
    const int o = T[f].off, l = T[f].len;
    if (l <= 4) {
        uint32_t a = __builtin_bswap32(dw(R, o)) >> (32 - 8 * l);
        if (f == 11) a &= 0xFF;
        return a;
    }
    const uint32_t a = __builtin_bswap32(dw(R, o)), b = __builtin_bswap32(dw(R, o + 4));
    return ((uint64_t)a << 32) | b;
}

// pack C values of width w into C*w/4 dwords
template <int C>
__device__ __forceinline__ void pack(const uint64_t (&v)[C], int w, uint32_t *o) {
    if (w == 1) {
#pragma unroll
        for (int i = 0; i < C / 4; ++i)
            o[i] = (uint32_t)(v[4 * i] & 0xFF) | (uint32_t)(v[4 * i + 1] & 0xFF) << 8 |
                   (uint32_t)(v[4 * i + 2] & 0xFF) << 16 | (uint32_t)(v[4 * i + 3] & 0xFF) << 24;
    } else if (w == 2) {
#pragma unroll
        for (int i = 0; i < C / 2; ++i) o[i] = (uint32_t)(v[2 * i] & 0xFFFF) | (uint32_t)(v[2 * i + 1] & 0xFFFF) << 16;
    } else if (w == 4) {
#pragma unroll
        for (int i = 0; i < C; ++i) o[i] = (uint32_t)v[i];
    } else {
#pragma unroll
        for (int i = 0; i < C; ++i) {
            o[2 * i] = (uint32_t)v[i];
            o[2 * i + 1] = (uint32_t)(v[i] >> 32);
        }
    }
}

template <int ND>
__device__ __forceinline__ void st(uint8_t *p, const uint32_t *o) {
    if constexpr (ND == 1) *(uint32_t *)p = o[0];
    else if constexpr (ND == 2) *(uint2 *)p = make_uint2(o[0], o[1]);
    else {
#pragma unroll
        for (int i = 0; i < ND / 4; ++i) ((uint4 *)p)[i] = make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
    }
}

template <int C, bool LOAD>
__global__ void __launch_bounds__(256) k_c(const uint4 *__restrict__ in, uint8_t *__restrict__ cols, uint32_t nwin,
                                           int contiguous) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    uint32_t w0 = wid, w1 = nwin, step = nw;
    if (contiguous) {  // each wave a contiguous range of windows
        const uint32_t per = (nwin + nw - 1) / nw;
        w0 = wid * per;
        w1 = min(nwin, w0 + per);
        step = 1;
    }
    for (uint32_t win = w0; win < w1; win += step) {
        const uint64_t r0 = (uint64_t)win * 64 * C + lane * C;
        uint32_t R[C][17];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            if (LOAD) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint4 v = in[(r0 + k) * 4 + j];
                    R[k][4 * j] = v.x, R[k][4 * j + 1] = v.y, R[k][4 * j + 2] = v.z, R[k][4 * j + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) R[k][j] = (uint32_t)(r0 + k) * 0x9E3779B9u + j;
            }
            R[k][16] = 0;
        }
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            uint64_t v[C];
#pragma unroll
            for (int k = 0; k < C; ++k) v[k] = val(R[k], f);
            uint32_t o[2 * C];
            const int w = T[f].w;
            pack<C>(v, w, o);
            uint8_t *p = cols + (uint64_t)coff(f) * N + r0 * w;
            if (w == 1) st<C / 4>(p, o);
            else if (w == 2) st<C / 2>(p, o);
            else if (w == 4) st<C>(p, o);
            else st<2 * C>(p, o);
        }
    }
}

// workgroup window of 1024 rows staged through LDS, column-major
template <bool LOAD>
__global__ void __launch_bounds__(256) k_lds(const uint4 *__restrict__ in, uint8_t *__restrict__ cols, uint32_t nwin,
                                             uint32_t mis = 0) {
    // mis: records start `mis` bytes past 16-byte alignment (buffer loads, 4-byte aligned)
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, 0x7FFFFFF0, 0x00020000);
    __shared__ __attribute__((aligned(16))) uint8_t S[ROWB * 1024];
    const uint32_t t = threadIdx.x;
    for (uint32_t win = blockIdx.x; win < nwin; win += gridDim.x) {
        const uint64_t r0 = (uint64_t)win * 1024 + 4 * t;
        uint32_t R[4][17];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (LOAD) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                    v4 v;
                    if (mis == 0xFFFFFFFFu) {
                        const uint4 u = in[(r0 + k) * 4 + j];
                        v = v4{u.x, u.y, u.z, u.w};
                    } else {
                        // win 31-bit offsets: window-relative resource
                        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
                            (void *)((const uint8_t *)in + (uint64_t)win * 65536), (short)0, 0x7FFFFFF0, 0x00020000);
                        v = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)((r0 + k - (uint64_t)win * 1024) * 64 + 16 * j + mis), 0, 0);
                    }
                    R[k][4 * j] = v.x, R[k][4 * j + 1] = v.y, R[k][4 * j + 2] = v.z, R[k][4 * j + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) R[k][j] = (uint32_t)(r0 + k) * 0x9E3779B9u + j;
            }
            R[k][16] = 0;
        }
        (void)rin;
        __syncthreads();  // previous window's LDS reads done
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            uint64_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = val(R[k], f);
            uint32_t o[8];
            const int w = T[f].w;
            pack<4>(v, w, o);
            uint8_t *p = S + coff(f) * 1024 + 4 * t * w;
            if (w == 1) st<1>(p, o);
            else if (w == 2) st<2>(p, o);
            else if (w == 4) st<4>(p, o);
            else st<8>(p, o);
        }
        __syncthreads();
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            const int w = T[f].w;
            const uint4 *src = (const uint4 *)(S + coff(f) * 1024);
            uint4 *dst = (uint4 *)(cols + (uint64_t)coff(f) * N + (uint64_t)win * 1024 * w);
            for (int j = t; j < 64 * w; j += 256) dst[j] = src[j];
        }
    }
}


// misaligned records loaded with 16-byte aligned loads and re-aligned in
// registers (per-lane dword shift: 2 v_cndmask per dword).  SPAN: one aligned
// span of the lane's 4 consecutive records (17 loads), else 5 loads/record.
template <bool SPAN, bool STORE = true>
__global__ void __launch_bounds__(256) k_lds_al(const uint4 *__restrict__ in, uint8_t *__restrict__ cols, uint32_t nwin,
                                                uint32_t mis) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t S[ROWB * 1024];
    const uint32_t t = threadIdx.x;
    for (uint32_t win = blockIdx.x; win < nwin; win += gridDim.x) {
        const uint64_t r0 = (uint64_t)win * 1024 + 4 * t;
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void *)((const uint8_t *)in + (uint64_t)win * 65536), (short)0, 0x7FFFFFF0, 0x00020000);
        const uint32_t a = (uint32_t)((r0 - (uint64_t)win * 1024) * 64) + mis;  // lane's first record
        const uint32_t dsh = (a >> 2) & 3;
        uint32_t R[4][17];
        if (SPAN) {
            uint32_t T[68 + 4];
#pragma unroll
            for (int j = 0; j < 17; ++j) {
                const v4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, (a & ~15u) + 16 * j, 0, 0);
                T[4 * j] = v.x, T[4 * j + 1] = v.y, T[4 * j + 2] = v.z, T[4 * j + 3] = v.w;
            }
#pragma unroll
            for (int j = 0; j < 67; ++j) T[j] = (dsh & 1) ? T[j + 1] : T[j];
#pragma unroll
            for (int j = 0; j < 65; ++j) T[j] = (dsh & 2) ? T[j + 2] : T[j];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int j = 0; j < 16; ++j) R[k][j] = T[16 * k + j];
                R[k][16] = 0;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t T[20];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const v4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, ((a + 64 * k) & ~15u) + 16 * j, 0, 0);
                    T[4 * j] = v.x, T[4 * j + 1] = v.y, T[4 * j + 2] = v.z, T[4 * j + 3] = v.w;
                }
                uint32_t U[19];
                const uint32_t m0 = 0u - (dsh & 1), m1 = 0u - ((dsh >> 1) & 1);
#pragma unroll
                for (int j = 0; j < 19; ++j) U[j] = (T[j + 1] & m0) | (T[j] & ~m0);
#pragma unroll
                for (int j = 0; j < 16; ++j) T[j] = (U[j + 2] & m1) | (U[j] & ~m1);
#pragma unroll
                for (int j = 0; j < 16; ++j) R[k][j] = T[j];
                R[k][16] = 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            uint64_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = val(R[k], f);
            uint32_t o[8];
            const int w = T[f].w;
            pack<4>(v, w, o);
            uint8_t *p = S + coff(f) * 1024 + 4 * t * w;
            if (w == 1) st<1>(p, o);
            else if (w == 2) st<2>(p, o);
            else if (w == 4) st<4>(p, o);
            else st<8>(p, o);
        }
        __syncthreads();
        if (STORE) {
#pragma unroll
        for (int f = 0; f < 20; ++f) {
            const int w = T[f].w;
            const uint4 *src = (const uint4 *)(S + coff(f) * 1024);
            uint4 *dst = (uint4 *)(cols + (uint64_t)coff(f) * N + (uint64_t)win * 1024 * w);
            for (int j = t; j < 64 * w; j += 256) dst[j] = src[j];
        }
        } else if (win == 0xFFFFFFFFu) cols[t] = S[t];
    }
}

__global__ void __launch_bounds__(256) k_copy16(const uint4 *__restrict__ in, uint4 *__restrict__ out, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
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
    const uint64_t in_b = 64 * N, out_b = (uint64_t)ROWB * N;
    uint4 *in;
    uint8_t *out;
    CK(hipMalloc(&in, in_b));
    CK(hipMalloc(&out, in_b + 4096));
    CK(hipMemset(in, 0x5A, in_b));
    const double full = (double)(in_b + out_b), wr = (double)out_b;
    auto rep = [&](const char *name, float ms, double bytes) {
        printf("  %-22s %.3f ms %6.0f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    for (int g : {cus * 2, cus * 4, cus * 8}) {
        printf("grid %d blocks x 256\n", g);
        rep("copy16", timeit([&] { k_copy16<<<g, 256>>>(in, (uint4 *)out, in_b / 16); }), 2.0 * in_b);
        if (0) rep("c4", timeit([&] { k_c<4, true><<<g, 256>>>(in, out, N / 256, 0); }), full);
        if (0) rep("c4 contiguous", timeit([&] { k_c<4, true><<<g, 256>>>(in, out, N / 256, 1); }), full);
        if (0) rep("c8", timeit([&] { k_c<8, true><<<g, 256>>>(in, out, N / 512, 0); }), full);
        if (0) rep("c8 contiguous", timeit([&] { k_c<8, true><<<g, 256>>>(in, out, N / 512, 1); }), full);
        rep("lds1024", timeit([&] { k_lds<true><<<g, 256>>>(in, out, N / 1024, 0xFFFFFFFFu); }), full);
        rep("lds1024 buf mis0", timeit([&] { k_lds<true><<<g, 256>>>(in, out, N / 1024 - 1, 0); }), full);
        rep("lds1024 buf mis4", timeit([&] { k_lds<true><<<g, 256>>>(in, out, N / 1024 - 1, 4); }), full);
        rep("al5 mis4", timeit([&] { k_lds_al<false><<<g, 256>>>(in, out, N / 1024 - 1, 4); }), full);
        rep("al5 mis4 nostore", timeit([&] { k_lds_al<false, false><<<g, 256>>>(in, out, N / 1024 - 1, 4); }), 64.0 * N);
        rep("al5 mis0", timeit([&] { k_lds_al<false><<<g, 256>>>(in, out, N / 1024 - 1, 0); }), full);
        rep("lds1024 buf mis8", timeit([&] { k_lds<true><<<g, 256>>>(in, out, N / 1024 - 1, 8); }), full);
        rep("c4_w (stores only)", timeit([&] { k_c<4, false><<<g, 256>>>(in, out, N / 256, 0); }), wr);
        rep("c8_w (stores only)", timeit([&] { k_c<8, false><<<g, 256>>>(in, out, N / 512, 0); }), wr);
        rep("lds1024_w", timeit([&] { k_lds<false><<<g, 256>>>(in, out, N / 1024, 0xFFFFFFFFu); }), wr);
    }
    return 0;
}
