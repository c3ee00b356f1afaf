// Sparse column arena probe (not product code).  profiles/r6/stride/ found that a 1.25e7-record T20
// decode runs at 0.61-0.63 of peak with its columns at their own stride and 0.67-0.73 with the
// columns 1e8 rows apart (a padded, mostly unused arena).  Does the gain need the padding's physical
// memory, or only the virtual spacing?  The T20 decode's memory pattern (tools/spacing_probe.hip's
// window kernel: 1024-row windows of 64-byte records through LDS into 20 column pieces) is timed with
// its columns placed
//   dense   one hipMalloc, stride = rows (the product's layout for this launch)
//   padded  one hipMalloc, stride = 1e8 rows (8x the memory)
//   sparse  stride = 1e8 rows, physical memory mapped (hipMemCreate + hipMemMap) only under each
//           column's used bytes: one reservation and one physical allocation per column
//   split   stride = rows, VMM-mapped the same way (columns that share a 2 MiB page share a mapping:
//           the control for "VMM instead of hipMalloc")
// each on `allocs` fresh allocations, `reps` launches each (HIP events).  Before any launch the host
// checks that every byte the kernel writes lies in a mapped range.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/sparse_probe tools/sparse_probe.hip
// usage: tools/sparse_probe [rows=12500000] [allocs=4] [reps=6]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
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
static const int hW[NC] = {4, 4, 4, 4, 4, 8, 8, 4, 4, 2, 2, 2, 1, 1, 1, 1, 4, 4, 1, 1};
constexpr int ROWS = 1024, REC = 64;

__global__ void __launch_bounds__(256) k_window(const uint4 *__restrict__ in, uint8_t *__restrict__ out, uint64_t cap,
                                                uint32_t nwin) {
    __shared__ uint4 lds[ROWS * REC / 16];
    const uint32_t G = gridDim.x, X = 8, x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X, start = x * per, end = min(nwin, start + per);
    for (uint32_t W = start + l; W < end; W += G / X) {
        const uint4 *src = in + (uint64_t)W * (ROWS * REC / 16);
#pragma unroll 4
        for (int i = threadIdx.x; i < ROWS * REC / 16; i += 256) lds[i] = src[i];
        __syncthreads();
        for (int c = 0; c < NC; ++c) {
            const int w = kW[c], o = kOff[c];
            uint4 *dst = (uint4 *)(out + cap * o + (uint64_t)W * ROWS * w);
            const int pieces = ROWS * w / 16;
            for (int p = threadIdx.x; p < pieces; p += 256) dst[p] = lds[(c * 64 + p) & (ROWS * REC / 16 - 1)];
        }
        __syncthreads();
    }
}

struct Arena {
    uint8_t *base = nullptr;
    size_t va = 0;
    bool vmm = false;
    bool access = true;  // hipMemSetAccess granted (always for hipMalloc)
    std::vector<std::pair<size_t, size_t>> maps;  // mapped [off, off + len)
    std::vector<hipMemGenericAllocationHandle_t> handles;
    std::vector<std::pair<size_t, size_t>> resv;  // VMM reservations [off, off + len)
};

static size_t gran_of() {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t g = 0;
    CK(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
    return std::max<size_t>(g, 2u << 20);  // whole 2 MiB pages (hipMemSetAccess refused 4 KiB-aligned pieces)
}

// VMM arena: the columns' merged byte ranges at their offsets from one base, each range its own
// reservation (at base + offset: the runtime granted access only to a mapping that starts its
// reservation) backed by its own physical allocation.  va: the span; ok = false if a reservation
// did not land where asked (then nothing is launched on it)
static Arena make_vmm(size_t va, const std::vector<std::pair<size_t, size_t>> &used, size_t gran) {
    Arena a;
    a.vmm = true;
    a.va = (va + gran - 1) / gran * gran;
    void *p = nullptr;
    CK(hipMemAddressReserve(&p, a.va, gran, nullptr, 0));  // find a free span, then give it back
    a.base = (uint8_t *)p;
    CK(hipMemAddressFree(p, a.va));
    std::vector<std::pair<size_t, size_t>> iv;
    for (auto u : used) iv.push_back({u.first / gran * gran, (u.first + u.second + gran - 1) / gran * gran});
    std::sort(iv.begin(), iv.end());
    std::vector<std::pair<size_t, size_t>> merged;
    for (auto v : iv) {
        if (!merged.empty() && v.first <= merged.back().second) merged.back().second = std::max(merged.back().second, v.second);
        else merged.push_back(v);
    }
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    hipMemAccessDesc acc = {};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = 0;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    a.access = true;
    for (auto m : merged) {
        const size_t len = m.second - m.first;
        void *q = nullptr;
        if (hipMemAddressReserve(&q, len, gran, a.base + m.first, 0) != hipSuccess || q != a.base + m.first) {
            (void)hipGetLastError();
            if (q) CK(hipMemAddressFree(q, len));
            a.access = false;
            break;
        }
        a.resv.push_back({m.first, len});
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, len, &prop, 0));
        CK(hipMemMap(a.base + m.first, len, 0, h, 0));
        a.handles.push_back(h);
        a.maps.push_back({m.first, len});
        if (hipMemSetAccess(a.base + m.first, len, &acc, 1) != hipSuccess) {
            (void)hipGetLastError();
            a.access = false;
            break;
        }
    }
    return a;
}

static Arena make_plain(size_t bytes) {
    Arena a;
    void *p = nullptr;
    CK(hipMalloc(&p, bytes));
    a.base = (uint8_t *)p;
    a.va = bytes;
    a.maps.push_back({0, bytes});
    return a;
}

static void free_arena(Arena &a) {
    if (a.vmm) {
        for (auto m : a.maps) CK(hipMemUnmap(a.base + m.first, m.second));
        for (auto h : a.handles) CK(hipMemRelease(h));
        for (auto r : a.resv) CK(hipMemAddressFree(a.base + r.first, r.second));
    } else {
        CK(hipFree(a.base));
    }
    a = Arena();
}

static bool covered(const Arena &a, size_t off, size_t len) {
    for (auto m : a.maps)
        if (off >= m.first && off + len <= m.first + m.second) return true;
    return false;
}

int main(int argc, char **argv) {
    const uint64_t rows = argc > 1 ? strtoull(argv[1], 0, 10) : 12500000ull;
    const int allocs = argc > 2 ? atoi(argv[2]) : 4;
    const int reps = argc > 3 ? atoi(argv[3]) : 6;
    int vmm_ok = 0;
    CK(hipDeviceGetAttribute(&vmm_ok, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
    const uint32_t nwin = (uint32_t)((rows + ROWS - 1) / ROWS);
    int off[NC], acc = 0;
    for (int c = 0; c < NC; ++c) {
        off[c] = acc;
        acc += hW[c];
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(kOff), off, sizeof off));
    const uint64_t in_b = (uint64_t)nwin * ROWS * REC;
    void *in;
    CK(hipMalloc(&in, in_b));
    CK(hipMemset(in, 3, in_b));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t grid = cus * 8;
    const size_t gran = vmm_ok ? gran_of() : 0;
    const uint64_t wide = 100000000ull;  // the 10^8 launch's stride, in rows
    printf("{\"vmm_supported\": %d, \"granularity\": %zu, \"rows\": %llu}\n", vmm_ok, gran, (unsigned long long)rows);
    fflush(stdout);
    const char *names[4] = {"dense", "padded", "sparse", "split"};
    for (int mode = 0; mode < 4; ++mode) {
        if (mode >= 2 && !vmm_ok) continue;
        const uint64_t cap = (mode == 1 || mode == 2) ? std::max<uint64_t>(wide, (uint64_t)nwin * ROWS) : (uint64_t)nwin * ROWS;
        std::vector<std::pair<size_t, size_t>> used;
        for (int c = 0; c < NC; ++c) used.push_back({(size_t)(cap * off[c]), (size_t)nwin * ROWS * hW[c]});
        for (int k = 0; k < allocs; ++k) {
            Arena a = mode < 2 ? make_plain(cap * REC + 4096) : make_vmm(cap * REC + 4096, used, gran);
            if (!a.access) {
                printf("{\"layout\": \"%s\", \"alloc\": %d, \"skipped\": \"hipMemSetAccess refused\"}\n", names[mode], k);
                fflush(stdout);
                free_arena(a);
                break;
            }
            for (auto u : used)
                if (!covered(a, u.first, u.second)) {
                    fprintf(stderr, "unmapped column range %zu + %zu\n", u.first, u.second);
                    exit(1);
                }
            hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, a.base, cap, nwin);
            CK(hipDeviceSynchronize());
            float sum = 0, best = 1e9;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(k_window, dim3(grid), dim3(256), 0, 0, (const uint4 *)in, a.base, cap, nwin);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                sum += ms;
                best = std::min(best, ms);
            }
            size_t mapped = 0;
            for (auto m : a.maps) mapped += m.second;
            printf("{\"layout\": \"%s\", \"alloc\": %d, \"stride_rows\": %llu, \"mapped_mb\": %.0f, \"ms\": %.4f, "
                   "\"best_ms\": %.4f, \"tbs\": %.3f}\n",
                   names[mode], k, (unsigned long long)cap, mapped / 1048576.0, sum / reps, best,
                   2.0 * nwin * ROWS * REC / (sum / reps) / 1e9);
            fflush(stdout);
            free_arena(a);
        }
    }
    CK(hipFree(in));
    return 0;
}
