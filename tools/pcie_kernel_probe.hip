// PCIe probe: copy engines (hipMemcpyAsync) against kernels that load from or store to pinned
// host memory directly, alone and concurrently, to find out whether the two directions of the
// link can be driven at once (one by a copy engine, the other by the CUs).
// build: hipcc --offload-arch=gfx950 -O2 -o tools/pcie_kernel_probe tools/pcie_kernel_probe.hip
// usage: tools/pcie_kernel_probe [MiB] [reps]      prints one JSON line
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// grid-stride 16-byte copy; either side may be host memory
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t step = (size_t)gridDim.x * blockDim.x;
  for (; i + 3 * step < n16; i += 4 * step) {
    uint4 a = src[i], b = src[i + step], c = src[i + 2 * step], d = src[i + 3 * step];
    dst[i] = a;
    dst[i + step] = b;
    dst[i + 2 * step] = c;
    dst[i + 3 * step] = d;
  }
  for (; i < n16; i += step) dst[i] = src[i];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  size_t mb = argc > 1 ? strtoul(argv[1], 0, 10) : 640;
  int reps = argc > 2 ? atoi(argv[2]) : 5;
  int blocks = getenv("PROBE_BLOCKS") ? atoi(getenv("PROBE_BLOCKS")) : 512;
  size_t n = mb << 20, n16 = n / 16;
  void *h_src, *h_dst, *d_a, *d_b;
  CK(hipHostMalloc(&h_src, n, hipHostMallocDefault));
  CK(hipHostMalloc(&h_dst, n, hipHostMallocDefault));
  CK(hipMalloc(&d_a, n));
  CK(hipMalloc(&d_b, n));
  CK(hipMemset(d_a, 1, n));
  CK(hipMemset(d_b, 2, n));
  for (size_t i = 0; i < n; i += 4096) ((char*)h_src)[i] = (char)i;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));

  auto h2d_dma = [&](hipStream_t s) { CK(hipMemcpyAsync(d_a, h_src, n, hipMemcpyHostToDevice, s)); };
  auto d2h_dma = [&](hipStream_t s) { CK(hipMemcpyAsync(h_dst, d_b, n, hipMemcpyDeviceToHost, s)); };
  auto h2d_krn = [&](hipStream_t s) {
    hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, (const uint4*)h_src, (uint4*)d_a, n16);
    CK(hipGetLastError());
  };
  auto d2h_krn = [&](hipStream_t s) {
    hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, (const uint4*)d_b, (uint4*)h_dst, n16);
    CK(hipGetLastError());
  };
  auto timed = [&](auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    double best = 1e9;
    for (int r = 0; r < reps; r++) {
      double t0 = now();
      fn();
      CK(hipDeviceSynchronize());
      double t = now() - t0;
      if (t < best) best = t;
    }
    return best;
  };
  double gb = n / 1e9;
  double t_h2d_dma = timed([&] { h2d_dma(s1); });
  double t_d2h_dma = timed([&] { d2h_dma(s2); });
  double t_h2d_krn = timed([&] { h2d_krn(s1); });
  double t_d2h_krn = timed([&] { d2h_krn(s2); });
  double t_dma_dma = timed([&] { h2d_dma(s1); d2h_dma(s2); });
  double t_dma_krn = timed([&] { h2d_dma(s1); d2h_krn(s2); });   // H2D on a copy engine, D2H by CUs
  double t_krn_dma = timed([&] { h2d_krn(s1); d2h_dma(s2); });   // H2D by CUs, D2H on a copy engine
  double t_krn_krn = timed([&] { h2d_krn(s1); d2h_krn(s2); });
  printf("{\"bytes\": %zu, \"blocks\": %d, \"h2d_dma_gbps\": %.2f, \"d2h_dma_gbps\": %.2f, "
         "\"h2d_kernel_gbps\": %.2f, \"d2h_kernel_gbps\": %.2f, \"duplex_dma_dma_gbps\": %.2f, "
         "\"duplex_h2d_dma_d2h_kernel_gbps\": %.2f, \"duplex_h2d_kernel_d2h_dma_gbps\": %.2f, "
         "\"duplex_kernel_kernel_gbps\": %.2f}\n",
         n, blocks, gb / t_h2d_dma, gb / t_d2h_dma, gb / t_h2d_krn, gb / t_d2h_krn, 2 * gb / t_dma_dma,
         2 * gb / t_dma_krn, 2 * gb / t_krn_dma, 2 * gb / t_krn_krn);
  // spot check the kernel copies
  CK(hipMemcpy(h_dst, d_b, 64, hipMemcpyDeviceToHost));
  if (((unsigned char*)h_dst)[0] != 2) {
    fprintf(stderr, "d2h check failed\n");
    return 2;
  }
  CK(hipStreamDestroy(s1));
  CK(hipStreamDestroy(s2));
  CK(hipFree(d_a));
  CK(hipFree(d_b));
  CK(hipHostFree(h_src));
  CK(hipHostFree(h_dst));
  return 0;
}
