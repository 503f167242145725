// PCIe probe with copy kernels instead of the DMA engines: the kernel reads (H2D) or writes
// (D2H) pinned, device-mapped host memory directly with 16-B coalesced accesses.  Times each
// direction alone and both at once on two streams, for a few grid sizes.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/pcie_kernel_probe tools/pcie_kernel_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                              uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) v[u] = src[i + 256 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) dst[i + 256 * u] = v[u];
  }
}

// latency-bound stand-in for a coder batch: 64 workgroups of dependent HBM loads
__global__ __launch_bounds__(256) void k_chase(const uint32_t* __restrict__ t, uint32_t mask,
                                               uint32_t* sink, int steps) {
  uint32_t x = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < steps; ++i) x = t[(x * 2654435761u + i) & mask] + x;
  if (x == 0x12345678u) sink[0] = x;
}

#define CK(x) do { if ((x) != hipSuccess) { printf("fail %s\n", #x); return 1; } } while (0)

int main() {
  const uint64_t n = 2ull << 30, n16 = n / 16;
  void *h_in, *h_out, *d_a, *d_b;
  CK(hipHostMalloc(&h_in, n, hipHostMallocMapped));
  CK(hipHostMalloc(&h_out, n, hipHostMallocMapped));
  CK(hipMalloc(&d_a, n));
  CK(hipMalloc(&d_b, n));
  void *hi_d, *ho_d;
  CK(hipHostGetDevicePointer(&hi_d, h_in, 0));
  CK(hipHostGetDevicePointer(&ho_d, h_out, 0));
  CK(hipMemset(d_b, 3, n));
  for (uint64_t i = 0; i < n; i += 4096) ((char*)h_in)[i] = 1;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  {  // per copy grid: both directions at once, and a latency-bound kernel beside them
    const uint32_t mask = (uint32_t)(n / 4 - 1);
    uint32_t* sink;
    CK(hipMalloc(&sink, 4));
    uint32_t cm[8];
    for (int i = 0; i < 8; ++i) cm[i] = 0xAAAAAAAAu;  // odd CUs: its own queue and CUs
    hipStream_t s3;
    CK(hipExtStreamCreateWithCUMask(&s3, 8, cm));
    hipEvent_t c0, c1;
    CK(hipEventCreate(&c0));
    CK(hipEventCreate(&c1));
    const int gs[] = {0, 16, 32, 64, 128, 256};
    for (int g : gs) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      CK(hipDeviceSynchronize());
      if (g) {
        hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s1, (const uint4*)hi_d, (uint4*)d_a, n16);
        hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s2, (const uint4*)d_b, (uint4*)ho_d, n16);
      }
      CK(hipEventRecord(c0, s3));
      hipLaunchKernelGGL(k_chase, dim3(64), dim3(256), 0, s3, (const uint32_t*)d_a, mask, sink, 4000);
      CK(hipEventRecord(c1, s3));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms, cms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipEventElapsedTime(&cms, c0, c1));
      printf("copy grid %3d: both at once %.1f GB/s each way; chase %.2f ms\n", g,
             g ? n / ms / 1e6 : 0.0, cms);
      fflush(stdout);
    }
  }
  {  // DMA engines: H2D by hipMemcpyAsync beside a 256-WG D2H copy kernel, and beside the chase
    const uint32_t mask = (uint32_t)(n / 4 - 1);
    uint32_t* sink;
    CK(hipMalloc(&sink, 4));
    hipEvent_t a0, a1, b0, b1;
    CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1)); CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1));
    for (int mode = 0; mode < 3; ++mode) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a0, s1));
      CK(hipMemcpyAsync(d_a, h_in, n, hipMemcpyHostToDevice, s1));
      CK(hipEventRecord(a1, s1));
      CK(hipEventRecord(b0, s2));
      if (mode == 0) hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, s2, (const uint4*)d_b, (uint4*)ho_d, n16);
      if (mode == 1) CK(hipMemcpyAsync(h_out, d_b, n, hipMemcpyDeviceToHost, s2));
      if (mode == 2) hipLaunchKernelGGL(k_chase, dim3(64), dim3(256), 0, s2, (const uint32_t*)d_b, mask, sink, 4000);
      CK(hipEventRecord(b1, s2));
      CK(hipDeviceSynchronize());
      float ma, mb;
      CK(hipEventElapsedTime(&ma, a0, a1));
      CK(hipEventElapsedTime(&mb, b0, b1));
      const char* nm[] = {"kernel D2H", "DMA D2H", "chase"};
      printf("DMA H2D %.1f GB/s beside %s: %.2f ms (%.1f GB/s)\n", n / ma / 1e6, nm[mode], mb, n / mb / 1e6);
      fflush(stdout);
    }
  }
  const int grids[] = {256};
  for (int g : grids) {
    float best[3] = {1e9f, 1e9f, 1e9f};
    for (int mode = 0; mode < 3; ++mode)
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        CK(hipDeviceSynchronize());
        if (mode != 1) hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s1, (const uint4*)hi_d, (uint4*)d_a, n16);
        if (mode != 0) hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s2, (const uint4*)d_b, (uint4*)ho_d, n16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best[mode]) best[mode] = ms;
      }
    printf("grid %5d: H2D alone %.1f GB/s, D2H alone %.1f GB/s, both at once %.1f GB/s each way\n", g,
           n / best[0] / 1e6, n / best[1] / 1e6, n / best[2] / 1e6);
    fflush(stdout);
  }
  return 0;
}
