// ubench_lds_unaligned.hip — does gfx950 (as configured by ROCm) honour byte-unaligned
// ds_write_b32 / ds_read_b32, and what do they cost?  Not part of the product: it decides the
// layout of the coder's per-lane LDS rings.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds_unaligned tools/ubench_lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32;
typedef uint64_t u64;

#define STRIDE 132  // bytes per lane region

static __device__ __forceinline__ void st32(u32 addr, u32 v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
static __device__ __forceinline__ u32 ld32(u32 addr) {
  u32 v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// correctness: each lane writes bytes 0..127 of its region with unaligned dword stores at
// positions advancing by 1..3 bytes; the later store overwrites the tail of the earlier one.
__global__ void k_check(u32* err, u32* sample) {
  __shared__ uint8_t buf[256 * STRIDE];
  const u32 tid = threadIdx.x;
  const u32 base = (u32)(uintptr_t)buf + tid * STRIDE;
  for (u32 i = 0; i < STRIDE; ++i) buf[tid * STRIDE + i] = 0xEE;
  __syncthreads();
  u32 p = 0, step = 1 + (tid % 3);
  while (p + 4 <= 128) {
    const u32 v = (p + tid) | ((p + tid + 1) << 8) | ((p + tid + 2) << 16) | ((p + tid + 3) << 24);
    st32(base + p, v);  // bytes p..p+3 = p+tid .. p+tid+3 (mod 256)
    p += step;
  }
  __syncthreads();
  u32 bad = 0;
  for (u32 i = 0; i < p; ++i)
    if (buf[tid * STRIDE + i] != (uint8_t)(i + tid)) ++bad;
  // unaligned read back
  for (u32 i = 0; i + 4 <= p; ++i) {
    const u32 v = ld32(base + i);
    const u32 want = (uint8_t)(i + tid) | ((uint8_t)(i + tid + 1) << 8) |
                     ((uint8_t)(i + tid + 2) << 16) | ((u32)(uint8_t)(i + tid + 3) << 24);
    if (v != want) ++bad;
  }
  atomicAdd(err, bad);
  if (tid == 1)
    for (int i = 0; i < 16; ++i) sample[i] = buf[tid * STRIDE + i];
}

// throughput: every lane stores one dword per step at its own advancing byte position (1 B per
// step on average, like the uniform encoder), 4 waves per SIMD
template <int ALIGNED>
__global__ __launch_bounds__(256) void k_rate(u32* out, u32 iters) {
  __shared__ uint8_t buf[256 * STRIDE];
  const u32 tid = threadIdx.x;
  const u32 base = (u32)(uintptr_t)buf + tid * STRIDE;
  u32 p = tid & 3, acc = tid;
  for (u32 i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const u32 a = ALIGNED ? (base + (p & 124)) : (base + (p & 127));
      st32(a, acc);
      acc = acc * 1664525u + 1013904223u;
      p += (acc >> 30) & 1 ? 1 : 0;
      p += 1;
    }
  }
  __syncthreads();
  out[blockIdx.x * 256 + tid] = buf[(tid * 7) % (256 * STRIDE)] + p;
}

int main() {
  u32 *err, *sample, *out;
  hipMalloc(&err, 4);
  hipMalloc(&sample, 64);
  hipMemset(err, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, err, sample);
  u32 e = 0, smp[16];
  hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
  hipMemcpy(smp, sample, 64, hipMemcpyDeviceToHost);
  printf("unaligned ds_write_b32/ds_read_b32 mismatches: %u (lane 1 bytes:", e);
  for (int i = 0; i < 16; ++i) printf(" %02x", smp[i]);
  printf(")\n");
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipMalloc(&out, (size_t)cus * 4 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const u32 iters = 4096;
  for (int al = 1; al >= 0; --al) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (al)
        hipLaunchKernelGGL(k_rate<1>, dim3(cus * 4), dim3(256), 0, 0, out, iters);
      else
        hipLaunchKernelGGL(k_rate<0>, dim3(cus * 4), dim3(256), 0, 0, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double wi = (double)cus * 4 * 4 * iters * 16;  // wave-instructions (stores)
      if (rep) printf("%s stores: %.2f ns per wave-store per CU (%.1f cycles at 2.09 GHz)\n",
                      al ? "aligned  " : "unaligned", ms * 1e6 / (wi / cus),
                      ms * 1e-3 * 2.09e9 / (wi / cus));
    }
  }
  return 0;
}
