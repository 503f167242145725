// ubench_sel.hip — cost of v_cndmask_b32 (VOP2, VCC) vs v_cndmask_b32_e64 (SGPR pair) in the
// shape the adaptive decoder uses them: a v_cmp producing the mask, then selects reading it.
// Not part of the product.  hipcc --offload-arch=gfx950 -O3 -o tools/ubench_sel tools/ubench_sel.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32;
typedef uint64_t u64;
#define ITERS 4096

__global__ void k_vcc(u32* out, u32 seed, u64* clk) {
  u32 a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a ^ 9, f = a + 11;
  u64 t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      asm volatile(
          "v_cmp_lt_u32_e32 vcc, %0, %1\n"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n"
          "v_cndmask_b32_e32 %3, %3, %4, vcc\n"
          "v_cndmask_b32_e32 %4, %4, %5, vcc\n"
          "v_cndmask_b32_e32 %5, %5, %2, vcc\n"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)::"vcc");
    }
  }
  u64 t1 = __builtin_readcyclecounter();
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f;
}

__global__ void k_sgpr(u32* out, u32 seed, u64* clk) {
  u32 a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a ^ 9, f = a + 11;
  u64 t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      asm volatile(
          "v_cmp_lt_u32_e64 s[40:41], %0, %1\n"
          "v_cndmask_b32_e64 %2, %2, %3, s[40:41]\n"
          "v_cndmask_b32_e64 %3, %3, %4, s[40:41]\n"
          "v_cndmask_b32_e64 %4, %4, %5, s[40:41]\n"
          "v_cndmask_b32_e64 %5, %5, %2, s[40:41]\n"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)::"s40", "s41");
    }
  }
  u64 t1 = __builtin_readcyclecounter();
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f;
}

__global__ void k_add(u32* out, u32 seed, u64* clk) {  // reference: 5 dependent-ish adds
  u32 a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a ^ 9, f = a + 11;
  u64 t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      asm volatile(
          "v_sub_u32_e32 %0, %0, %1\n"
          "v_add_u32_e32 %2, %2, %3\n"
          "v_add_u32_e32 %3, %3, %4\n"
          "v_add_u32_e32 %4, %4, %5\n"
          "v_add_u32_e32 %5, %5, %2\n"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f));
    }
  }
  u64 t1 = __builtin_readcyclecounter();
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f;
}

int main() {
  u32* out;
  u64* clk;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&clk, 64);
  const char* nm[3] = {"cmp+4 cndmask_e32 (vcc)", "cmp+4 cndmask_e64 (sgpr)", "5 add/sub"};
  for (int wps = 1; wps <= 8; wps *= 2) {
    for (int kk = 0; kk < 3; ++kk) {
      const int blocks = 256 * 4 * wps;  // wps waves per SIMD over 256 CUs x 4 SIMDs
      for (int rep = 0; rep < 2; ++rep) {
        if (kk == 0) hipLaunchKernelGGL(k_vcc, blocks, 64, 0, 0, out, 1, clk);
        if (kk == 1) hipLaunchKernelGGL(k_sgpr, blocks, 64, 0, 0, out, 1, clk);
        if (kk == 2) hipLaunchKernelGGL(k_add, blocks, 64, 0, 0, out, 1, clk);
      }
      hipDeviceSynchronize();
      u64 c;
      hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
      printf("waves/SIMD %d  %-28s %.2f cycles per 5-instruction group (per wave)\n", wps, nm[kk],
             (double)c / (ITERS * 8));
    }
  }
  return 0;
}
