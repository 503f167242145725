// ubench_issue.hip — VALU issue rate of ONE wave per SIMD with independent instructions (8
// chains), against several waves per SIMD: the adaptive kernels run at 1.25 waves per SIMD
// (LDS-bound), so their speed is a single wave's issue rate.  Kernel time by hipEvents.
// Not part of the product.  hipcc --offload-arch=gfx950 -O3 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32;
#define ITERS 8192

#define OP8(I)                                                                              \
  asm volatile(I " %0, %0, %8\n\t" I " %1, %1, %8\n\t" I " %2, %2, %8\n\t" I " %3, %3, %8\n\t" \
               I " %4, %4, %8\n\t" I " %5, %5, %8\n\t" I " %6, %6, %8\n\t" I " %7, %7, %8"    \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),        \
                 "+v"(a7)                                                                   \
               : "v"(k))

#define KERN(NAME, I)                                                                     \
  __global__ void NAME(u32* out, u32 k) {                                                 \
    u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,   \
        a6 = a0 + 6, a7 = a0 + 7;                                                         \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      OP8(I);                                                                             \
      OP8(I);                                                                             \
      OP8(I);                                                                             \
      OP8(I);                                                                             \
    }                                                                                     \
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
  }
KERN(k_add, "v_add_u32_e32")
KERN(k_mul, "v_mul_lo_u32")
KERN(k_bfi, "v_xor_b32_e32")

// v_cmp into VCC then VCC-reading selects, vs the same through an SGPR pair (8 chains)
#define SEL8(CMP, SEL, MK)                                                                   \
  asm volatile(CMP "\n\t" SEL " %0, %0, %8, " MK "\n\t" SEL " %1, %1, %8, " MK "\n\t" SEL      \
                   " %2, %2, %8, " MK "\n\t" SEL " %3, %3, %8, " MK "\n\t" CMP "\n\t" SEL       \
                   " %4, %4, %8, " MK "\n\t" SEL " %5, %5, %8, " MK "\n\t" SEL " %6, %6, %8, "  \
                   MK "\n\t" SEL " %7, %7, %8, " MK                                            \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),        \
                 "+v"(a7)                                                                   \
               : "v"(k)                                                                     \
               : "vcc", "s40", "s41")
#define KSEL(NAME, CMP, SEL, MK)                                                          \
  __global__ void NAME(u32* out, u32 k) {                                                 \
    u32 a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,   \
        a6 = a0 + 6, a7 = a0 + 7;                                                         \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      SEL8(CMP, SEL, MK);                                                                 \
      SEL8(CMP, SEL, MK);                                                                 \
      SEL8(CMP, SEL, MK);                                                                 \
      SEL8(CMP, SEL, MK);                                                                 \
    }                                                                                     \
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
  }
KSEL(k_selv, "v_cmp_lt_u32_e32 vcc, %0, %8", "v_cndmask_b32_e32", "vcc")
KSEL(k_sels, "v_cmp_lt_u32_e64 s[40:41], %0, %8", "v_cndmask_b32_e64", "s[40:41]")

int main() {
  u32* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int dev;
  hipGetDevice(&dev);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  const char* nm[5] = {"v_add_u32", "v_mul_lo_u32", "v_xor_b32", "cmp+4cnd vcc", "cmp+4cnd sgpr"};
  for (int kk = 0; kk < 5; ++kk)
    for (int wps = 1; wps <= 8; wps *= 2) {
      const int blocks = 256 * 4 * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (kk == 0) hipLaunchKernelGGL(k_add, blocks, 64, 0, 0, out, 3);
        if (kk == 1) hipLaunchKernelGGL(k_mul, blocks, 64, 0, 0, out, 3);
        if (kk == 2) hipLaunchKernelGGL(k_bfi, blocks, 64, 0, 0, out, 3);
        if (kk == 3) hipLaunchKernelGGL(k_selv, blocks, 64, 0, 0, out, 3);
        if (kk == 4) hipLaunchKernelGGL(k_sels, blocks, 64, 0, 0, out, 3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)ITERS * (kk >= 3 ? 40 : 32) * wps;  // wave-instructions per SIMD
      const double cyc = ms * 1e-3 * clk * 1e3;
      printf("%-14s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (%.3f ms, %d MHz)\n",
             nm[kk], wps, cyc / instr_per_simd, ms, clk / 1000);
    }
  return 0;
}
