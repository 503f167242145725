// ubench_halfwave.hip — does a wave64 VALU instruction with only some lanes active cost less
// issue time on gfx950 (SIMD-32: a wave64 instruction in two passes)?  VERDICT r04 next #2: if
// an instruction with exec[63:32] == 0 took half the cycles, the adaptive decoder (LDS-bound at
// 1.25 waves per SIMD) could run 32-lane half-waves at twice the waves per SIMD.
//
// Each wave runs ITERS x 32 instructions of one class, 8 independent chains (issue-bound), or
// one dependent chain (latency-bound), with exec = 64, 32 (lanes 0-31), 16 or 1 active lanes,
// at 1, 2 and 4 waves per SIMD.  Lane 0 stamps s_memtime around the loop: cycles per
// wave-instruction of one wave = delta / (ITERS x 32); per SIMD = that / waves per SIMD.
// Not part of the product.  hipcc --offload-arch=gfx950 -O3 -o tools/ubench_halfwave tools/ubench_halfwave.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
typedef uint32_t u32;
typedef uint64_t u64;
#define ITERS 4096

#define OP8(I)                                                                              \
  asm volatile(I " %0, %0, %8\n\t" I " %1, %1, %8\n\t" I " %2, %2, %8\n\t" I " %3, %3, %8\n\t" \
               I " %4, %4, %8\n\t" I " %5, %5, %8\n\t" I " %6, %6, %8\n\t" I " %7, %7, %8"    \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),        \
                 "+v"(a7)                                                                   \
               : "v"(k))
#define DEP8(I)                                                                             \
  asm volatile(I " %0, %0, %1\n\t" I " %0, %0, %1\n\t" I " %0, %0, %1\n\t" I " %0, %0, %1\n\t" \
               I " %0, %0, %1\n\t" I " %0, %0, %1\n\t" I " %0, %0, %1\n\t" I " %0, %0, %1"    \
               : "+v"(a0)                                                                   \
               : "v"(k))
#define MAD8()                                                                              \
  asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[40:41], %8, %8, %1\n\t" \
               "v_mad_u64_u32 %2, s[40:41], %8, %8, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\t" \
               "v_mad_u64_u32 %4, s[40:41], %8, %8, %4\n\tv_mad_u64_u32 %5, s[40:41], %8, %8, %5\n\t" \
               "v_mad_u64_u32 %6, s[40:41], %8, %8, %6\n\tv_mad_u64_u32 %7, s[40:41], %8, %8, %7"   \
               : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) \
               : "v"(k)                                                                     \
               : "s40", "s41")

// kind: 0 v_add_u32 x 8 chains, 1 v_add_u32 one chain, 2 v_mad_u64_u32 x 8 chains,
// 3 v_xor_b32 x 8 chains
template <int KIND>
__global__ __launch_bounds__(64) void k_issue(u64* cyc, u32* out, u32 k, u32 active) {
  const u32 lane = threadIdx.x;
  u32 a0 = lane, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
      a7 = a0 + 7;
  u64 b0 = lane, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6,
      b7 = b0 + 7;
  u64 t0 = 0, t1 = 0;
  if (lane < active) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
      if (KIND == 0) { OP8("v_add_u32_e32"); OP8("v_add_u32_e32"); OP8("v_add_u32_e32"); OP8("v_add_u32_e32"); }
      if (KIND == 1) { DEP8("v_add_u32_e32"); DEP8("v_add_u32_e32"); DEP8("v_add_u32_e32"); DEP8("v_add_u32_e32"); }
      if (KIND == 2) { MAD8(); MAD8(); MAD8(); MAD8(); }
      if (KIND == 3) { OP8("v_xor_b32_e32"); OP8("v_xor_b32_e32"); OP8("v_xor_b32_e32"); OP8("v_xor_b32_e32"); }
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  out[blockIdx.x * 64 + lane] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (u32)(b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7);
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  int n_cu = 256;
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int max_blocks = n_cu * 4 * 4;
  u64* dcyc;
  u32* out;
  (void)hipMalloc(&dcyc, max_blocks * sizeof(u64));
  (void)hipMalloc(&out, (size_t)max_blocks * 64 * sizeof(u32));
  const char* names[4] = {"v_add_u32 x8 chains", "v_add_u32 dep chain", "v_mad_u64_u32 x8", "v_xor_b32 x8"};
  const u32 actives[4] = {64, 32, 16, 1};
  printf("{\"cus\": %d, \"iters\": %d, \"rows\": [\n", n_cu, ITERS);
  bool first = true;
  for (int kind = 0; kind < 4; ++kind)
    for (int wps = 1; wps <= 4; wps *= 2)
      for (u32 act : actives) {
        const int blocks = n_cu * 4 * wps;  // one-wave blocks: wps waves on each of 4 SIMDs/CU
        std::vector<u64> h(blocks);
        for (int rep = 0; rep < 2; ++rep) {
          if (kind == 0) hipLaunchKernelGGL(k_issue<0>, blocks, 64, 0, 0, dcyc, out, 3u, act);
          if (kind == 1) hipLaunchKernelGGL(k_issue<1>, blocks, 64, 0, 0, dcyc, out, 3u, act);
          if (kind == 2) hipLaunchKernelGGL(k_issue<2>, blocks, 64, 0, 0, dcyc, out, 3u, act);
          if (kind == 3) hipLaunchKernelGGL(k_issue<3>, blocks, 64, 0, 0, dcyc, out, 3u, act);
          (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h.data(), dcyc, blocks * sizeof(u64), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double med = (double)h[blocks / 2] / (ITERS * 32.0);
        printf("%s {\"op\": \"%s\", \"waves_per_simd\": %d, \"active_lanes\": %u, "
               "\"wave_cycles_per_instr\": %.3f, \"simd_cycles_per_instr\": %.3f}\n",
               first ? " " : ",", names[kind], wps, act, med, med / wps);
        first = false;
      }
  printf("]}\n");
  return 0;
}
