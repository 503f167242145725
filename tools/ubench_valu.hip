// ubench_valu.hip — issue cost and latency of the VALU / LDS instructions the coder kernels use
// (gfx950).  Not part of the product: it measures the instruction prices DESIGN.md §5 uses to
// choose between formulations of the symbol step.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip && tools/ubench_valu
//
// thr: 8 independent chains per wave, 8 waves per SIMD (throughput: cycles per wave-instruction
//      per SIMD); lat: 1 chain, 1 wave per SIMD (dependent-issue latency, cycles).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint64_t u64;
typedef uint32_t u32;

#define ITERS 4096
#define REP 4

#define CHAIN8(INSN, T)                                                                         \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r1) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r2) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r3) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r4) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r5) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r6) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r7) : "v"(k));

#define CHAIN1(INSN, T)                                                                         \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));                                                       \
  asm volatile(INSN : "+v"(r0) : "v"(k));

#define DEFK(NAME, INSN, T)                                                                     \
  __global__ __launch_bounds__(256) void thr_##NAME(u64* out, u32 seed, u64* clk) {             \
    u32 k = seed + threadIdx.x;                                                                  \
    T r0 = k, r1 = k + 1, r2 = k + 2, r3 = k + 3, r4 = k + 4, r5 = k + 5, r6 = k + 6,            \
      r7 = k + 7;                                                                                \
    u64 t0 = __builtin_readcyclecounter(), w0 = __builtin_amdgcn_s_memrealtime();               \
    for (int i = 0; i < ITERS; ++i) {                                                            \
      CHAIN8(INSN, T) CHAIN8(INSN, T) CHAIN8(INSN, T) CHAIN8(INSN, T)                            \
    }                                                                                            \
    u64 t1 = __builtin_readcyclecounter(), w1 = __builtin_amdgcn_s_memrealtime();               \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                                   \
      clk[0] = t1 - t0;                                                                          \
      clk[1] = w1 - w0;                                                                          \
    }                                                                                            \
    out[blockIdx.x * 256 + threadIdx.x] =                                                        \
        (u64)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7);                                            \
  }                                                                                              \
  __global__ __launch_bounds__(64) void lat_##NAME(u64* out, u32 seed, u64* clk) {              \
    u32 k = seed + threadIdx.x;                                                                  \
    T r0 = k;                                                                                    \
    u64 t0 = __builtin_readcyclecounter();                                                       \
    for (int i = 0; i < ITERS; ++i) {                                                            \
      CHAIN1(INSN, T) CHAIN1(INSN, T) CHAIN1(INSN, T) CHAIN1(INSN, T)                            \
    }                                                                                            \
    u64 t1 = __builtin_readcyclecounter();                                                       \
    if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;                                   \
    out[blockIdx.x * 64 + threadIdx.x] = (u64)r0;                                                \
  }

DEFK(v_add_u32, "v_add_u32 %0, %0, %1", u32)
DEFK(v_xor_b32, "v_xor_b32 %0, %0, %1", u32)
DEFK(v_lshlrev_b32, "v_lshlrev_b32 %0, %1, %0", u32)
DEFK(v_lshlrev_b64, "v_lshlrev_b64 %0, %1, %0", u64)
DEFK(v_lshrrev_b64, "v_lshrrev_b64 %0, %1, %0", u64)
DEFK(v_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %0", u64)
DEFK(v_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %1, %0", u64)
DEFK(v_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1", u32)
DEFK(v_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1", u32)
DEFK(v_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1", u32)
DEFK(v_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1", u32)
DEFK(v_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0", u32)
DEFK(v_cmp_lt_u64, "v_cmp_lt_u64_e32 vcc, %0, %0", u64)
DEFK(v_cmp_lt_u32, "v_cmp_lt_u32_e32 vcc, %0, %1", u32)
DEFK(v_cndmask_b32, "v_cndmask_b32_e32 %0, %0, %1, vcc", u32)
DEFK(v_add_co_u32, "v_add_co_u32_e32 %0, vcc, %0, %1", u32)
DEFK(v_alignbit_b32, "v_alignbit_b32 %0, %0, %1, %1", u32)
DEFK(v_alignbyte_b32, "v_alignbyte_b32 %0, %0, %1, %1", u32)
DEFK(v_perm_b32, "v_perm_b32 %0, %0, %1, %1", u32)
DEFK(v_bfe_u32, "v_bfe_u32 %0, %0, %1, 8", u32)
DEFK(v_ffbh_u32, "v_ffbh_u32 %0, %0", u32)
DEFK(v_cvt_f32_u32, "v_cvt_f32_u32 %0, %0", u32)
DEFK(v_cvt_u32_f32, "v_cvt_u32_f32 %0, %0", u32)
DEFK(v_rcp_f32, "v_rcp_f32 %0, %0", u32)
DEFK(v_mul_f32, "v_mul_f32 %0, %0, %1", u32)
DEFK(v_lshl_or_b32, "v_lshl_or_b32 %0, %0, 8, %1", u32)
DEFK(v_or3_b32, "v_or3_b32 %0, %0, %1, %0", u32)
DEFK(v_min_u32, "v_min_u32 %0, %0, %1", u32)
DEFK(v_sub_u32, "v_sub_u32 %0, %0, %1", u32)
DEFK(v_cvt_f64_u32, "v_cvt_f64_u32 %0, %1", u64)
DEFK(v_rcp_f64, "v_rcp_f64 %0, %0", u64)
DEFK(v_fma_f64, "v_fma_f64 %0, %0, %0, %0", u64)
DEFK(v_mov_b64, "v_mov_b64 %0, %0", u64)
DEFK(v_lshrrev_b32, "v_lshrrev_b32 %0, %1, %0", u32)

DEFK(v_and_b32, "v_and_b32 %0, %0, %1", u32)
DEFK(v_or_b32, "v_or_b32 %0, %0, %1", u32)
DEFK(v_lshlrev_b32_c, "v_lshlrev_b32 %0, 3, %0", u32)
DEFK(v_lshrrev_b32_c, "v_lshrrev_b32 %0, 3, %0", u32)
DEFK(v_ashrrev_i32, "v_ashrrev_i32 %0, %1, %0", u32)
DEFK(v_max_u32, "v_max_u32 %0, %0, %1", u32)
DEFK(v_subrev_u32, "v_subrev_u32 %0, %0, %1", u32)
DEFK(v_add3_u32, "v_add3_u32 %0, %0, %1, %0", u32)
DEFK(v_lshl_add_u32, "v_lshl_add_u32 %0, %0, 2, %1", u32)
DEFK(v_cndmask_e64, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]", u32)
DEFK(v_bfi_b32, "v_bfi_b32 %0, %0, %1, %0", u32)
DEFK(v_not_b32, "v_not_b32 %0, %0", u32)
DEFK(v_mov_b32, "v_mov_b32 %0, %1", u32)
DEFK(v_add_f32, "v_add_f32 %0, %0, %1", u32)
DEFK(v_fma_f32, "v_fma_f32 %0, %0, %1, %0", u32)
DEFK(v_add_u32_e64, "v_add_u32_e64 %0, %0, %1", u32)
DEFK(v_xor_e64, "v_xor_b32_e64 %0, %0, %1", u32)
DEFK(v_sub_co_u32, "v_sub_co_u32_e32 %0, vcc, %0, %1", u32)
DEFK(v_min_f32, "v_min_f32 %0, %0, %1", u32)
DEFK(v_cmp_e64_u32, "v_cmp_lt_u32_e64 s[2:3], %0, %1", u32)
DEFK(v_mul_u32_u24_b, "v_mul_u32_u24 %0, %0, %1", u32)
DEFK(v_add_u32_b, "v_add_u32 %0, %0, %1", u32)
DEFK(v_lshlrev_b32_b, "v_lshlrev_b32 %0, %1, %0", u32)
DEFK(v_lshrrev_b32_b, "v_lshrrev_b32 %0, %1, %0", u32)
DEFK(mix_add_ffbh, "v_add_u32 %0, %0, %1\n v_ffbh_u32 %0, %0", u32)
DEFK(v_pk_add_u16, "v_pk_add_u16 %0, %0, %1", u32)

// LDS gathers: 64 lanes read random dwords of a 1 KiB / 64 KiB table (bank conflicts included)
template <int MASK>
__global__ __launch_bounds__(256) void thr_lds(u64* out, u32 seed, u64* clk) {
  __shared__ u32 t[16384];
  for (u32 j = threadIdx.x; j < 16384; j += 256) t[j] = j * 2654435761u;
  __syncthreads();
  u32 a0 = (seed + threadIdx.x * 977u) & MASK, a1 = (a0 * 7 + 1) & MASK, a2 = (a0 * 13 + 5) & MASK,
      a3 = (a0 * 31 + 9) & MASK;
  u64 t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a0 = t[a0] & MASK;
      a1 = t[a1] & MASK;
      a2 = t[a2] & MASK;
      a3 = t[a3] & MASK;
    }
  }
  u64 t1 = __builtin_readcyclecounter();
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int wg_per_cu = 8;  // 8 x 4 waves = 8 waves per SIMD
  const int nblk = cus * wg_per_cu;
  u64 *out, *clk;
  hipMalloc(&out, (size_t)nblk * 256 * 8);
  hipMalloc(&clk, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double winst = (double)nblk * 4 * ITERS * 32;  // wave-instructions (thr)
  const double per_simd = winst / (cus * 4.0);
  double ghz = 0;
  printf("%-18s %10s %10s\n", "op", "thr_cyc", "lat_cyc");
#define RUN(NAME)                                                                               \
  {                                                                                             \
    hipLaunchKernelGGL(thr_##NAME, dim3(nblk), dim3(256), 0, 0, out, 1u, clk);                   \
    hipEventRecord(e0);                                                                         \
    hipLaunchKernelGGL(thr_##NAME, dim3(nblk), dim3(256), 0, 0, out, 1u, clk);                   \
    hipEventRecord(e1);                                                                         \
    hipEventSynchronize(e1);                                                                    \
    float ms = 0;                                                                               \
    hipEventElapsedTime(&ms, e0, e1);                                                           \
    u64 h[2];                                                                                   \
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);                                               \
    if (ghz == 0) ghz = (double)h[0] / (double)h[1] * 0.1;                                      \
    const double thr = ms * 1e-3 * ghz * 1e9 / per_simd;                                        \
    hipLaunchKernelGGL(lat_##NAME, dim3(cus * 4), dim3(64), 0, 0, out, 1u, clk);                 \
    hipDeviceSynchronize();                                                                     \
    hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);                                                \
    const double lat = (double)h[0] / (ITERS * 32.0);                                           \
    printf("%-18s %10.2f %10.2f\n", #NAME, thr, lat);                                           \
  }
  RUN(v_add_u32)
  printf("# shader clock %.3f GHz (s_memtime / s_memrealtime)\n", ghz);
  RUN(v_xor_b32) RUN(v_lshlrev_b32) RUN(v_lshrrev_b32) RUN(v_lshlrev_b64) RUN(v_lshrrev_b64)
  RUN(v_lshl_add_u64) RUN(v_mad_u64_u32) RUN(v_mul_lo_u32) RUN(v_mul_hi_u32) RUN(v_mul_u32_u24)
  RUN(v_mul_hi_u32_u24) RUN(v_mad_u32_u24) RUN(v_cmp_lt_u64) RUN(v_cmp_lt_u32) RUN(v_cndmask_b32)
  RUN(v_add_co_u32) RUN(v_alignbit_b32) RUN(v_alignbyte_b32) RUN(v_perm_b32) RUN(v_bfe_u32)
  RUN(v_ffbh_u32) RUN(v_cvt_f32_u32) RUN(v_cvt_u32_f32) RUN(v_rcp_f32) RUN(v_mul_f32)
  RUN(v_lshl_or_b32) RUN(v_or3_b32) RUN(v_min_u32) RUN(v_sub_u32) RUN(v_cvt_f64_u32)
  RUN(v_rcp_f64) RUN(v_fma_f64) RUN(v_mov_b64)
  RUN(v_and_b32) RUN(v_or_b32) RUN(v_lshlrev_b32_c) RUN(v_lshrrev_b32_c) RUN(v_ashrrev_i32)
  RUN(v_max_u32) RUN(v_subrev_u32) RUN(v_add3_u32) RUN(v_lshl_add_u32) RUN(v_cndmask_e64)
  RUN(v_bfi_b32) RUN(v_not_b32) RUN(v_mov_b32) RUN(v_add_f32) RUN(v_fma_f32) RUN(v_add_u32_e64)
  RUN(v_xor_e64) RUN(v_sub_co_u32) RUN(v_min_f32) RUN(v_cmp_e64_u32) RUN(v_mul_u32_u24_b)
  RUN(v_add_u32_b) RUN(v_lshlrev_b32_b) RUN(v_lshrrev_b32_b) RUN(mix_add_ffbh) RUN(v_pk_add_u16)
#define RUN_LDS(MASK)                                                                           \
  {                                                                                             \
    hipLaunchKernelGGL(thr_lds<MASK>, dim3(nblk / 2), dim3(256), 0, 0, out, 1u, clk);            \
    hipEventRecord(e0);                                                                         \
    hipLaunchKernelGGL(thr_lds<MASK>, dim3(nblk / 2), dim3(256), 0, 0, out, 1u, clk);            \
    hipEventRecord(e1);                                                                         \
    hipEventSynchronize(e1);                                                                    \
    float ms = 0;                                                                               \
    hipEventElapsedTime(&ms, e0, e1);                                                           \
    const double n = (double)(nblk / 2) * 4 * ITERS * 32 / (cus * 4.0);                         \
    printf("%-18s %10.2f %10s  (random ds_read_b32 over %d dwords, 4 waves/SIMD)\n",            \
           "lds_gather", ms * 1e-3 * ghz * 1e9 / n, "-", MASK + 1);                             \
  }
  RUN_LDS(255) RUN_LDS(16383)
  return 0;
}
