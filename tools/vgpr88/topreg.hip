// tools/vgpr88/topreg.hip — isolate the co-resident corruption in a few
// instructions.
//
// patchrun / rename.py showed: the round-1 encoder goes wrong, on every wave whose VGPR block
// does not start at physical register 0, exactly when its `nbits` register — read as the 32-bit
// shift amount of v_lshrrev_b64 — is the LAST register of the allocation.  Here each kernel
// keeps a shift amount in register vT and runs a loop of one 64-bit (or, as a control, 32-bit)
// instruction reading it; T = 63 is the top of a 64-register allocation, T = 62 / 59 are not.
// Every lane's result is checked on the host, per VGPR base (HW_REG_GPR_ALLOC).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#define STR_(x) #x
#define STR(x) STR_(x)

// One kernel per case.  S: the register holding the cycling 32-bit operand s; X0:X1 the pair
// holding the 64-bit operand x; OPLINE computes v[4:5] from them.  The compiler's own registers
// stay below 56, so the allocation is max(S, X1) + 1 rounded up to 8 (64 for every case here).
#define TOPREG_KERNEL(NAME, S, X0, X1, OPLINE)                                                 \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t* alloc, uint32_t iters) { \
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;                                        \
    const uint32_t lo = 0x9E3779B9u * (g + 1), hi = 0x85EBCA6Bu ^ g, s0 = g & 63;             \
    uint32_t r0, r1;                                                                          \
    asm volatile(                                                                             \
        "v_mov_b32 v" STR(S) ", %2\n\t"                                                       \
        "v_mov_b32 v" STR(X0) ", %3\n\t"                                                      \
        "v_mov_b32 v" STR(X1) ", %4\n\t"                                                      \
        "v_mov_b32 v6, 0\n\t"                                                                 \
        "v_mov_b32 v7, 0\n\t"                                                                 \
        "s_mov_b32 s40, %5\n"                                                                 \
        "1:\n\t" OPLINE "\n\t"                                                                \
        "v_xor_b32 v6, v6, v4\n\t"                                                            \
        "v_xor_b32 v7, v7, v5\n\t"                                                            \
        "v_add_u32 v" STR(S) ", 1, v" STR(S) "\n\t"                                           \
        "v_and_b32 v" STR(S) ", 63, v" STR(S) "\n\t"                                          \
        "s_sub_u32 s40, s40, 1\n\t"                                                           \
        "s_cmp_lg_u32 s40, 0\n\t"                                                             \
        "s_cbranch_scc1 1b\n\t"                                                               \
        "v_mov_b32 %0, v6\n\t"                                                                \
        "v_mov_b32 %1, v7"                                                                    \
        : "=v"(r0), "=v"(r1)                                                                  \
        : "v"(s0), "v"(lo), "v"(hi), "s"(iters)                                               \
        : "v4", "v5", "v6", "v7", "v" STR(S), "v" STR(X0), "v" STR(X1), "v56", "s40", "s41",   \
          "s42", "s43", "scc");                                                               \
    out[2 * g] = r0;                                                                          \
    out[2 * g + 1] = r1;                                                                      \
    if ((threadIdx.x & 63) == 0) alloc[g >> 6] = __builtin_amdgcn_s_getreg(0xF805);           \
  }

// 64-bit shifts, the amount (32-bit src0) in the top register v63: the round-1 encoder's case
TOPREG_KERNEL(k_shr64_t63, 63, 2, 3, "v_lshrrev_b64 v[4:5], v63, v[2:3]")
TOPREG_KERNEL(k_shr64_t62, 62, 2, 3, "v_lshrrev_b64 v[4:5], v62, v[2:3]")
TOPREG_KERNEL(k_shr64_t59, 59, 2, 3, "v_lshrrev_b64 v[4:5], v59, v[2:3]")
TOPREG_KERNEL(k_shl64_t63, 63, 2, 3, "v_lshlrev_b64 v[4:5], v63, v[2:3]")
TOPREG_KERNEL(k_asr64_t63, 63, 2, 3, "v_ashrrev_i64 v[4:5], v63, v[2:3]")
// 32-bit ops reading v63 (controls)
TOPREG_KERNEL(k_shr32_t63, 63, 2, 3, "v_lshrrev_b32 v4, v63, v2\n\tv_mov_b32 v5, v3")
TOPREG_KERNEL(k_align_t63, 63, 2, 3, "v_alignbit_b32 v4, v3, v2, v63\n\tv_mov_b32 v5, v3")
// other 64-bit results with v63 as a 32-bit source
TOPREG_KERNEL(k_mad64_t63, 63, 2, 3, "v_mad_u64_u32 v[4:5], s[42:43], v63, v2, v[2:3]")
TOPREG_KERNEL(k_mad64_t62, 62, 2, 3, "v_mad_u64_u32 v[4:5], s[42:43], v62, v2, v[2:3]")
TOPREG_KERNEL(k_cvtf64_t63, 63, 2, 3, "v_cvt_f64_u32 v[4:5], v63")
// the 64-bit operand in the top pair v[62:63], the amount in v8
TOPREG_KERNEL(k_shr64_x63, 8, 62, 63, "v_lshrrev_b64 v[4:5], v8, v[62:63]")
TOPREG_KERNEL(k_mov64_x63, 8, 62, 63, "v_mov_b64 v[4:5], v[62:63]")
// the 64-bit shift's destination in the top pair
TOPREG_KERNEL(k_shr64_d63, 8, 2, 3,
              "v_lshrrev_b64 v[62:63], v8, v[2:3]\n\tv_mov_b32 v4, v62\n\tv_mov_b32 v5, v63")
// the same instruction with the amount in v55 and v56 named (allocation 64, v63 unused)
TOPREG_KERNEL(k_shr64_t55, 55, 2, 3, "v_lshrrev_b64 v[4:5], v55, v[2:3]")

typedef void (*kfn)(uint32_t*, uint32_t*, uint32_t);

static uint64_t expect(uint32_t g, uint32_t iters, int op) {
  const uint64_t x = ((uint64_t)(0x85EBCA6Bu ^ g) << 32) | (uint32_t)(0x9E3779B9u * (g + 1));
  uint32_t s = g & 63;
  uint64_t acc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    uint64_t r;
    switch (op) {
      case 0: r = x >> s; break;
      case 1: r = x << s; break;
      case 2: r = (uint64_t)((int64_t)x >> s); break;
      case 3: r = ((uint64_t)(uint32_t)x >> (s & 31)) | (x & 0xFFFFFFFF00000000ull); break;
      case 4: r = (uint64_t)s * (uint32_t)x + x; break;
      case 5: r = (uint32_t)(x >> (s & 31)) | (x & 0xFFFFFFFF00000000ull); break;
      case 6: {
        const double d = (double)s;
        memcpy(&r, &d, 8);
        break;
      }
      default: r = x; break;
    }
    acc ^= r;
    s = (s + 1) & 63;
  }
  return acc;
}

int main(int argc, char** argv) {
  const uint32_t wgs = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 0) : 2048;
  const uint32_t iters = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 0) : 20000;
  struct V {
    const char* name;
    kfn f;
    int op;
  } vs[] = {{"shr64 amt v63 (top)", k_shr64_t63, 0}, {"shr64 amt v62", k_shr64_t62, 0},
            {"shr64 amt v59", k_shr64_t59, 0},       {"shl64 amt v63 (top)", k_shl64_t63, 1},
            {"asr64 amt v63 (top)", k_asr64_t63, 2}, {"shr32 amt v63 (top)", k_shr32_t63, 3},
            {"alignbit v63 (top)", k_align_t63, 5},  {"mad64 src v63 (top)", k_mad64_t63, 4},
            {"mad64 src v62", k_mad64_t62, 4},       {"cvt_f64 src v63 (top)", k_cvtf64_t63, 6},
            {"shr64 x v[62:63]", k_shr64_x63, 0},    {"mov64 x v[62:63]", k_mov64_x63, 7},
            {"shr64 dst v[62:63]", k_shr64_d63, 0},  {"shr64 amt v55, v56 named", k_shr64_t55, 0}};
  const uint32_t n = wgs * 256;
  uint32_t *dout, *dal;
  if (hipMalloc(&dout, 8ull * n) != hipSuccess || hipMalloc(&dal, 4ull * (n / 64)) != hipSuccess)
    return 1;
  std::vector<uint32_t> out(2ull * n), al(n / 64);
  for (const V& v : vs) {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, (const void*)v.f);
    hipLaunchKernelGGL(v.f, dim3(wgs), dim3(256), 0, 0, dout, dal, iters);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("%s: launch failed\n", v.name);
      return 1;
    }
    (void)hipMemcpy(out.data(), dout, 8ull * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(al.data(), dal, 4ull * (n / 64), hipMemcpyDeviceToHost);
    std::map<uint32_t, std::pair<uint32_t, uint32_t>> by;  // vgpr base -> (waves, bad waves)
    uint32_t bad = 0;
    for (uint32_t w = 0; w < n / 64; ++w) {
      uint32_t wb = 0;
      for (uint32_t g = 64 * w; g < 64 * w + 64; ++g) {
        const uint64_t e = expect(g, iters, v.op);
        if (out[2 * g] != (uint32_t)e || out[2 * g + 1] != (uint32_t)(e >> 32)) ++wb;
      }
      bad += wb;
      auto& b = by[(al[w] & 63) * 8];
      b.first++;
      b.second += wb != 0;
    }
    printf("%-18s vgprs %3d: bad lanes %u of %u\n", v.name, fa.numRegs, bad, n);
    for (auto& kv : by)
      printf("    vgpr base %3u: waves %5u bad %5u\n", kv.first, kv.second.first, kv.second.second);
  }
  return 0;
}
