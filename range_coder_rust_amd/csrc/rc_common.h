// rc_common.h — definitions shared by the kernels of librc_amd.so (internal, not installed).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/range_coder.h"

typedef uint64_t u64;
typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32 u32x3 __attribute__((ext_vector_type(3)));

#define TOP16 (1ull << 48)  // range_coder.rs:24

// VGPR allocation floor.  On this gfx950 stack a kernel allocated 88 VGPRs (an odd number of
// 8-register granules) corrupts co-resident waves on the same SIMD, while the identical
// instruction stream allocated 96 VGPRs is correct.  Each kernel clobbers a
// register so its allocation is a multiple of 16; build() rejects any other count.
#define RC_VGPR_FLOOR_32() asm volatile("; vgpr floor 32" ::: "v31")
#define RC_VGPR_FLOOR_48() asm volatile("; vgpr floor 48" ::: "v47")
#define RC_VGPR_FLOOR_64() asm volatile("; vgpr floor 64" ::: "v63")
#define RC_VGPR_FLOOR_96() asm volatile("; vgpr floor 96" ::: "v95")
#define RC_VGPR_FLOOR_80() asm volatile("; vgpr floor 80" ::: "v79")
#define RC_VGPR_FLOOR_112() asm volatile("; vgpr floor 112" ::: "v111")
#define RC_VGPR_FLOOR_128() asm volatile("; vgpr floor 128" ::: "v127")
#define RC_VGPR_FLOOR_144() asm volatile("; vgpr floor 144" ::: "v143")
#define RC_VGPR_FLOOR_160() asm volatile("; vgpr floor 160" ::: "v159")

// Scratch builds only ("what binds"): -DRC_FILL=n adds n filler VALU
// instructions to every symbol step of the static coders, each dependent only on the previous
// filler (their register is carried in the coder state).  If the step is bound by VALU issue
// the kernel slows by n x the filler's issue cost per wave-symbol; if it waits on latency, the
// fillers ride in idle issue slots.  -DRC_FILL_OP picks the instruction, so the marginal cost
// of each instruction class can be measured inside the real kernels (tools/fill_cost.sh).
#ifdef RC_FILL
#ifndef RC_FILL_OP
#define RC_FILL_OP 0
#endif
// the filler register: a VGPR pair for the 64-bit instructions, one VGPR otherwise; the scalar
// and branch fillers (RC_FILL_OP >= 20) carry an SGPR, the LDS filler a VGPR address
#if RC_FILL_OP >= 20 && RC_FILL_OP < 24
struct rc_fill_t {
  u32 x;
  __device__ rc_fill_t& operator=(int v) { x = (u32)v; return *this; }
};
static __device__ __forceinline__ void rc_filler_one(rc_fill_t& f) {
  switch (RC_FILL_OP) {
    // (a fixed SGPR, clobbered: a state member would turn divergent at the decoders' redo
    // paths and could not stay scalar)
    case 20: asm volatile("s_add_u32 s100, s100, 1" ::: "s100", "scc"); break;              // SALU
    case 21: asm volatile("s_cmp_eq_u32 s100, 1\n\ts_cbranch_scc1 0" ::: "s100", "scc"); break;  // SALU + branch
    case 22: asm volatile("s_cmp_eq_u32 s100, 1" ::: "s100", "scc"); break;                 // the SALU of 21
    default: {  // 23: one LDS read of a table word, waited for by its consumer (a VALU add)
      const u32 w = *(const volatile __attribute__((address_space(3))) u32*)(uintptr_t)(f.x & 0xFCu);
      f.x += w;
    }
  }
}
#else
#if RC_FILL_OP == 2 || RC_FILL_OP == 3 || RC_FILL_OP == 5 || RC_FILL_OP == 8 || RC_FILL_OP == 16
typedef u64 rc_fill_t;
#else
typedef u32 rc_fill_t;
#endif
static __device__ __forceinline__ void rc_filler_one(u64& x) {
  u64 c;
  switch (RC_FILL_OP) {
    case 2: asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x)); break;
    case 3: asm volatile("v_mad_u64_u32 %0, %1, %2, %2, %0" : "+v"(x), "=s"(c) : "v"((u32)(x >> 7))); break;
    case 5: asm volatile("v_cmp_gt_u64_e64 %0, %1, %1" : "=s"(c) : "v"(x)); break;
    case 8: asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(x)); break;
    default: asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x)); break;
  }
}
static __device__ __forceinline__ void rc_filler_one(u32& x) {
  u64 c;
  switch (RC_FILL_OP) {
    case 0: asm volatile("v_add_u32 %0, 1, %0" : "+v"(x)); break;
    case 1: asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(x)); break;
    case 4: asm volatile("v_mad_u32_u24 %0, %0, %0, %0" : "+v"(x)); break;
    case 6: asm volatile("v_alignbit_b32 %0, %0, %0, %0" : "+v"(x)); break;
    case 7: asm volatile("v_perm_b32 %0, %0, %0, %0" : "+v"(x)); break;
    case 9: asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x)); break;
    case 10: asm volatile("v_bfe_u32 %0, %0, 1, 8" : "+v"(x)); break;
    case 11: asm volatile("v_lshl_add_u32 %0, %0, 3, %0" : "+v"(x)); break;
    case 12: asm volatile("v_ffbh_u32 %0, %0" : "+v"(x)); break;
    case 13: asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x)); break;
    case 14: asm volatile("v_cmp_gt_u32_e64 %0, %1, %1" : "=s"(c) : "v"(x)); break;
    // a compare into VCC and a select reading it, against the same through an SGPR pair (the
    // pair is the price DESIGN.md §5 gives a VCC read, measured in isolation in round 1)
    // (with the 2 wait states a VALU read of a VALU-written SGPR needs on gfx950)
    case 24: asm volatile("v_cmp_lt_u32_e32 vcc, 1, %0\n\ts_nop 1\n\tv_cndmask_b32_e32 %0, 1, %0, vcc" : "+v"(x) : : "vcc"); break;
    case 25: asm volatile("v_cmp_lt_u32_e64 %1, 1, %0\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, 1, %0, %1" : "+v"(x), "=s"(c)); break;
    case 15: asm volatile("v_mul_f32 %0, %0, %0" : "+v"(x)); break;
    default: asm volatile("v_xor_b32 %0, 1, %0" : "+v"(x)); break;
  }
}
#endif
#define RC_FILLER(x)                                                   \
  do {                                                                 \
    _Pragma("unroll") for (int i_ = 0; i_ < RC_FILL; ++i_)             \
        rc_filler_one(x);                                              \
  } while (0)
#else
#define RC_FILLER(x) \
  do {               \
  } while (0)
#endif

// Scratch builds only (-DRC_STAMP, tools/stamp_probe.py): per-wave stamps.  Lane 0
// of every wave records the constant 100 MHz clock (s_memrealtime) and the shader clock
// (s_memtime) at kernel entry and exit, with HW_ID and XCC_ID, into a buffer of its translation
// unit; rc_stamp_read_<tu>() copies the records out and clears them.  Vector stores only.
struct RcStamp {
  u64 rt0, rt1;  // s_memrealtime at entry / exit (100 MHz, one clock for the whole device)
  u64 c0, c1;    // s_memtime at entry / exit (shader cycles)
  u32 hwid, xcc; // HW_REG_HW_ID, HW_REG_XCC_ID
  u32 nsym, pad; // symbols of lane 0's chunk
};
#define RC_STAMP_SLOTS 65536u
#ifdef RC_STAMP
#define RC_STAMP_DEFINE(tu)                                                                  \
  static __device__ RcStamp g_stamp_##tu[RC_STAMP_SLOTS];                                    \
  extern "C" int rc_stamp_read_##tu(void* dst, size_t n) {                                   \
    if (n > RC_STAMP_SLOTS) n = RC_STAMP_SLOTS;                                              \
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamp_##tu), n * sizeof(RcStamp)) != hipSuccess) \
      return -1;                                                                             \
    static RcStamp zero[1024];                                                               \
    for (size_t i = 0; i < RC_STAMP_SLOTS; i += 1024)                                        \
      if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_##tu), zero, sizeof(zero), i * sizeof(RcStamp)) \
          != hipSuccess)                                                                     \
        return -1;                                                                           \
    return (int)n;                                                                           \
  }
#define RC_STAMP_BEGIN()                                  \
  const u64 st_rt0_ = __builtin_amdgcn_s_memrealtime(); \
  const u64 st_c0_ = __builtin_amdgcn_s_memtime()
#define RC_STAMP_END(tu, slot, lane, nsym_) RC_STAMP_END_(tu, slot, lane, nsym_)
#define RC_STAMP_END_(tu, slot, lane, nsym_)                                         \
  do {                                                                               \
    const u64 st_c1_ = __builtin_amdgcn_s_memtime();                                 \
    const u64 st_rt1_ = __builtin_amdgcn_s_memrealtime();                            \
    if ((lane) == 0 && (slot) < RC_STAMP_SLOTS) {                                    \
      RcStamp* p_ = &g_stamp_##tu[slot];                                             \
      p_->rt0 = st_rt0_;                                                             \
      p_->rt1 = st_rt1_;                                                             \
      p_->c0 = st_c0_;                                                               \
      p_->c1 = st_c1_;                                                               \
      p_->hwid = __builtin_amdgcn_s_getreg(0xF804); /* HW_ID, 32 bits */              \
      p_->xcc = __builtin_amdgcn_s_getreg(0xF814);  /* XCC_ID */                      \
      p_->nsym = (u32)(nsym_);                                                       \
      p_->pad = 1u;                                                                  \
    }                                                                                \
  } while (0)
#else
#define RC_STAMP_DEFINE(tu)
#define RC_STAMP_BEGIN() \
  do {                   \
  } while (0)
#define RC_STAMP_END(tu, slot, lane, nsym) \
  do {                                     \
  } while (0)
#endif

static __device__ __forceinline__ u32 hi32(u64 v) { return (u32)(v >> 32); }

// a - b (64-bit) with the borrow in an SGPR pair: the compiler's v_subb_co_u32_e32 reads VCC,
// and a VALU read of VCC costs ~13 extra SIMD cycles on gfx950 (tools/ubench_issue.hip).
// A VALU write of an SGPR read by a VALU as its carry-in needs 2 wait states on gfx950 (hipcc
// pads its own v_sub_co -> v_subb_co_e64 pairs with them; it pads nothing inside an asm
// string): the s_nop 1 between the two.  Without it the borrow may be read stale
// (DESIGN.md §6).
static __device__ __forceinline__ u64 sub64(u64 a, u64 b) {
  u32 lo, hi;
  u64 c;
  asm("v_sub_co_u32_e64 %0, %2, %3, %4\n\ts_nop 1\n\tv_subb_co_u32_e64 %1, %2, %5, %6, %2"
      : "=&v"(lo), "=&v"(hi), "=&s"(c)
      : "v"((u32)a), "v"((u32)b), "v"(hi32(a)), "v"(hi32(b)));
  return ((u64)hi << 32) | lo;
}
// the same with a given as two halves (no register pair needed for it)
static __device__ __forceinline__ u64 sub64(u32 alo, u32 ahi, u64 b) {
  u32 lo, hi;
  u64 c;
  asm("v_sub_co_u32_e64 %0, %2, %3, %4\n\ts_nop 1\n\tv_subb_co_u32_e64 %1, %2, %5, %6, %2"
      : "=&v"(lo), "=&v"(hi), "=&s"(c)
      : "v"(alo), "v"((u32)b), "v"(ahi), "v"(hi32(b)));
  return ((u64)hi << 32) | lo;
}

// (m & a) | (~m & b) for a mask m of 0 / ~0: one v_bfi_b32, written out.  From the C form the
// compiler turns selects on masks back into v_cmp + v_cndmask_b32 on VCC (a VALU read of VCC
// costs ~13 extra SIMD cycles), or narrows selects of u16 values to 16-bit
// xor / and / bitop3 sequences and re-extends their results.
static __device__ __forceinline__ u32 msel(u32 m, u32 a, u32 b) {
  u32 r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// msel from C: with the mask opaque (smask, or masks the compiler cannot trace to a compare) it
// compiles to one v_bfi_b32 / v_bitop3_b32, and unlike the asm form its consumers are not padded
// (the hazard recognizer cannot see into inline asm, so it puts an s_nop before the next
// dependent VOP1/VOP2 instruction)
static __device__ __forceinline__ u32 mselc(u32 m, u32 a, u32 b) { return (a & m) | (b & ~m); }

// the sign of v as a mask (0 / ~0), opaque to the compiler (which otherwise turns selects on it
// back into v_cmp + v_cndmask_b32 on VCC)
static __device__ __forceinline__ u32 smask(u32 v) {
  u32 r;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(r) : "v"(v));
  return r;
}

// Global (not flat) memory access.  A flat access also counts in lgkmcnt, so every LDS wait
// would wait for it too; pointers that pass through LDS or integer casts lose their address
// space and compile to flat unless cast back like this.
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) u32 g_u32;
typedef __attribute__((address_space(1))) u64 g_u64;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
static __device__ __forceinline__ u32 gload(const u32* p) { return *(const g_u32*)p; }
static __device__ __forceinline__ u64 gload64(const u64* p) { return *(const g_u64*)p; }
static __device__ __forceinline__ u32x4 gload16(const u32x4* p) { return *(const g_u32x4*)p; }
static __device__ __forceinline__ void gstore8(uint8_t* p, u32 v) { *(g_u8*)p = (uint8_t)v; }
static __device__ __forceinline__ void gstore32(uint8_t* p, u32 v) { *(g_u32*)p = v; }
static __device__ __forceinline__ void gstore64(uint8_t* p, u64 v) { *(g_u64*)p = v; }
static __device__ __forceinline__ void gstore128(uint8_t* p, u32x4 v) { *(g_u32x4*)p = v; }

// A pinned host buffer of at least `bytes` (<= 1 MiB) for this host thread, grown on demand
// (rc_kernels.hip).  Host <-> device transfers of small control data go through it: async
// copies to and from pageable memory returned wrong bytes intermittently on this stack
// (DESIGN.md §6), pinned ones are plain stream-ordered DMA.  Contents are the caller's until
// its next call on the same thread.
void* rc_pinned_scratch_(size_t bytes);

// Adaptive order-0 model parameters (rc_model_create_adaptive)
struct AdaptParams {
  u32 n;      // alphabet size (1..256)
  u32 inc;    // count increment per coded symbol
  u32 limit;  // halve the counts when the total exceeds this ...
  u32 pmask;  // ... at every period-th symbol (period = pmask + 1, a power of two)
  const u64* magic;  // [65536]: floor((2^64 - 1) / t) for range / t (model-owned, device)
};

// rc_adaptive.hip: launches on `stream`; validate arguments before calling
hipError_t rc_adaptive_encode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* syms, const u64* sym_off, u32 n_chunks,
                                     uint8_t* out, const u64* out_off, u64* out_len,
                                     u32* flags);
hipError_t rc_adaptive_decode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* code, const u64* code_off,
                                     const u64* code_len, uint8_t* syms_out, const u64* sym_off,
                                     u32 n_chunks, u32* flags);

// Run-time switches (include/range_coder.h, "Environment"): read from the environment ONCE per
// context, by rc_ctx_create, and carried by the context.  Nothing reads the environment per
// launch or per call, so a stray variable set later cannot change a live context.  One kill
// switch per feature; the measurement overrides of earlier rounds are compile-time options of
// scratch builds (-DRC_PRIO_LAST=x, -DRC_PRIO_RANK, -DRC_PRIO_ROT=k, -DRC_DEC_LDS_PAD=bytes,
// -DRC_STREAM_COPY_WGS=n).
struct RcKnobs {
  bool prio;               // RC_PRIO=off: every wave at priority 0 (oldest-first issue)
  u32 dec_pair;            // RC_DEC_PAIR=512 | 1024: the pair-bucket decoder (LUT 3) for the
                           //   models that carry its table (tests and measurements)
  bool stream_service;     // RC_STREAM_SERVICE=0: the per-call stream API always launches
  bool stream_dma;         // RC_STREAM_DMA=1: the host pipeline moves everything by DMA
  bool stream_direct;      // RC_STREAM_DIRECT=0: the host pipeline stages outputs in HBM
  u64 stream_batch_bytes;  // RC_STREAM_BATCH_BYTES=n: the host pipeline's batch size (0: default)
  bool hist_hot;           // RC_HIST_HOT=0: the histogram without its ballot-counted hot symbol
};
RcKnobs rc_knobs_from_env();                      // rc_kernels.hip (rc_ctx_create only)
// rc_resume.hip: ask the process's stream-service waves to leave before a batch launch (a
// resident wave would hold the hardware queue its stream shares with the launch's)
void rc_svc_yield_all_();
const RcKnobs& rc_ctx_knobs_(const rc_ctx* ctx);  // rc_kernels.hip
