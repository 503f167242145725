// rc_static.h — shared definitions of the static-model kernels (rc_encode.hip, rc_decode.inc).
//
// One independent stream ("chunk", a fresh reference Encoder/Decoder) per lane; 64 chunks per
// wave run the reference's sequential per-symbol loop in lock-step.  The arithmetic restates
// src/range_coder.rs (param_update :53-92, left_shift :95-100, no_carry_expansion :110-116,
// range_reduction_expansion :126-135), src/encoder.rs (encode :24-37, finish :40-46) and
// src/decoder.rs (new :14-23, decode :38-54) bit-exactly, with these MI355X-specific choices:
//  * coder state (lower_bound, range, decoder data window) lives in VGPR pairs;
//  * the PModel snapshot (cum, c) and the decoder's inverse-CDF table live in LDS;
//  * the no-carry loop (range_coder.rs:83-85) is evaluated in closed form: it settles exactly
//    k = clz64(low ^ (low + range)) / 8 bytes (proof in DESIGN.md §3), so the wave does not
//    diverge on it;
//  * range / total (range_coder.rs:38-40) is a shift for power-of-two totals and an exact
//    multiply-high by a host-computed reciprocal otherwise (no 64-bit divide on the VALU);
//  * the decoder's find_index division + binary search (sample_impl.rs:27-45) is replaced by a
//    float hint -> LDS inverse-CDF table -> exact integer verification r*cum[s] <= data-low <
//    r*cum[s+1], which yields the same index for every input, valid or corrupt;
//  * encoder: symbols are read 64 B per lane per tile; settled bytes go through a per-lane LDS
//    ring and are written by cooperative flush rounds, 16 chunks x 64 B per store instruction;
//  * decoder: the code is read 64 B per lane into a per-lane LDS ring one 16-symbol phase
//    ahead; decoded symbols are written 16 B per lane per phase.
#pragma once
#include "rc_common.h"

#include <stdlib.h>
#include <string.h>

#define WG 256
#define WAVES (WG / 64)
#define ENC_RING 32          // dwords per lane in the encoder's output ring (128 B)
#ifndef DEC_RING
#define DEC_RING 16          // dwords per lane in the decoder's input ring (64 B)
#endif
#ifndef DEC_MIRROR
#define DEC_MIRROR 2         // mirror slots past the ring, so a 3-dword read never wraps
#endif
#define DEC_RING_ALLOC (DEC_RING + DEC_MIRROR)
#ifndef DEC_PF
#define DEC_PF 2             // 16-B blocks per ring refill (32 B, one 16-symbol phase ahead)
#endif
#ifndef DEC_LD
#define DEC_LD 4             // 16-B blocks per global load burst (64 B: two refills)
#endif
#ifndef DEC_PAIR512_LD
#define DEC_PAIR512_LD DEC_LD  // load burst of the 512-lane pair decoder (2 waves/SIMD shapes)
#endif
#ifndef DEC_OUT_BURST
#define DEC_OUT_BURST 4      // 16-B symbol blocks per lane per output burst (4: 64 B)
#endif
#ifndef DEC_SPEC
#define DEC_SPEC 1           // every SM decoder takes the speculative step (verify deferred)
#endif
#ifndef ENC_PAIR
#define ENC_PAIR 1           // small-model encoders test the rare path once per two symbols
#endif
#ifndef DEC_SEL_FILL
#define DEC_SEL_FILL 1       // LUT 4 (pow2): the select's wait states do useful work (round 6)
#endif
#ifndef DEC_CHECK_SPAN
#define DEC_CHECK_SPAN 8     // small-model decoders: symbols between ring checks in a phase
#endif
#ifndef DEC_TAB_LDS
#define DEC_TAB_LDS 1        // direct-LUT decoders: keep the (cum, c) table in LDS too
#endif
#ifdef RC_RING_GUARD
// scratch builds only (not part of the C ABI): a decoder read code bytes its ring had not staged
#define RC_F_RING_GUARD 0x100u
#endif
#define LUT_BITS 12
#define LUT_MAX_ENTRIES (1u << LUT_BITS)
#ifndef SM_LUT_BITS
// buckets of small models (total <= 2^16).  11 bits would keep LUT + table + rings of a
// 256-lane workgroup at 30 KiB, 5 workgroups (5 waves per SIMD) per CU instead of 4; measured
// within 0.5% at 2^20 chunks (3.2 rounds of resident lanes instead of 4)
#define SM_LUT_BITS 12
#endif

enum { DIV_POW2 = 0, DIV_MAGIC = 1 };

struct ModelArgs {
  const uint2* tab;  // [256] (cum, c); entries s >= n_symbols hold (0xFFFFFFFF, 0)
  const u32* lut;    // decoder buckets: s0 | s1 << 8 | split << 16 (small models, total <=
                     // 2^16: s0 | s1 << 8 | cum[s1] << 16, and s1 = s0 without a split)
  u64 magic;         // floor((2^64 - 1) / total) for DIV_MAGIC
  u32 n;             // alphabet size (1..256)
  u32 total;         // total_freq
  u32 lg;            // log2(total) for DIV_POW2
  u32 lut_shift;     // bucket = q >> lut_shift
  u32 lut_max;       // number of buckets - 1
  u32 lut_bits;      // bucket tables: log2(buckets) (LUT_BITS, or SM_LUT_BITS for small models)
  float ftotal;      // (float)total
  u32 direct;        // 1: lut[q] = s | cum << 8 | c << 20 for every q < total (total <= 2048)
                     // 2: lut[4q..4q+3] = {cum, c, s, total/c as f32} (256 <= total <= 512)
  const u32* pair;   // pair-bucket tables (k_decode_static LUT 3; null when the model has none):
                     // PAIR_S_WORDS words of {s0 | s1 << 8} (u16 per bucket), then one 16-B
                     // entry per bucket {cum0 | c0 << 16, cum1 | c1 << 16, total/c0, total/c1}
  u32 la_shift;      // small bucket models (LUT 4): bucket byte address = (q >> la_shift) & la_mask
  u32 la_mask;
  float la_magic;    // 1.5 * 2^(23 + la_shift): fma(X, G, la_magic)'s low bits are q >> la_shift
  double inv_up;     // 1 / total rounded up (small models, DIV_MAGIC: range / total in f64)
  u32 prio_base;     // set per launch (rc_prio_policy): workgroup b >= prio_base runs at
  u32 prio_step;     //   s_setprio min(3, 1 + (b - prio_base) / prio_step); ~0: all at 0
  u32 prio_rot;      // set per launch: 0, or rotate priorities every 2^prio_rot ticks of the
                     // 100 MHz clock (rc_prio_rotate)
  u32 flat;          // 1: the flat model (256 symbols, every c = 1, total 256): cum[s] = s, so
                     // the coders need no table (k_decode_static LUT 5, k_encode_static FLAT)
};

// Wave priority ("the end of a launch").  Every chunk is one lane's serial stream
// and the chunks are of equal length, so a launch ends with a ramp-down in which the waves
// dispatched last run with fewer and fewer partners per SIMD.  Issue is arbitrated by priority,
// then age: at equal priority the oldest wave of a SIMD runs nearly unimpeded and the youngest
// takes the leftover slots, which stretches the end of the launch.  Two remedies, set per
// launch by rc_prio_policy from the kernel's residency R (workgroups the chip holds at once):
//  * static: the workgroups of the last rounds run at a higher priority, so the last-dispatched
//    waves catch up with the older ones instead of finishing alone;
//  * rotating (rc_prio_rotate): every 64 symbols a wave sets its priority to ((t >> k) + its
//    wave slot) mod 4, t = s_memrealtime.  The waves of a SIMD hold distinct slots (HW_ID wave
//    id), so at any moment they hold different priorities and each takes every priority in
//    turn: issue goes round-robin at 2^k x 10 ns granularity instead of oldest-first, and waves
//    that started together finish together (the two waves of one 512-lane workgroup on a SIMD,
//    whose slots are released together; rounds that divide the grid evenly).
// Control: RC_PRIO=off in the environment of rc_ctx_create (RcKnobs) turns priorities off;
// scratch builds override every kernel's default at compile time: -DRC_PRIO_LAST=x (the last x
// rounds at priority 1, x may be fractional), -DRC_PRIO_RANK (the last three rounds at 1, 2, 3),
// -DRC_PRIO_ROT=k (rotation every 2^k ticks, 0 off).
struct PrioPolicy {
  float last_rounds;  // > 0: the last last_rounds x R workgroups at priority 1
  bool rank;          // the last three rounds at 1, 2, 3
  u32 rot;            // rotation shift (0: none; kRotAuto: 10 if the grid fits one round, else 12)
};
static constexpr u32 kRotAuto = 0xFFu;
// The kernels' defaults, from same-box stamp runs at 2^20 and 2^17 chunks (DESIGN.md §5,
// "wave priorities"; profiles/r05/prio_c/):
//  * encoder (4 waves per SIMD, 16 per SIMD in all at 2^20: four even rounds): rotation every
//    2^12 ticks (uniform encode -3.1%, Zipf -3.1%, 2^17 -3.8%);
//  * 256-lane decoders (5 waves per SIMD: 3.2 rounds): the last round at priority 1 (uniform
//    decode -2.2%; rotation makes their rounds end together and the last 0.2 round alone, +4%);
//  * 512-lane small-model decoder (two waves of one workgroup per SIMD): rotation, every 2^12
//    ticks over several rounds (Zipf decode -5.8%), 2^10 when the grid is one round (the 2^17
//    shard, -4.0%).
static constexpr PrioPolicy kPrioEncoder{0.0f, false, 12u};
static constexpr PrioPolicy kPrioDecoder{1.0f, false, 0u};
static constexpr PrioPolicy kPrioDecoder512{0.0f, false, kRotAuto};
static inline void rc_prio_policy(ModelArgs& a, PrioPolicy dflt, u32 grid, u32 resident,
                                  const RcKnobs& k) {
  a.prio_base = ~0u;
  a.prio_step = 1u << 31;
  a.prio_rot = 0;
  if (!k.prio) return;
  PrioPolicy p = dflt;
#ifdef RC_PRIO_LAST
  p = {(float)(RC_PRIO_LAST), false, 0u};
#endif
#ifdef RC_PRIO_RANK
  p = {0.0f, true, 0u};
#endif
#ifdef RC_PRIO_ROT
  p.rot = (u32)(RC_PRIO_ROT);
#endif
  if (p.rot == kRotAuto) p.rot = resident && grid > resident ? 12u : 10u;
  a.prio_rot = p.rot;
  if (!resident) return;
  if (p.rank) {
    a.prio_base = grid > 3 * resident ? grid - 3 * resident : 0u;
    a.prio_step = resident;
  } else if (p.last_rounds > 0.0f) {
    const u32 n = (u32)(p.last_rounds * (float)resident);
    a.prio_base = n < grid ? grid - n : 0u;
  }
}
static __device__ __forceinline__ void rc_prio_rotate(u32 k) {
  if (!k) return;
  const u32 t = (u32)(__builtin_amdgcn_s_memrealtime() >> k);
  const u32 p = (t + __builtin_amdgcn_s_getreg(0xF804)) & 3u;  // HW_ID bits 3:0: wave slot
  if (p == 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
static __device__ __forceinline__ void rc_set_prio(const ModelArgs& m) {
  const u32 b = __builtin_amdgcn_readfirstlane(blockIdx.x);
  if (b < m.prio_base) return;
  const u32 p = 1u + (b - m.prio_base) / m.prio_step;
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(1);
}
// workgroups of `kernel` the current device holds at once with `lds` bytes of dynamic LDS
// (occupancy x CUs), cached per (device, kernel, lds); 0 when the runtime cannot say (host)
u32 rc_resident_wgs(const void* kernel, int block, size_t lds);

// Small bucket models (k_decode_static LUT 4: 2048 < total <= 2^16; the pair decoder, LUT 3, is
// opt-in, RC_DEC_PAIR).  LDS
// holds the symbol table at address 0, one 16-B entry {cum, c, total/c as f32, s} per symbol at
// byte 16 s, then up to 2^SMB_LUT_BITS 8-B buckets {16 s0 | 16 s1 << 16, 0x4B400000 + cum[s1]}
// at SMB_LUT_OFF: the candidate's table address is one v_cndmask_b32 over its bucket entry's
// halves, and the candidate's whole entry one ds_read_b128.  2^12 buckets (32 KiB: buckets of
// 16 frequencies at total 2^16, where the Zipf(1.2) model has no bucket with three symbol
// starts) run in 512-lane workgroups, so that the LDS per wave stays that of 2^11 buckets in
// 256-lane ones (4 waves per SIMD); models with total <= 2^14 get fewer buckets and 256 lanes.
#ifndef SMB_LUT_BITS
#define SMB_LUT_BITS 12u
#endif
#define SMB_WG(lut_entries) ((lut_entries) > 2048u ? 512u : (u32)WG)
#define SMB_TAB_WORDS 1024u                      // the symbol table
#define SMB_LUT_OFF (SMB_TAB_WORDS * 4)          // bytes

// Pair-bucket decoding (LUT 3): models with 2^15 < total <= 2^16 (buckets of 16 frequencies) and
// every c < 2^16.  A bucket's entry holds both candidates of its bucket table entry, so the
// symbol step reads LDS once (the bucket decoder reads the bucket, then the candidate's table
// entry).  The u16 symbol pairs come first in LDS, the entries at PAIR_ENT_OFF.
#define PAIR_BUCKETS 4096u
#define PAIR_S_WORDS (PAIR_BUCKETS / 2)
#define PAIR_ENT_OFF (PAIR_S_WORDS * 4)            // bytes
#define PAIR_WORDS (PAIR_S_WORDS + 4 * PAIR_BUCKETS)


// RangeCoder::range_par_total (range_coder.rs:38-40): range / total, exact.
// SM (256 <= total <= 2^16), total not a power of two: two f64 steps with u = 1/total rounded
// up.  q1 = trunc(rh u) = floor(rh / total): the exact product is >= rh / total, and exceeds it
// by at most rh 2^-52 / total < 2^-28 while the distance to the next integer is >= 1 / total >=
// 2^-16, so neither the error nor the product's rounding (to nearest, or toward zero; q1 < 2^24
// is representable) reaches another integer.  Then n = (rh - q1 total) 2^32 + rl < total 2^32 <=
// 2^48 is exact in f64 (one fma), and q0 = trunc(n u) = floor(n / total) by the same argument
// (error < 2^-4 / total, rounding ulp 2^-20 below 2^32).  range / total = q1 2^32 + q0.  Ten
// instructions instead of the 64 x 64 high product, its fix-up and their register copies.
#ifndef RC_DIV_F64
#define RC_DIV_F64 1  // 0: the 64 x 64 high product for small models too (scratch A/B builds)
#endif
template <int DIV, int SM = 0>
static __device__ __forceinline__ u64 range_par_total(u64 range, const ModelArgs& m) {
  if (DIV == DIV_POW2) return range >> m.lg;
  if (SM && RC_DIV_F64) {
    const u32 rh = hi32(range), rl = (u32)range;
    const u32 q1 = (u32)((double)rh * m.inv_up);
    const u32 rem = rh - __umul24(q1, m.total);
    const u32 q0 = (u32)(__builtin_fma((double)rem, 4294967296.0, (double)rl) * m.inv_up);
    return ((u64)q1 << 32) | q0;
  }
  u64 q = __umul64hi(range, m.magic);  // q in {floor - 1, floor}
  u64 rem = range - q * (u64)m.total;
  return rem >= (u64)m.total ? q + 1 : q;
}

#ifndef MAD24_C
#define MAD24_C 1  // the 24-bit high-half mad from C (inline asm makes the hazard recognizer pad)
#endif
// r * v for the coder's products (range_coder.rs:65, :70).  SM (256 <= total <= 2^16): r < 2^56
// and v <= 2^16, so the high half is a 24-bit multiply.  SM is written out as two
// instructions, lo(r)*v as a 64-bit product plus a 24-bit mad into its high half: from the C
// form the compiler re-derives the low half with an extra v_mul_lo_u32 and zeroes the mad's
// addend with two moves (three extra VALU per product).
template <int SM>
static __device__ __forceinline__ u64 mul_rv(u64 r, u32 v) {
  if (SM) {
    u64 p, c;
    u32 h;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c) : "v"((u32)r), "v"(v));
    h = MAD24_C ? __umul24(hi32(r), v) + hi32(p) : 0u;
    if (!MAD24_C) asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(hi32(r)), "v"(v), "v"(hi32(p)));
    return ((u64)h << 32) | (u32)p;
  }
  return r * (u64)v;
}


// r * v + a (mod 2^64): the same two instructions with the 64-bit addend folded into the first
template <int SM>
static __device__ __forceinline__ u64 mad_rv(u64 r, u32 v, u64 a) {
  if (SM) {
    u64 p, c;
    u32 h;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(p), "=s"(c) : "v"((u32)r), "v"(v), "v"(a));
    h = MAD24_C ? __umul24(hi32(r), v) + hi32(p) : 0u;
    if (!MAD24_C) asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(hi32(r)), "v"(v), "v"(hi32(p)));
    return ((u64)h << 32) | (u32)p;
  }
  return r * (u64)v + a;
}

// v_ffbh_u32 as the hardware defines it: 0xFFFFFFFF for 0 (the clz builtins are undefined there)
static __device__ __forceinline__ u32 ffbh(u32 v) {
  u32 r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// launchers (one translation unit each, so the variants compile in parallel)
hipError_t rc_static_encode_launch(hipStream_t stream, const RcKnobs& k, const ModelArgs& a,
                                   int div, int smv, const uint8_t* syms, const u64* sym_off,
                                   u32 n_chunks, uint8_t* out, const u64* out_off, u64* out_len,
                                   u32* flags);
// dynamic LDS bytes of k_decode_static for a model (lut3: the pair-bucket variant, wgs lanes
// per workgroup)
size_t rc_static_decode_lds(const ModelArgs& a, int lut3, u32 wgs);
hipError_t rc_static_decode_launch_pow2(hipStream_t stream, const RcKnobs& k, const ModelArgs& a,
                                        int sm,
                                        const uint8_t* code, const u64* code_off,
                                        const u64* code_len, uint8_t* syms_out,
                                        const u64* sym_off, u32 n_chunks, u32* flags);
hipError_t rc_static_decode_launch_magic(hipStream_t stream, const RcKnobs& k, const ModelArgs& a,
                                         int sm,
                                         const uint8_t* code, const u64* code_off,
                                         const u64* code_len, uint8_t* syms_out,
                                         const u64* sym_off, u32 n_chunks, u32* flags);

