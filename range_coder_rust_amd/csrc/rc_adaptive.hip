// rc_adaptive.hip — MI355X (gfx950) kernels of the adaptive order-0 model (SURVEY.md §8a A17,
// config C4).
//
// The model is build-defined (the reference ships none).  Per chunk, c[i] = 1 for i < n; after
// the i-th coded symbol s, c[s] += inc, and at every period-th symbol all counts are halved,
// c = (c + 1) >> 1, if the total exceeds limit.  The coder sees (c[s], cum[s], total) before
// the update, through the reference's PModel interface (pmodel.rs:4-12).  It runs the
// reference's param_update (range_coder.rs:53-92) and Decoder::decode (decoder.rs:38-54)
// bit-exactly, as the static kernels do (the same closed-form renormalisation).
//
// Layout: one chunk per lane, one wave per workgroup.  Each lane's counts live in LDS as a
// 255-node tree of u16 (32 KiB per wave, so 5 waves per CU).  Node 256 — the total — lives in a
// register.  The tree is interleaved by lane, so one node row is one conflict-free 128-B access:
//     node j (1..255) = the counts of symbols [j - lowbit(j), j),  at byte (j-1)*128 + col,
// col = 4 (lane mod 32) + 2 (lane div 32) (bank-conflict free per 32-lane group).
// Read top-down, that is the left-subtree-sum tree over the 256 symbols.  For symbol s, level l
// (0..7) visits node (s & ~(2*step-1)) | step, step = 128 >> l, and turns right iff bit 7-l of s
// is set.  Read as a Fenwick tree, it turns into counts and back in place for the halving.
// Node values stay below 2^16 because the total does: limit + inc * period <= 65535.
//
// Encoder symbol step: the 8 path nodes are read one symbol ahead, packed in
// u16 pairs, so cum[s] = sum over right turns and cum[s+1] = the same sum with the bits of s+1
// (the walk of s+1 agrees with that of s above its lowest zero bit) are 4 v_dot2_u32_u16 each,
// c[s] = cum[s+1] - cum[s], and the update c[s] += inc is 4 v_pk_mad_u16 written back as u16s.
// Output bytes go through a 128-bit shift register; every 4 symbols its complete dwords are
// stored as one 12-B write that also rewrites the (identical) dwords before them.
//
// Decoder symbol step: the target frequency comes from a float hint x * total / range; the top
// three tree levels (7 nodes, fixed addresses) are read one symbol ahead, levels 3-5 are one
// 7-node lookahead read and levels 6-7 one 3-node read, so the walk costs two dependent LDS
// round trips.  The exact interval test r*cum <= x < r*(cum+c) then confirms the symbol
// (FreqTable::find_index, sample_impl.rs:27-45); a wrong hint takes a rare exact path.
//
// range / total (range_coder.rs:38-40) uses a float64 reciprocal of the total (computed one
// symbol ahead) and an exact integer correction.
#include "rc_common.h"

#include <stdlib.h>

#define AWG 64  // one wave per workgroup
#define TREE_BYTES (255 * 128)
#define TREE128_BYTES (127 * 128)  // the decoder's tree for models of <= 128 symbols
#define ROW(j) (((j) - 1) * 128)  // byte offset of node j's row

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

static __device__ __forceinline__ u32 clz32(u32 v) { return (u32)__builtin_clz(v); }  // v != 0

// ~1/t to well under 2^-40 relative error: v_rcp_f64 plus one Newton step
static __device__ __forceinline__ double cvt_f64(u32 v);
static __device__ __forceinline__ double recip(u32 t) {
  const double d = cvt_f64(t);
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}

// range_par_total (range_coder.rs:38-40): floor(v / t) for 1 <= t < 2^16, exact.  Each
// quotient half is floor or floor - 1 from the float64 product, then corrected.  The
// corrections use sign masks (d >> 31), not compares: a VALU read of VCC (v_cndmask_b32_e32,
// v_addc_co_u32) costs ~4x a plain op on gfx950 (tools/ubench_sel.hip).
static __device__ __forceinline__ u32 fixup(u32& q, u32 rem, u32 t) {  // rem < 2t
  const u32 d = rem - t;
  // q + 1 + (d >> 31 arithmetic): +1 unless rem < t, one v_add3_u32 (the compiler's form of
  // it is a not, a shift and an add)
  asm("v_add3_u32 %0, %0, 1, %1" : "+v"(q) : "v"((u32)((int)d >> 31)));
  return min(rem, d);  // rem mod t
}
static __device__ __forceinline__ u64 div_total(u64 v, u32 t, double rt) {
  const u32 hi = hi32(v), lo = (u32)v;
  u32 qh = (u32)(cvt_f64(hi) * rt);
  const u32 rh = fixup(qh, hi - qh * t, t);
  const double num = fma(cvt_f64(rh), 4294967296.0, cvt_f64(lo));  // < 2^48: exact
  u32 ql = (u32)(num * rt);
  fixup(ql, lo - ql * t, t);  // (rh:lo) - ql*t < 2t: its low 32 bits are the value
  return ((u64)qh << 32) | ql;
}

// range_par_total (range_coder.rs:38-40): floor(v / t) for 1 <= t < 2^16 from the model's
// table entry M = floor((2^64 - 1) / t): q = mulhi(v, M) is floor(v / t) or one less (v < 2^64,
// so v / 2^64 < 1 is all M's truncation can lose), and v - q t < 2t tells which, in 32 bits.
static __device__ __forceinline__ u64 div_magic(u64 v, u32 t, u64 M) {
  const u64 q = __umul64hi(v, M);
  const u32 d = (u32)v - (u32)q * t - t;  // remainder - t (the remainder is < 2t: 32 bits do)
  return q + (1u + smask(d));             // (an opaque sign mask: no v_cmp + v_cndmask on VCC)
}

// u32 -> f64 as the single instruction (the compiler widens (double)hi32(x) into a u64
// conversion: a second convert and an f64 add)
static __device__ __forceinline__ double cvt_f64(u32 v) {
  double d;
  asm("v_cvt_f64_u32 %0, %1" : "=v"(d) : "v"(v));
  return d;
}

// r * v for v < 2^16 (r < 2^64 / v: no overflow)
static __device__ __forceinline__ u64 mul_r(u64 r, u32 v) {
  return (u64)(u32)r * v + ((u64)(hi32(r) * v) << 32);
}

// ---- LDS access by byte address (this kernel's only LDS is the dynamic tree, at offset 0) ----
typedef __attribute__((address_space(3))) uint16_t l_u16;
static __device__ __forceinline__ u32 lrd(u32 a) { return *(const l_u16*)(uintptr_t)a; }
static __device__ __forceinline__ void lwr(u32 a, u32 v) { *(l_u16*)(uintptr_t)a = (uint16_t)v; }

// ---- the per-lane count tree: node j at t[(j - 1) * 64] ----

// NN: the symbols the tree spans (256; 128 for the decoder of models of <= 128 symbols, whose
// tree is nodes 1..127 only: node 128, the count of symbols 0..127, is the total itself)
template <u32 NN = 256>
static __device__ __forceinline__ void tree_init(uint16_t* t, u32 n) {
  for (u32 j = 1; j < NN; ++j) {
    const u32 lo = j - (j & (0u - j));
    t[(j - 1) * 64] = (uint16_t)(n > lo ? min(n, j) - lo : 0u);
  }
}

// every c = (c + 1) >> 1: Fenwick -> counts (reverse pass), halve, counts -> Fenwick
template <u32 NN = 256>
static __device__ __forceinline__ void tree_halve(uint16_t* t, u32& total) {
  for (u32 j = NN - 1; j >= 1; --j) {
    const u32 k = j + (j & (0u - j));
    if (k < NN) t[(k - 1) * 64] = (uint16_t)(t[(k - 1) * 64] - t[(j - 1) * 64]);
  }
  u32 sum = 0, nt = 0;
  for (u32 j = 1; j < NN; ++j) {
    const u32 v = t[(j - 1) * 64];
    sum += v;
    nt += (v + 1) >> 1;
    t[(j - 1) * 64] = (uint16_t)((v + 1) >> 1);
  }
  nt += (total - sum + 1) >> 1;  // c[NN - 1] lives only in the total
  for (u32 j = 1; j < NN; ++j) {
    const u32 k = j + (j & (0u - j));
    if (k < NN) t[(k - 1) * 64] = (uint16_t)(t[(k - 1) * 64] + t[(j - 1) * 64]);
  }
  total = nt;
}

// FreqTable::find_index for q < total (rare exact path): the s with cum[s] <= q < cum[s]+c[s]
static __device__ __forceinline__ u32 tree_find(const uint16_t* t, u32 q, u32 total, u32& cum, u32& c) {
  u32 pos = 0, rem = q, b = total;
  for (int l = 0; l < 8; ++l) {
    const u32 j = pos | (128u >> l);
    const u32 v = t[(j - 1) * 64];
    const bool right = rem >= v;
    pos = right ? j : pos;
    rem = right ? rem - v : rem;
    b = right ? b - v : v;
  }
  cum = q - rem;
  c = b;
  return pos;
}

// c[s] += inc (rare exact path): every node whose left subtree holds s
static __device__ __forceinline__ void tree_add(uint16_t* t, u32 s, u32 inc) {
  for (int l = 0; l < 8; ++l) {
    const u32 step = 128u >> l;
    if (!(s & step)) {
      uint16_t* p = t + ((((s & ~(2 * step - 1)) | step) - 1) * 64);
      *p = (uint16_t)(*p + inc);
    }
  }
}

static __device__ __forceinline__ u32 wave_min(u32 v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (u32)__shfl_xor((int)v, o));
  return v;
}
static __device__ __forceinline__ u32 wave_max(u32 v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (u32)__shfl_xor((int)v, o));
  return v;
}

// byte j (0..15, per lane) of a 16-B block in registers
static __device__ __forceinline__ u32 byte_at(const u32x4& b, u32 j) {
  u32 w = b.x;
  w = (j >> 2) == 1 ? b.y : w;
  w = (j >> 2) == 2 ? b.z : w;
  w = (j >> 2) == 3 ? b.w : w;
  return (w >> (8 * (j & 3))) & 255u;
}

__device__ u32x4 g_zero16;  // load target of lanes without input (never written)

// ------------------------------------------------------------------------------------------
// Encoder
// ------------------------------------------------------------------------------------------

// Output: a 128-bit shift register W0..W3 (W0 oldest) whose low B bits are the stream bytes
// not yet stored, MSB first, above them the last bytes already stored.  Stream byte k sits at
// slot byte a + k of the dword-aligned origin o (a = slot address & 3, counted as B = 8a
// phantom bytes at the start), so every complete dword is aligned in memory.
struct AEnc {
  u64 low, range;
  u32 W0, W1, W2, W3, B, wpos;  // wpos: origin-relative byte of the next complete dword
  u32 total, err;
  double rt;
};

struct AOut {  // per-lane output geometry
  uint8_t* o;  // slot address & ~3
  u32 a;       // slot address & 3
  u32 end;     // a + capacity (clamped to 32 bits): origin-relative end of the slot
};

// the same for nb = 8n <= 24 (the coder's settled bytes): every word is hi32({Wi:Wi+1} << nb),
// byte j from byte 4 + j - n of the pair, so four v_perm_b32 share one selector,
// hi32(0x0706050403020100 << nb).  (From C: four 64-bit shifts and the register-pair copies that
// assemble their operands.)
static __device__ __forceinline__ void out_push8(AEnc& e, u32 hl, u32 nb) {
  const u32 sel = hi32(0x0706050403020100ull << nb);
  const u32 w0 = __builtin_amdgcn_perm(e.W0, e.W1, sel);
  const u32 w1 = __builtin_amdgcn_perm(e.W1, e.W2, sel);
  const u32 w2 = __builtin_amdgcn_perm(e.W2, e.W3, sel);
  e.W3 = __builtin_amdgcn_perm(e.W3, hl, sel);
  e.W0 = w0;
  e.W1 = w1;
  e.W2 = w2;
  e.B += nb;
}

// shift the register left by nb bits (0..32) and append the top nb bits of hl
static __device__ __forceinline__ void out_push(AEnc& e, u32 hl, u32 nb) {
  e.W0 = hi32((((u64)e.W0 << 32) | e.W1) << nb);
  e.W1 = hi32((((u64)e.W1 << 32) | e.W2) << nb);
  e.W2 = hi32((((u64)e.W2 << 32) | e.W3) << nb);
  e.W3 = hi32((((u64)e.W3 << 32) | hl) << nb);
  e.B += nb;
}


typedef u32 u32x3 __attribute__((ext_vector_type(3)));
typedef __attribute__((address_space(1))) u32x3 g_u32x3;

// store the complete dwords (B <= 127, so at most 3): the 12 bytes ending at the last of them,
// the dwords before it being ones already stored (still in the register, unchanged).  Bytes
// outside [a, end) — the phantom start, or past a too-small slot — are never written.
static __device__ __forceinline__ void out_flush(AEnc& e, const AOut& g, bool wr) {
  const u32 cnt = e.B >> 5, sh = e.B & 31u;
  const u32 v1 = __builtin_bswap32(__builtin_amdgcn_alignbit(e.W0, e.W1, sh));
  const u32 v2 = __builtin_bswap32(__builtin_amdgcn_alignbit(e.W1, e.W2, sh));
  const u32 v3 = __builtin_bswap32(__builtin_amdgcn_alignbit(e.W2, e.W3, sh));
  const u32 st = e.wpos + 4 * cnt - 12;  // wraps below 0 near the start
  const bool fast = (int)st >= (int)g.a && st + 12 <= g.end;
  if (wr && fast) {
    u32x3 v = {v1, v2, v3};
    *(g_u32x3*)(g.o + st) = v;
  } else if (wr) {
    const u32 vv[3] = {v1, v2, v3};
#pragma unroll
    for (u32 b = 0; b < 12; ++b) {
      const u32 pos = st + b;
      if ((int)pos >= (int)g.a && pos < g.end) gstore8(g.o + pos, vv[b >> 2] >> (8 * (b & 3)));
    }
  }
  e.wpos += 4 * cnt;
  e.B = sh;
}

// param_update (range_coder.rs:53-92) for (c, cum) under total tot: narrowing, closed-form
// no_carry_expansion (<= 3 bytes: range >= 2^32 here), the settled bytes into the register.
// Returns whether range_reduction_expansion has work (rare).
static __device__ __forceinline__ bool enc_code(AEnc& e, u32 cum, u32 c, u32 tot, double rt) {
  const u64 r = div_total(e.range, tot, rt);
  e.range = mul_r(r, c);
  e.low += mul_r(r, cum);
  const u32 nb = clz32(hi32(e.low) ^ hi32(e.low + e.range)) & 24u;
  out_push8(e, hi32(e.low), nb);
  e.low <<= nb;
  e.range <<= nb;
  return hi32(e.range) < 0x10000u;
}

// range_reduction_expansion (range_coder.rs:126-135); leaves B <= 31
static __device__ __forceinline__ void enc_reduce(AEnc& e, const AOut& g, bool wr) {
  while (e.range < TOP16) {
    e.range = ~e.low & (TOP16 - 1);
    if (e.B > 112) out_flush(e, g, wr);
    out_push8(e, hi32(e.low), 8);
    e.low <<= 8;
    e.range <<= 8;
  }
  out_flush(e, g, wr);
}

// The tree state of one symbol, prepared and loaded one symbol ahead.  Level l's node on the
// path of s is at a[l] + ROW(128 >> l), its value v[l] (packed in u16 pairs only at use, so
// nothing waits for the loads before then); bs/bs1 pack the turn bits of s and s+1 for the
// level pairs (2k: hi half, 2k+1: lo half), nbm those of ~s.
struct ESym {
  u32 a[8];
  u32 bs[4], bs1[4], nbm[4];
  u32 s1hi;  // (s + 1) >> 8: cum[256] is the total
  u32 s;
  u32 v[8];
};
// keep the symbol bits above level l's turn (s bits 8-l.., at byte bit 7+) and the lane column
#define LMASK(l) ((0x7F80u & ~(((256u >> (l)) - 1u) << 7)) | 0x7Fu)

typedef __attribute__((address_space(3))) char l_char;
// LDS byte address a: the kernels' only LDS is the dynamic tree, which starts at 0 (tb, the
// tree's base, is kept for the halving's pointer accesses and must be 0)
#define LRD(tb, a) ((u32) * (const __attribute__((address_space(3))) uint16_t*)(uintptr_t)(a))
#define LWR(tb, a, v) (*(__attribute__((address_space(3))) uint16_t*)(uintptr_t)(a) = (uint16_t)(v))

// The turn-bit words of every symbol value (bs, bs1, nbm of ESym; 48 B per symbol, 12 KiB):
// three 16-B loads from this L1-resident table replace ~20 shifts and masks per symbol in the
// model wave, whose instruction count bounds the encoder.  They are loaded two symbols ahead
// (ETurn), so their latency stays off the symbol chain.
struct ETurnTable {
  u32 w[256][12];
};
static constexpr ETurnTable make_turn_table() {
  ETurnTable t{};
  for (u32 s = 0; s < 256; ++s) {
    const u32 u = s | (s << 15), s1 = s + 1, u1 = s1 | (s1 << 15);
    for (int k = 0; k < 4; ++k) {
      t.w[s][k] = (u >> (6 - 2 * k)) & 0x10001u;
      t.w[s][4 + k] = (u1 >> (6 - 2 * k)) & 0x10001u;
      t.w[s][8 + k] = t.w[s][k] ^ 0x10001u;
    }
  }
  return t;
}
__device__ const ETurnTable g_turn_table = make_turn_table();

struct ETurn {
  u32x4 b0, b1, b2;
};
static __device__ __forceinline__ ETurn eturn_load(u32 s) {
  const u32x4* t = (const u32x4*)g_turn_table.w[s];
  return ETurn{gload16(t), gload16(t + 1), gload16(t + 2)};
}

// symbol s, whose turn bits tb were loaded earlier
static __device__ __forceinline__ void esym_prep(ESym& q, u32 s, u32 col, const ETurn& t) {
  const u32 X = (s << 7) | col;
#pragma unroll
  for (int l = 0; l < 8; ++l) q.a[l] = X & LMASK(l);
  q.bs[0] = t.b0.x, q.bs[1] = t.b0.y, q.bs[2] = t.b0.z, q.bs[3] = t.b0.w;
  q.bs1[0] = t.b1.x, q.bs1[1] = t.b1.y, q.bs1[2] = t.b1.z, q.bs1[3] = t.b1.w;
  q.nbm[0] = t.b2.x, q.nbm[1] = t.b2.y, q.nbm[2] = t.b2.z, q.nbm[3] = t.b2.w;
  q.s1hi = (s + 1) >> 8;
  q.s = s;
}

static __device__ __forceinline__ void esym_load(ESym& q, l_char* tb) {
#pragma unroll
  for (int l = 0; l < 8; ++l) q.v[l] = LRD(tb, q.a[l] + ROW(128u >> l));
}

// cum[s] and c[s] = cum[s+1] - cum[s] from the path values; then c[s] += inc: inc on the nodes
// where the walk turned left, written back as u16s
static __device__ __forceinline__ void esym_code(const ESym& q, l_char* tb, u32 total, us2 incp,
                                                 u32& cum, u32& c) {
  us2 vp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    vp[k] = (us2){(unsigned short)q.v[2 * k + 1], (unsigned short)q.v[2 * k]};
  u32 a0 = __builtin_amdgcn_udot2(vp[0], __builtin_bit_cast(us2, q.bs[0]), 0u, false);
  u32 a1 = __builtin_amdgcn_udot2(vp[0], __builtin_bit_cast(us2, q.bs1[0]),
                                  __umul24(q.s1hi, total), false);
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    a0 = __builtin_amdgcn_udot2(vp[k], __builtin_bit_cast(us2, q.bs[k]), a0, false);
    a1 = __builtin_amdgcn_udot2(vp[k], __builtin_bit_cast(us2, q.bs1[k]), a1, false);
  }
  cum = a0;
  c = a1 - a0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const us2 nv = vp[k] + __builtin_bit_cast(us2, q.nbm[k]) * incp;
    LWR(tb, q.a[2 * k + 1] + ROW(128u >> (2 * k + 1)), nv.x);
    LWR(tb, q.a[2 * k] + ROW(128u >> (2 * k)), nv.y);
  }
}

// Encoder::finish (encoder.rs:40-46) when fin (8 x left_shift), then the last partial dword;
// returns the stream length
static __device__ __forceinline__ u32 enc_finish(AEnc& e, const AOut& g, bool wr, bool fin) {
  out_flush(e, g, wr);
  if (fin) {
    out_push(e, hi32(e.low), 32);
    out_push(e, (u32)e.low, 32);
    out_flush(e, g, wr);
  }
  const u32 rb = e.B >> 3;
  for (u32 m = 0; m < rb; ++m) {
    const u32 pos = e.wpos + m;
    if (wr && pos >= g.a && pos < g.end) gstore8(g.o + pos, e.W3 >> (e.B - 8 * (m + 1)));
  }
  return e.wpos + rb - g.a;
}

// ---- the two-wave encoder ----
// The adaptive model does not depend on the coder.  Wave 0 of a workgroup (the model wave)
// walks and updates the 64 trees and hands (cum, c, total) per symbol to wave 1 (the coder
// wave) through an LDS FIFO of two 8-symbol halves: while the model fills one half, the coder
// codes the other, and one barrier per 8 symbols swaps them.  Tree + FIFO = 40 KiB, so 4
// workgroups (8 waves) share a CU and each SIMD issues for 2 waves, at ~2.5 instead of ~5
// cycles per VALU instruction (tools/ubench_issue.hip).
#define EWG 128
#define FIFO_SYMS 8
#define FIFO_OFF TREE_BYTES                  // 32640: 8-B aligned, right after the tree
#define FIFO_BYTES (2 * FIFO_SYMS * 64 * 8)  // 8 KiB
// entry (half h, symbol j, lane L): (cum | c << 16, total | bad << 31); a wave's 64 entries are
// one contiguous 512-B run (conflict-free ds_write_b64 / ds_read_b64)
#define FIFO_AT(h, j, lane) (FIFO_OFF + ((((h) * FIFO_SYMS + (j)) * 64 + (lane)) << 3))

typedef u32 u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 l_u32x2;

static __device__ __forceinline__ u32x2 fifo_get(u32 a) { return *(const l_u32x2*)(uintptr_t)a; }

// the 16 stream symbols [16 g, 16 g + 16) of a lane (its stream starts at byte mis of block 0)
// as 4 words, from its 16-B blocks g and g + 1: a dword shift by mis >> 2 (two mask stages,
// m0 / m1 = its bits as 0 / ~0), then a byte funnel by mis & 3
static __device__ __forceinline__ void funnel4(u32 (&w)[4], const u32x4& b0, const u32x4& b1,
                                               u32 m0, u32 m1, u32 mis) {
  const u32 v[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  u32 v1[7], v2[5];
#pragma unroll
  for (int i = 0; i < 7; ++i) v1[i] = msel(m0, v[i + 1], v[i]);
#pragma unroll
  for (int i = 0; i < 5; ++i) v2[i] = msel(m1, v1[i + 2], v1[i]);
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_alignbyte(v2[k + 1], v2[k], mis);
}

// The model wave's step t: symbols i = 8 t + j of every lane into FIFO half H.  All lanes are at
// the same symbol index, so the period's halving check is a scalar test.  The next symbol's
// tree reads are issued while the current one finishes, after the halving check.
template <int H>
static __device__ __forceinline__ void model_step(ESym& q, ETurn& tn, u32& total,
                                                  const u32 (&w)[2], u32 wn, u32 t,
                                                  uint16_t* tcol, l_char* tb, u32 col, u32 lane,
                                                  us2 incp, const AdaptParams& p) {
#pragma unroll
  for (int j = 0; j < FIFO_SYMS; ++j) {
    u32 cum, c;
    const u32 s = q.s;
    esym_code(q, tb, total, incp, cum, c);
    const u32 tot = total;
    total += p.inc;
    if (((8u * t + j) & p.pmask) == p.pmask) {  // adapt_update's halving check
      const bool h = total > p.limit;
      if (__builtin_expect(__any((int)h), 0)) {
        if (h) tree_halve(tcol, total);
      }
    }
    const u32 sn = j < 7 ? (w[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 255u : wn & 255u;
    const u32 s2 = j + 2 < 8 ? (w[(j + 2) >> 2] >> (8 * ((j + 2) & 3))) & 255u
                             : (wn >> (8 * (j - 6))) & 255u;
    ESym qn;
    esym_prep(qn, sn, col, tn);  // tn: symbol sn's turn bits, loaded a symbol ago
    tn = eturn_load(s2);
    esym_load(qn, tb);
    // bit 31: a symbol outside the alphabet (the reference panics, sample_impl.rs:19), where
    // the coder stops; c >= 1 keeps entries codable for lanes past their chunk's end
    const u32 e1 = ((p.n - 1u - s) & 0x80000000u) | tot;
    *(l_u32x2*)(uintptr_t)FIFO_AT(H, j, lane) = (u32x2){cum | (max(c, 1u) << 16), e1};
    q = qn;
  }
}

static __device__ __forceinline__ void model_wave(const AdaptParams& p, const uint8_t* sp, u64 n,
                                                  bool live, u32 lane, u32 T,
                                                  uint16_t* s_tree) {
  l_char* tb = (l_char*)s_tree;
  const u32 col = ((lane & 31u) << 2) | ((lane >> 5) << 1);
  uint16_t* tcol = s_tree + (col >> 1);
  tree_init(tcol, p.n);
  const us2 incp = {(unsigned short)p.inc, (unsigned short)p.inc};
  u32 total = p.n;
  const u32 mis = (u32)(uintptr_t)sp & 15u;
  const bool has = live && n > 0;
  const u32x4* bp = (const u32x4*)(sp - mis);
  const u32 blast = has ? (u32)((mis + n - 1) >> 4) : 0u;  // last block holding a symbol
  auto blk = [&](u32 u) -> u32x4 { return gload16(has ? bp + min(u, blast) : &g_zero16); };
  const u32 m0 = 0u - ((mis >> 2) & 1u), m1 = 0u - ((mis >> 3) & 1u);
  // blocks g + 1 and g + 2 are in registers (or in flight) while group g is modelled; the block
  // loaded during group g is first needed a group later
  u32x4 Ba = blk(1), Bb = blk(2);
  u32 nw[4];
  funnel4(nw, blk(0), Ba, m0, m1, mis);  // group 0
  ESym q;
  esym_prep(q, nw[0] & 255u, col, eturn_load(nw[0] & 255u));
  esym_load(q, tb);
  ETurn tn = eturn_load((nw[0] >> 8) & 255u);
  // group t / 2 (two steps), a barrier after each step: T + 1 barriers in all, as in the coder
  // wave.  Bx = block t/2 + 1, By = block t/2 + 2; Bx is then reloaded with block t/2 + 3.
  auto group = [&](u32 t, u32x4& Bx, const u32x4& By) {
    u32 cw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cw[k] = nw[k];
    if (t < T) {
      funnel4(nw, Bx, By, m0, m1, mis);  // the next group (its first symbol is looked ahead)
      Bx = blk((t >> 1) + 3);
      const u32 wa[2] = {cw[0], cw[1]};
      model_step<0>(q, tn, total, wa, cw[2], t, tcol, tb, col, lane, incp, p);
    }
    __syncthreads();
    if (t + 1 <= T) {
      if (t + 1 < T) {
        const u32 wb[2] = {cw[2], cw[3]};
        model_step<1>(q, tn, total, wb, nw[0], t + 1, tcol, tb, col, lane, incp, p);
      }
      __syncthreads();
    }
  };
  // two groups per iteration, the two block registers swapping roles: a loop-carried rotation
  // (B1 = B2; B2 = load) made the compiler copy the new load at the loop latch and wait there
  // for it, a whole HBM latency per 16 symbols
  for (u32 t = 0; t <= T; t += 4) {
    group(t, Ba, Bb);
    if (t + 2 <= T) group(t + 2, Bb, Ba);
  }
}

// The coder wave's step: FIFO half H, symbols i0 .. i0 + 7 of every lane.  A lane whose chunk
// ends inside the step, or meets a symbol outside the alphabet, first finishes per lane and then
// runs along with its writes off.
template <int H>
static __device__ __forceinline__ void coder_step(AEnc& e, const AOut& g, bool& wr, bool& done,
                                                  u32 i0, u64 n, u64 cap, u32 lane, u32 k,
                                                  const AdaptParams& p, u64* out_len,
                                                  u32* flags) {
  bool slow = !done && (u64)i0 + FIFO_SYMS > n;
  if (p.n < 256) {  // an entry of this chunk flagged bad in this step
    bool bad = false;
#pragma unroll
    for (int j = 0; j < FIFO_SYMS; ++j)
      bad = bad || ((u64)i0 + j < n && (fifo_get(FIFO_AT(H, j, lane)).y >> 31));
    slow = slow || (!done && bad);
  }
  if (__builtin_expect(__any((int)slow), 0)) {
    if (slow) {
      for (u32 j = 0; j < FIFO_SYMS && (u64)i0 + j < n; ++j) {
        const u32x2 en = fifo_get(FIFO_AT(H, j, lane));
        if (en.y >> 31) {
          e.err = RC_F_BAD_SYMBOL;
          break;
        }
        if (e.B > 96) out_flush(e, g, wr);
        const u32 tot = en.y & 0xFFFFu;
        if (enc_code(e, en.x & 0xFFFFu, en.x >> 16, tot, recip(tot))) enc_reduce(e, g, wr);
      }
      const u32 len = enc_finish(e, g, wr, e.err == 0);
      out_len[k] = len;
      flags[k] = e.err ? e.err : ((u64)len > cap ? RC_F_CAPACITY : 0u);
      done = true;
      wr = false;
    }
  }
#pragma unroll
  for (int j = 0; j < FIFO_SYMS; ++j) {
    const u32x2 en = fifo_get(FIFO_AT(H, j, lane));
    const u32 tot = en.y & 0xFFFFu;
    const bool rare = enc_code(e, en.x & 0xFFFFu, en.x >> 16, tot, recip(tot));
    if (__builtin_expect(__any((int)rare), 0)) {
      if (rare) enc_reduce(e, g, wr);
    }
    if ((j & 3) == 3) out_flush(e, g, wr);
  }
}

static __device__ __forceinline__ void coder_wave(const AdaptParams& p, u64 n, u64 cap,
                                                  uint8_t* lo, bool live, u32 lane, u32 k,
                                                  u32 T, u64* out_len, u32* flags) {
  AEnc e;
  e.low = 0;
  e.range = ~0ull;  // RangeCoder::default (range_coder.rs:13-20)
  e.W0 = e.W1 = e.W2 = e.W3 = 0;
  e.wpos = 0;
  e.err = 0;
  AOut g;
  g.o = (uint8_t*)((uintptr_t)lo & ~(uintptr_t)3);
  g.a = (u32)((uintptr_t)lo & 3);
  g.end = g.a + (u32)min(cap, (u64)(0xFFFFFF00u - g.a));
  e.B = 8 * g.a;
  bool wr = live, done = !live;
  for (u32 t = 0; t <= T; t += 2) {  // the model wave's barrier sequence, one step behind
    if (t >= 1) coder_step<1>(e, g, wr, done, 8 * (t - 1), n, cap, lane, k, p, out_len, flags);
    __syncthreads();
    if (t + 1 <= T) {
      coder_step<0>(e, g, wr, done, 8 * t, n, cap, lane, k, p, out_len, flags);
      __syncthreads();
    }
  }
  if (!done) {  // chunks ending on a step boundary: Encoder::finish
    const u32 len = enc_finish(e, g, wr, true);
    out_len[k] = len;
    flags[k] = (u64)len > cap ? RC_F_CAPACITY : 0u;
  }
}

__global__ __launch_bounds__(EWG) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_encode_adaptive(
    AdaptParams p, const uint8_t* __restrict__ syms, const u64* __restrict__ sym_off,
    u32 n_chunks, uint8_t* __restrict__ out, const u64* __restrict__ out_off,
    u64* __restrict__ out_len, u32* __restrict__ flags) {
  extern __shared__ uint16_t s_tree[];
  const u32 lane = threadIdx.x & 63u;
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 k = blockIdx.x * 64 + lane;
  bool live = k < n_chunks;
  RC_VGPR_FLOOR_128();
  u64 n = 0, cap = 0;
  const uint8_t* sp = syms;
  uint8_t* lo = out;
  if (live) {
    const u64 a = sym_off[k], b = out_off[k];
    n = sym_off[k + 1] - a;
    sp = syms + a;
    lo = out + b;
    cap = out_off[k + 1] - b;
  }
  if (n > RC_MAX_CHUNK_SYMBOLS) {  // 32-bit stream positions (include/range_coder.h)
    if (wave == 1) {
      out_len[k] = 0;
      flags[k] = RC_F_TOO_LONG;
    }
    live = false;
    n = 0;
  }
  // 8-symbol steps: the same count in both waves (they hold the same 64 chunks)
  const u32 T = __builtin_amdgcn_readfirstlane(wave_max(live ? (u32)((n + 7) >> 3) : 0u));
  if (wave == 0)
    model_wave(p, sp, n, live, lane, T, s_tree);
  else
    coder_wave(p, n, cap, lo, live, lane, k, T, out_len, flags);
}

// ------------------------------------------------------------------------------------------
// Decoder
// ------------------------------------------------------------------------------------------
//
// The decoder is bound by how fast ONE wave issues: the 32 KiB tree per wave leaves room for 5
// waves per CU, so most SIMDs run a single wave, which issues an instruction every ~4-5 cycles
// whatever the instruction (profiles/r02/pmc_adaptive_*.txt: 73% of wave time issuing, 23%
// waiting).  The symbol step is therefore written for instruction count:
//  * the code window is three dwords in registers, (cpos & ~3) + 0, 4, 8, shifted by one dword
//    when a symbol crosses a dword boundary; the next dword is loaded then, by the crossing
//    lanes only, and is needed no earlier than the next crossing (one symbol later at least);
//  * the walk tracks ~rem and (upper bound - q - 1), so each level is one add, one sign mask,
//    one max, one min and the path bit; the count comes out as e1 - ~rem;
//  * r * cum and r * c for 256-symbol models are a 64-bit mad plus a 24-bit mad each.

// u32 -> f32 and f32 -> u32 (saturating) as single instructions
static __device__ __forceinline__ float cvt_f32(u32 v) {
  float f;
  asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"(v));
  return f;
}
static __device__ __forceinline__ u32 cvt_u32_sat(float f) {
  u32 v;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(v) : "v"(f));
  return v;
}

// r * v (range_coder.rs:65, :70).  SM (256-symbol models, so total >= 256): r < 2^56 and
// v < 2^16, so the high half is a 24-bit mad into the high half of lo(r) * v.
template <int SM>
static __device__ __forceinline__ u64 mul_rs(u64 r, u32 v) {
  if (SM) {
    u64 p, c;
    u32 h;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c) : "v"((u32)r), "v"(v));
    h = __umul24(hi32(r), v) + hi32(p);  // (C, not asm: see MAD24_C in rc_static.h)
    return ((u64)h << 32) | (u32)p;
  }
  return mul_r(r, v);
}

// the code of one chunk: its dword-aligned origin and the offset of the last dword holding a
// code byte (every load is clamped to it, so none leaves the chunk's last dword)
struct ACode {
  const uint8_t* o;
  u32 dwl;
};
static __device__ __forceinline__ u32 ldw(const ACode& g, u32 off) {
  return gload((const u32*)(g.o + off));
}

struct ADec {
  u64 low, range;
  u32 xlo, xhi;  // x = Decoder::data - lower_bound (mod 2^64): all find_index needs
  u32 total;
  float tf;      // (float)total
  u64 M, Mn;     // magic[total] for this symbol, magic[total + inc] (loaded one symbol ahead)
  u32 cpos;      // origin-relative position of the next code byte (a + 8 primed + shifted in)
  u32 D0, D1, D2;  // the code dwords at (cpos & ~3) + 0, 4, 8 (offsets clamped to dwl)
  u32 d2o;         // offset of D2
  u32 L0, L1a, L1b, L2a, L2b, L2c, L2d;  // tree levels 0-2 (fixed nodes) of this symbol
};

template <u32 NN>
static __device__ __forceinline__ void dec_preread(ADec& d, u32 col) {
  if (NN == 256) {
    d.L0 = lrd(col + ROW(128));
    d.L1b = lrd(col + ROW(192));
    d.L2c = lrd(col + ROW(160));
    d.L2d = lrd(col + ROW(224));
  }
  d.L1a = lrd(col + ROW(64));
  d.L2a = lrd(col + ROW(32));
  d.L2b = lrd(col + ROW(96));
}

// nb <= 3 code bytes consumed (Decoder::shift_left_buffer, decoder.rs:31-35): a whole dword is
// consumed when bit 2 of the position flips.  Every lane then (re)loads the dword after its
// window (the same one when it did not cross): a load into the loop-carried register only for
// the crossing lanes makes the compiler copy that register, and wait for the load to do it.
static __device__ __forceinline__ void win_step(ADec& d, const ACode& g, u32 nb) {
  const u32 c2 = d.cpos + nb;
  u32 mc, d2n;  // mc = ~0: crossed into the next dword (bit 2 of the position flipped)
  asm("v_bfe_i32 %0, %1, 2, 1" : "=v"(mc) : "v"(d.cpos ^ c2));
  d.D0 = mselc(mc, d.D1, d.D0);
  d.D1 = mselc(mc, d.D2, d.D1);
  asm("v_mad_i32_i24 %0, %1, -4, %2" : "=v"(d2n) : "v"(mc), "v"(d.d2o));  // d2o + 4 if crossed
  d.d2o = min(d2n, g.dwl);
  d.D2 = ldw(g, d.d2o);
  d.cpos = c2;
}

// The walk for target q < total: symbol s, cum[s], c[s], and per level the visited node's
// row base P[l] (its node at P[l] + ROW(128 >> l)) and updated value nv[l] (+inc on a left
// turn).  It tracks nrem = ~rem and e1 = (upper end of the current subtree) - q - 1: with
// nd = v + nrem = ~(rem - v), a right turn (rem >= v) is nd < 0, rem' = min(rem, rem - v) is
// nrem' = max(nrem, nd), and a left turn makes the upper end cum + v, so e1' = min(e1, nd)
// (a right turn leaves it: nd is then >= 2^32 - 2^16 > e1).  At the end c = e1 + 1 + rem =
// e1 - nrem.
struct DWalk {
  u32 s, cum, c;
  u32 nv[8], P[8];
};

// (NN = 128: level 0, node 128, holds the total, so every target q < total turns left there:
// the walk starts at level 1 and never addresses nodes 129..255)
template <u32 NN>
static __device__ __forceinline__ void dec_walk(DWalk& w, const ADec& d, u32 q, u32 col,
                                                u32 inc) {
  u32 nrem = ~q, e1 = d.total + nrem, P = col;
  u32 mr[8];  // ~0: the walk turned right at that level
#define RC_LEVEL(l, V)                                  \
  {                                                     \
    const u32 v_ = (V), nd_ = v_ + nrem;                \
    mr[l] = smask(nd_);                                 \
    w.nv[l] = v_ + mselc(mr[l], 0u, inc);                \
    w.P[l] = P;                                         \
    nrem = max(nrem, nd_);                              \
    e1 = min(e1, nd_);                                  \
    P |= mr[l] & ((128u >> (l)) * 128u);                \
  }
  if (NN == 256) {
    RC_LEVEL(0, d.L0)
    RC_LEVEL(1, mselc(mr[0], d.L1b, d.L1a))
    const u32 t0 = mselc(mr[0], d.L2c, d.L2a), t1 = mselc(mr[0], d.L2d, d.L2b);
    RC_LEVEL(2, mselc(mr[1], t1, t0))
  } else {
    mr[0] = 0u;
    RC_LEVEL(1, d.L1a)
    RC_LEVEL(2, mselc(mr[1], d.L2b, d.L2a))
  }
  {  // levels 3-5: one 7-node read below P
    const u32 r3 = lrd(P + ROW(16)), r4a = lrd(P + ROW(8)), r4b = lrd(P + ROW(24));
    const u32 r5a = lrd(P + ROW(4)), r5b = lrd(P + ROW(12));
    const u32 r5c = lrd(P + ROW(20)), r5d = lrd(P + ROW(28));
    RC_LEVEL(3, r3)
    RC_LEVEL(4, mselc(mr[3], r4b, r4a))
    const u32 u0 = mselc(mr[3], r5c, r5a), u1 = mselc(mr[3], r5d, r5b);
    RC_LEVEL(5, mselc(mr[4], u1, u0))
  }
  {  // levels 6-7: one 3-node read
    const u32 r6 = lrd(P + ROW(2)), r7a = lrd(P + ROW(1)), r7b = lrd(P + ROW(3));
    RC_LEVEL(6, r6)
    RC_LEVEL(7, mselc(mr[6], r7b, r7a))
  }
#undef RC_LEVEL
  w.s = (P - col) >> 7;
  w.cum = q + nrem + 1u;  // q - rem
  w.c = e1 - nrem;
}

// c[s] += inc on the walked path (NN = 128: from level 1; node 128 is the total)
template <u32 NN>
static __device__ __forceinline__ void dec_update(const DWalk& w) {
#pragma unroll
  for (int l = NN == 256 ? 0 : 1; l < 8; ++l) lwr(w.P[l] + ROW(128u >> l), w.nv[l]);
}

// Decoder::decode (decoder.rs:38-54) with FreqTable::find_index (sample_impl.rs:27-45) and the
// model update; returns the symbol.  Wave-uniform call sites only (rare branches inside).
// at: symbol i is a period end ((i + 1) % period == 0); UNI: at is wave-uniform.
template <bool UNI, int SM, u32 NN>
static __device__ __forceinline__ u32 dec_step(ADec& d, const ACode& g, u32 col, uint16_t* tcol,
                                               const AdaptParams& p, bool at) {
  // levels 0-2 of the tree (fixed nodes) first: their LDS latency hides behind the hint and
  // range / total.  (Read at the end of the previous symbol and carried instead, they are
  // re-zero-extended by the compiler at the loop latch, which also waits for them there.)
  dec_preread<NN>(d, col);
  // (kept here by a scheduling barrier: left to itself the scheduler issues these reads just
  // before the walk needs them, after the hint and the division, and waits for them there)
  __builtin_amdgcn_sched_barrier(0);
  // hint q ~ x * total / range from the high halves (range >= 2^48: relative error <= 2^-15),
  // clamped to total - 1: the walk's upper-end tracking relies on q < total
  const float X = cvt_f32(d.xhi), R = cvt_f32(hi32(d.range));
  const u32 q = min(cvt_u32_sat(X * (d.tf * __builtin_amdgcn_rcpf(R))), d.total - 1u);
  const u64 r = div_magic(d.range, d.total, d.M);
  DWalk wk;
  dec_walk<NN>(wk, d, q, col, p.inc);
  u64 A = mul_rs<SM>(r, wk.cum), B = mul_rs<SM>(r, wk.c);
  u64 dx = sub64(d.xlo, d.xhi, A);
  // exact check r*cum <= x < r*(cum+c) as one unsigned test (A + B <= range: a wrapped x - A
  // is >= B)
  if (__builtin_expect(__any((int)(dx >= B)), 0)) {
    if (dx >= B) {  // exact rfreq = min(x / r, total - 1), then the walk again
      const u64 x = ((u64)d.xhi << 32) | d.xlo;
      u32 qe = d.total - 1;
      if (x < mul_r(r, d.total)) {
        qe = min(q, d.total - 1);
        u64 a = mul_r(r, qe);
        while (a > x) {
          --qe;
          a -= r;
        }
        while (x - a >= r) {
          ++qe;
          a += r;
        }
      }
      dec_walk<NN>(wk, d, qe, col, p.inc);
      A = mul_r(r, wk.cum);
      B = mul_r(r, wk.c);
      dx = sub64(d.xlo, d.xhi, A);
    }
  }
  dec_update<NN>(wk);
  d.total += p.inc;
  d.M = d.Mn;  // magic[total], loaded during this symbol unless a halving changes the total
  if (!UNI || at) {  // the halving check, before the next symbol's tree reads
    const bool h = at && d.total > p.limit;
    if (__builtin_expect(__any((int)h), 0)) {
      if (h) {
        tree_halve<NN>(tcol, d.total);
        d.M = gload64(p.magic + d.total);
      }
    }
  }
  d.Mn = gload64(p.magic + (d.total + p.inc));  // for the next symbol (total < 2^16 - inc)
  d.tf = (float)d.total;
  // param_update (range_coder.rs:53-92), closed form (<= 3 bytes: range >= 2^32 here)
  d.low += A;
  const u32 k8 = clz32(hi32(d.low) ^ hi32(d.low + B)) & 24u;
  d.low <<= k8;
  d.range = B << k8;
  // data' = data << k8 | bytes and low' = (low + A) << k8, so x' = (x - A) << k8 | the k8 / 8
  // code bytes at cpos: xl is ONE v_perm_b32 over {dx_lo, W} with selector
  // hi32(0x0706050400010203 << k8) (W = the 4 code bytes at cpos, first byte in byte 0)
  const u32 W = __builtin_amdgcn_alignbyte(d.D1, d.D0, d.cpos);
  d.xlo = __builtin_amdgcn_perm((u32)dx, W, hi32(0x0706050400010203ull << k8));
  d.xhi = hi32(dx << k8);
  u32 nb;  // k8 >> 3 as a plain shift (the compiler's v_bfe from the clz result costs more)
  asm("v_lshrrev_b32 %0, 3, %1" : "=v"(nb) : "v"(k8));
  win_step(d, g, nb);
  if (__builtin_expect(__any((int)(hi32(d.range) < 0x10000u)), 0)) {
    while (d.range < TOP16) {  // range_reduction_expansion (range_coder.rs:126-135)
      d.range = ~d.low & (TOP16 - 1);
      d.low <<= 8;
      d.range <<= 8;
      const u32 byte = (d.D0 >> (8 * (d.cpos & 3u))) & 255u;  // D0 holds the byte at cpos
      d.xhi = __builtin_amdgcn_alignbyte(d.xhi, d.xlo, 3);
      d.xlo = (d.xlo << 8) | byte;
      win_step(d, g, 1);
    }
  }
  return wk.s;
}

struct DecLane {
  ADec d;
  ACode g;
  bool done;
  u32 hd, nt, tl, col, k, a;
  u64 clen;
  uint8_t* op;
  uint16_t* tcol;
};

// lanes with all their tiles decoded: the tail symbols (per lane) and the flag
template <int SM, u32 NN>
static __device__ __forceinline__ void dec_lane_end(DecLane& L, const AdaptParams& p, u32 t,
                                                    u32* flags) {
  for (u32 j = 0; j < L.tl; ++j) {
    const u32 i = L.hd + 16 * t + j;
    gstore8(L.op + i,
            dec_step<false, SM, NN>(L.d, L.g, L.col, L.tcol, p, (i & p.pmask) == p.pmask));
  }
  // shift_left_buffer panics once more bytes are needed than the stream holds (decoder.rs:33)
  flags[L.k] = (u64)(L.d.cpos - L.a) > L.clen ? RC_F_TRUNCATED : 0u;
  L.done = true;
}

template <bool UNI, int SM, u32 NN>
static __device__ __forceinline__ void dec_tiles(DecLane& L, const AdaptParams& p, u32 T,
                                                 u32 hd_u, u32* flags) {
  for (u32 t = 0; t < T; ++t) {
    if (__any((int)(!L.done && t == L.nt))) {
      if (!L.done && t == L.nt) dec_lane_end<SM, NN>(L, p, t, flags);
    }
    const u32 i0 = hd_u + 16 * t;
    const u32 dd = (p.pmask - (L.hd + 16 * t)) & p.pmask;
    u32 o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      bool at;
      if (UNI)
        at = ((i0 + j) & p.pmask) == p.pmask;
      else  // lanes past their chunk's end halve too: it keeps every total below 2^16, which
            // the magic-table loads rely on
        at = ((u32)j & p.pmask) == dd;
      o[j >> 2] |= dec_step<UNI, SM, NN>(L.d, L.g, L.col, L.tcol, p, at) << (8 * (j & 3));
    }
    if (!L.done) gstore128(L.op + L.hd + 16 * t, (u32x4){o[0], o[1], o[2], o[3]});
  }
  if (!L.done) dec_lane_end<SM, NN>(L, p, T, flags);
}

template <int SM, u32 NN>
__global__ __launch_bounds__(AWG) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_decode_adaptive(
    AdaptParams p, const uint8_t* __restrict__ code, const u64* __restrict__ code_off,
    const u64* __restrict__ code_len, uint8_t* __restrict__ syms_out,
    const u64* __restrict__ sym_off, u32 n_chunks, u32* __restrict__ flags) {
  extern __shared__ uint16_t s_tree[];
  const u32 lane = threadIdx.x;
  DecLane L;
  L.k = blockIdx.x * AWG + lane;
  const bool live = L.k < n_chunks;
  RC_VGPR_FLOOR_128();
  u64 n = 0;
  L.clen = 0;
  const uint8_t* cp = code;
  L.op = syms_out;
  if (live) {
    cp = code + code_off[L.k];
    L.clen = code_len[L.k];
    const u64 a = sym_off[L.k];
    n = sym_off[L.k + 1] - a;
    L.op = syms_out + a;
  }
  const bool too_long = live && n > RC_MAX_CHUNK_SYMBOLS;  // 32-bit stream positions
  const bool trunc0 = live && !too_long && L.clen < 8;  // Decoder::new panics (decoder.rs:21)
  if (too_long) flags[L.k] = RC_F_TOO_LONG;
  if (trunc0) flags[L.k] = RC_F_TRUNCATED;
  L.done = !live || trunc0 || too_long;
  if (L.done) n = 0;
  // lane L's u16 at byte 4 (L mod 32) + 2 (L div 32) of each row: a ds_read_u16 / ds_write_b16
  // serves lanes 0-31 and 32-63 as separate groups, and within a group every lane has its own
  // bank (lane pairs sharing a dword conflicted 2-way whenever they read different rows)
  L.col = ((lane & 31u) << 2) | ((lane >> 5) << 1);
  L.tcol = s_tree + (L.col >> 1);
  tree_init<NN>(L.tcol, p.n);
  ADec& d = L.d;
  d.total = p.n;
  d.tf = (float)p.n;
  d.M = gload64(p.magic + p.n);
  d.Mn = gload64(p.magic + (p.n + p.inc));
  d.low = 0;
  d.range = ~0ull;

  // code: origin = the dword holding the first byte; lanes without a stream read g_zero16
  const bool has = !L.done;
  L.a = has ? (u32)((uintptr_t)cp & 3u) : 0u;
  L.g.o = has ? cp - L.a : (const uint8_t*)&g_zero16;
  // n <= 2^25 symbols consume at most 8 + 12 n < 2^29 bytes: code past 2^32 - 256 is never read
  const u64 cl = min(L.clen, (u64)0xFFFFFF00u);
  L.g.dwl = has ? (u32)((L.a + cl - 1) & ~3ull) : 12u;
  {
    // Decoder::new primes 8 bytes (decoder.rs:14-23), big-endian: dwords 0-2 from the origin
    const u32 w0 = ldw(L.g, 0), w1 = ldw(L.g, min(4u, L.g.dwl)), w2 = ldw(L.g, min(8u, L.g.dwl));
    d.xhi = __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, L.a));  // data - low, low = 0
    d.xlo = __builtin_bswap32(__builtin_amdgcn_alignbyte(w2, w1, L.a));
    d.cpos = L.a + 8;  // (cpos & ~3) = 8
    d.D0 = w2;
    d.D1 = ldw(L.g, min(12u, L.g.dwl));
    d.d2o = min(16u, L.g.dwl);
    d.D2 = ldw(L.g, d.d2o);
  }

  // output: symbols [0, hd) until it is 16-B aligned (per lane, byte stores), nt 16-symbol
  // tiles, then tl symbols
  const u32 mis = (u32)(uintptr_t)L.op & 15u;
  L.hd = live ? (u32)min((u64)((16u - mis) & 15u), n) : 0u;
  L.nt = live ? (u32)((n - L.hd) >> 4) : 0u;
  L.tl = live ? (u32)((n - L.hd) & 15u) : 0u;
  for (u32 j = 0; __any((int)(j < L.hd && !L.done)); ++j) {
    if (j < L.hd && !L.done) {
      gstore8(L.op + j,
              dec_step<false, SM, NN>(d, L.g, L.col, L.tcol, p, (j & p.pmask) == p.pmask));
    }
  }
  const u32 T = wave_max(L.done ? 0u : L.nt);
  const u32 hmin = wave_min(L.done ? 16u : L.hd), hmax = wave_max(L.done ? 0u : L.hd);
  if (hmin >= hmax)
    dec_tiles<true, SM, NN>(L, p, T, hmax, flags);
  else
    dec_tiles<false, SM, NN>(L, p, T, 0, flags);
}

hipError_t rc_adaptive_encode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* syms, const u64* sym_off, u32 n_chunks,
                                     uint8_t* out, const u64* out_off, u64* out_len,
                                     u32* flags) {
  hipLaunchKernelGGL(k_encode_adaptive, dim3((n_chunks + 63) / 64), dim3(EWG),
                     TREE_BYTES + FIFO_BYTES, stream, p, syms, sym_off, n_chunks, out, out_off,
                     out_len, flags);
  return hipGetLastError();
}

hipError_t rc_adaptive_decode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* code, const u64* code_off,
                                     const u64* code_len, uint8_t* syms_out, const u64* sym_off,
                                     u32 n_chunks, u32* flags) {
  // 256-symbol models keep total >= 256 (every count >= 1), so r < 2^56: 24-bit high products.
  // Models of <= 128 symbols decode with the 127-node tree (16 KiB per wave instead of 32: 8
  // waves per CU, held by their 176 VGPRs, instead of the 5 the LDS allows with 255 nodes).
  const dim3 grid((n_chunks + AWG - 1) / AWG), block(AWG);
  if (p.n == 256)
    hipLaunchKernelGGL((k_decode_adaptive<1, 256>), grid, block, TREE_BYTES, stream, p, code,
                       code_off, code_len, syms_out, sym_off, n_chunks, flags);
  else if (p.n <= 128)
    hipLaunchKernelGGL((k_decode_adaptive<0, 128>), grid, block, TREE128_BYTES, stream, p, code,
                       code_off, code_len, syms_out, sym_off, n_chunks, flags);
  else
    hipLaunchKernelGGL((k_decode_adaptive<0, 256>), grid, block, TREE_BYTES, stream, p, code,
                       code_off, code_len, syms_out, sym_off, n_chunks, flags);
  return hipGetLastError();
}
