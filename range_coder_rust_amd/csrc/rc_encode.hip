// rc_encode.hip — k_encode_static, the static-model encoder (see rc_static.h for the design
// notes shared with the decoder).
#include "rc_static.h"

#include <map>
#include <mutex>
#include <tuple>

// ------------------------------------------------------------------------------------------
// Encoder
//
// Per lane: one chunk.  Input: 64-symbol tiles (4 x 16 B per lane, issued one tile ahead).
// Output: settled bytes are packed into dwords and pushed into a per-lane 128-B LDS ring every
// symbol (unconditionally: when fewer than 4 bytes are ready the push writes the next, still
// free, slot and does not advance).  HBM writes are cooperative: when any lane's ring holds
// FLUSH_AT bytes, the wave runs a flush round in which every lane holding a complete 64-B unit
// hands it over; each store instruction then writes 16 chunks x 64 B (whole 64-B units), which
// the per-lane pattern (one 16-B granule of 64 different lines per instruction) cannot.
// ------------------------------------------------------------------------------------------
#define ENC_UNIT 64    // bytes per flush unit
#define FLUSH_AT 88    // ring fill (whole dwords past fpos) forcing a flush round
// Ring budget.  A push writes the slot of the incomplete dword, so the settled bytes past fpos
// must stay <= 4 * ENC_RING - 1.  After a flush round they are <= FLUSH_AT - 1 (whole dwords <
// FLUSH_AT, plus <= 3 bytes in the incomplete one).  Flush checks come every 8 symbols and after
// every rare path.  Until the next check, small models on the paired path (ENC_PAIR) settle at
// most 3 pairs of 3-byte symbols, then one pair whose two symbols both take the rare path (3
// no-carry bytes + up to 7 range_reduction_expansion bytes each); unpaired (and wide) models
// at most 7 symbols of <= 3 bytes and one rare symbol (<= 8 no-carry + 7 reduction bytes).
static_assert(FLUSH_AT % 4 == 0, "FLUSH_AT counts whole dwords");
static_assert(ENC_UNIT == 64 && ENC_RING % 4 == 0, "a flush granule's 4 ring dwords must not wrap");
static_assert(FLUSH_AT - 1 + 6 * 3 + 2 * (3 + 7) <= 4 * ENC_RING - 1,
              "paired small-model encoder may overrun its output ring");
static_assert(FLUSH_AT - 1 + 7 * 3 + (8 + 7) <= 4 * ENC_RING - 1,
              "unpaired encoder may overrun its output ring");
// Ring layout.  ENC_ROWS 1: a wave's 8 KiB ring holds 8 lane groups of 1 KiB (lanes 8g .. 8g+7);
// in a group, slot j is the 32-B row j and lane L's dword sits at byte 4 (L & 7) of it.  A lane's
// column base K then has no bits inside the row field (byte bits 5-9), so the slot of the dword
// at stream bit B is at K | (B & 0x3E0): one v_and_or_b32 (the column-major layout below needs an
// and plus a v_lshl_add_u32).  Four slots of a flush granule are four consecutive rows: two
// ds_read2_b32 from one address.  Per-symbol pushes of the lanes of a 32-lane store group meet
// in 4 banks per (L & 7) class, a conflict only when three or four of those lanes sit at the same
// slot mod 4.
// ENC_ROWS 0 (round 4): column-major, slot j of lane L at dword 64 j + L (stride 256 B).
#ifndef ENC_ROWS
#define ENC_ROWS 1
#endif
#define ENC_SLOT_BYTES (ENC_ROWS ? 32u : 256u)  // byte distance between a lane's slots j, j + 1
// LDS dword index of lane L's column inside its wave's ring
static __device__ __forceinline__ u32 ring_col(u32 L) {
  return ENC_ROWS ? (L >> 3) * 256u + (L & 7u) : L;
}
#ifndef ENC_TILE_Q
#define ENC_TILE_Q 4  // 16-B blocks per symbol load (4: 64-B bursts, one 64-symbol tile)
#endif
#ifndef ENC_WAVES
#define ENC_WAVES 4   // waves per SIMD the register allocation must allow
#endif
static_assert(ENC_TILE_Q == 4 || ENC_TILE_Q == 2, "tiles of 64 or 32 symbols");
#define SINK_SLOTS 65536
__device__ uint4 g_sink[SINK_SLOTS];  // dummy symbol tiles of dead lanes (contents irrelevant)
RC_STAMP_DEFINE(enc)  // (scratch -DRC_STAMP builds only)

struct Enc {
  u64 low, range;  // RangeCoder state (range_coder.rs:7-12)
  u64 acc;         // settled bytes, newest in the low bits; the B & 31 lowest are not pushed
  u32 B;           // bit position of the next settled byte, from the 64-B aligned slot base:
                   // dword B >> 5 of the stream is the incomplete one (its ring slot is free)
  u32 fthr;        // 8 (fpos + FLUSH_AT), fpos the byte position of the next unit to store:
                   // the flush test is one compare against B (enc_ready)
#ifdef RC_FILL
  rc_fill_t fill;  // scratch builds: the filler instructions' register
#endif
  u32 err;         // first RC_F_* error of this chunk (SM: OR of staged table flags)
  u32 ring;        // LDS byte address of this lane's ring column: dword j at ring + j * ENC_SLOT_BYTES.
                   // The ring holds stream dwords as values (first byte in the top bits);
                   // the flush rounds byte-swap them on the way out.
};

// ring dword `slot` of the lane whose column is at LDS byte address `col`
static __device__ __forceinline__ void ring_put(u32 col, u32 slot, u32 v) {
  *(__attribute__((address_space(3))) u32*)(uintptr_t)(col + slot * ENC_SLOT_BYTES) = v;
}

// byte position of the incomplete dword (everything below it has been pushed to the ring)
static __device__ __forceinline__ u32 enc_wpos(const Enc& e) { return (e.B >> 5) << 2; }

// byte position of the next unit to store
static __device__ __forceinline__ u32 enc_fpos(const Enc& e) { return (e.fthr >> 3) - FLUSH_AT; }

// enc_wpos(e) - fpos >= T for T a multiple of 4, tested as B >= 8 (fpos + T): fpos + T is a
// multiple of 4, so rounding B >> 3 down to one (enc_wpos) cannot cross it; against the kept
// threshold fthr = 8 (fpos + FLUSH_AT) that is one compare (T = FLUSH_AT) or an add and one
static __device__ __forceinline__ bool enc_ready(const Enc& e, u32 T) {
  return e.B >= e.fthr - 8u * (FLUSH_AT - T);
}

// Per-chunk output geometry shared with the other lanes of the wave (flush rounds)
struct EncOut {
  uint8_t* gbase;  // 64-B aligned base of the slot
  u32 lo_ok, hi_ok;  // writable byte window [lo_ok, hi_ok) relative to gbase
};

// One flush round.  The chunks of the wave that hold a complete 64-B unit (`has`) are ranked
// (v_mbcnt over their ballot) and listed in the wave's LDS rank table as fpos | lane (fpos is
// a multiple of 64), so the round runs ceil(ready / 16) steps instead of 4: in step j, lane L
// moves granule (L & 3) of the unit of the (16 j + L/4)-th ready chunk.  Granules touching the
// slot edges are written byte by byte (first unit of a misaligned slot, capacity end).
static __device__ __forceinline__ void enc_round(Enc& e, bool has, u32 lane, const u32* wring,
                                                 const EncOut* wout, u32* wrank) {
  const u64 M = __builtin_amdgcn_ballot_w64(has);
  const u32 ready = (u32)__builtin_popcountll(M);  // (wave-uniform: s_bcnt1)
  if (has) {
    const u32 r = __builtin_amdgcn_mbcnt_hi((u32)(M >> 32), __builtin_amdgcn_mbcnt_lo((u32)M, 0u));
    wrank[r] = enc_fpos(e) | lane;
  }
  const u32 g = lane & 3;
#pragma unroll
  for (u32 j = 0; j < 4; ++j) {
    if (16 * j >= ready) break;  // (wave-uniform)
    const u32 k = 16 * j + (lane >> 2);
    const bool act = k < ready;
    if (act) {
      const u32 rec = wrank[k];
      const u32 c = rec & 63u, fp = rec & ~63u;
      // fp is a multiple of ENC_UNIT = 64 B, so the granule's first slot is a multiple of 4 and
      // its 4 dwords never wrap the ring: one address, two ds_read2 (st64 for column-major)
      const u32 slot = ((fp >> 2) + 4 * g) & (ENC_RING - 1);
      constexpr u32 SD = ENC_SLOT_BYTES / 4;  // dwords between slots
      const u32* rp = wring + ring_col(c) + slot * SD;
      const uint4 v = make_uint4(__builtin_bswap32(rp[0]), __builtin_bswap32(rp[SD]),
                                 __builtin_bswap32(rp[2 * SD]), __builtin_bswap32(rp[3 * SD]));
      const EncOut o = wout[c];
      const u32 p0 = fp + 16 * g;
      if (p0 >= o.lo_ok && p0 + 16 <= o.hi_ok) {
        u32x4 g16;
        g16.x = v.x;
        g16.y = v.y;
        g16.z = v.z;
        g16.w = v.w;
        gstore128(o.gbase + p0, g16);
      } else {
        // (rare: the first unit of a misaligned slot, the capacity end) a rolled loop, byte b
        // of the granule in the low byte of r.x: this path is inlined at every flush site, and
        // unrolled it made the encoder's symbol loops too large to unroll themselves
        uint4 r = v;
#pragma unroll 1
        for (u32 b = 0; b < 16; ++b) {
          const u32 p = p0 + b;
          if (p >= o.lo_ok && p < o.hi_ok) gstore8(o.gbase + p, r.x);
          r = make_uint4(__builtin_amdgcn_alignbit(r.y, r.x, 8),
                         __builtin_amdgcn_alignbit(r.z, r.y, 8),
                         __builtin_amdgcn_alignbit(r.w, r.z, 8), r.w >> 8);
        }
      }
    }
  }
  e.fthr += has ? 8u * ENC_UNIT : 0u;
}

// a flush round when some lane's ring is at the threshold (wave-uniform call sites only).  One
// round is enough: a ring never holds more than 4 * ENC_RING - 1 = 127 settled bytes past fpos
// (the static_asserts above), so after it moved a unit every lane holds at most 63 < FLUSH_AT.
static __device__ __forceinline__ void enc_flush(Enc& e, u32 lane, const u32* wring,
                                                 const EncOut* wout, u32* wrank) {
  static_assert(4 * ENC_RING - 1 - ENC_UNIT < FLUSH_AT, "one flush round must suffice");
  if (__builtin_expect(__any((int)enc_ready(e, FLUSH_AT)), 0))
    enc_round(e, enc_ready(e, ENC_UNIT), lane, wring, wout, wrank);
}

// One settled byte, with a conditional push (rare paths only).
static __device__ __forceinline__ void enc_emit_byte(Enc& e, u32 b) {
  e.acc = (e.acc << 8) | b;
  e.B += 8;
  if ((e.B & 31) == 0) ring_put(e.ring, ((e.B >> 5) - 1) & (ENC_RING - 1), (u32)e.acc);
}

// Rare tail of param_update for one lane: the no-carry loop when >= 4 bytes settle
// (range_coder.rs:110-116, continued byte by byte) and range_reduction_expansion (:126-135).
static __device__ __forceinline__ void enc_rare(Enc& e) {
  while (((e.low ^ (e.low + e.range)) >> 56) == 0) {
    enc_emit_byte(e, (u32)(e.low >> 56));
    e.low <<= 8;
    e.range <<= 8;
  }
  while (e.range < TOP16) {
    e.range = ~e.low & (TOP16 - 1);
    enc_emit_byte(e, (u32)(e.low >> 56));
    e.low <<= 8;
    e.range <<= 8;
  }
}

// the output of one symbol: its nb settled bits, the top nb bits of lh (hi32 of the lower bound
// before the shift), into the accumulator and pushed to the ring: the slot of the dword that
// was incomplete before the symbol gets the 32 bits above the (new) incomplete ones; if it is
// still incomplete the slot is rewritten later.  Slot (B >> 5) & (ENC_RING - 1) sits at byte
// 32 slot of the column (ENC_ROWS): ring | (B & 0x3E0), one v_and_or_b32; column-major at byte
// 256 slot, (B & 0x3E0) << 3, an and plus one v_lshl_add_u32 (written out: the compiler's form
// is a shift, an and and an add)
static __device__ __forceinline__ void enc_out(Enc& e, u32 lh, u32 nb) {
#ifndef RC_EXP_NOOUT  // (scratch builds: the coder's arithmetic alone, output dropped; timing only)
  // acc = acc << nb | the top nb bits of lh (nb = 8n, n <= 3), as two byte permutations that
  // share one selector: hi32({a1:a0} << nb) and hi32({a0:lh} << nb), selector byte j = 4 + j - n
  // (for nb = 0 both are the identity).  (From C: a subtract, a bit-field extract, a 64-bit shift
  // and an OR.)
  const u32 sel = hi32(0x0706050403020100ull << nb);
  const u32 a0 = (u32)e.acc, a1 = hi32(e.acc);
  e.acc = ((u64)__builtin_amdgcn_perm(a1, a0, sel) << 32) | __builtin_amdgcn_perm(a0, lh, sel);
  u32 saddr;
  if (ENC_ROWS) {
    saddr = (e.B & ((ENC_RING - 1) << 5)) | e.ring;
  } else {
    u32 soff;
    asm("v_and_b32 %0, %1, %2" : "=v"(soff) : "i"((ENC_RING - 1) << 5), "v"(e.B));
    asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(saddr) : "v"(soff), "v"(e.ring));
  }
  e.B += nb;
  *(__attribute__((address_space(3))) u32*)(uintptr_t)saddr = (u32)(e.acc >> (e.B & 31u));
#endif
}

// Encoder::encode (encoder.rs:24-37) -> RangeCoder::param_update (range_coder.rs:53-92),
// common path without branches, up to the closed-form no_carry_expansion: sets lh (hi32 of the
// lower bound before the shift) and nb (the bits that settle), shifts the state, and returns
// true when the lane needs enc_rare() (after enc_out of this symbol).
// SM: 0 wide model; 1 small model (256 <= total <= 2^16) that may hold entries the reference
// cannot encode; 2 small and complete (256 symbols, every c > 0: nothing to check); 3 the flat
// model (complete, every c = 1, total 256: enc_tab synthesises the entries)
template <int DIV, int SM>
static __device__ __forceinline__ bool enc_core(Enc& e, const ModelArgs& m, uint2 t, u32& lh_out,
                                                u32& nb_out) {
#ifdef RC_FILL
  RC_FILLER(e.fill);
#endif
  u32 c, cum;
  if (SM >= 2) {  // (3: the flat model, c = 1 folds the range product away)
    cum = t.x;
    c = t.y;
  } else if (SM) {  // bad entries were staged as (flag << 24, 1): accumulate, sort out at the end
    // (as an asm OR: left to itself the compiler defers all the ORs to the end of the loop
    // and spills every table entry)
    asm volatile("v_or_b32 %0, %0, %1" : "+v"(e.err) : "v"(t.x));
    cum = t.x & 0xFFFFFFu;
    c = t.y;
  } else {
    const bool bad = t.y == 0;  // zero frequency (reference: endless loop) or outside alphabet
    const u32 code = t.x == 0xFFFFFFFFu ? RC_F_BAD_SYMBOL : RC_F_ZERO_FREQ;
    e.err = (bad && e.err == 0) ? code : e.err;
    c = bad ? 1u : t.y;
    cum = bad ? 0u : t.x;
  }
  const u64 r = range_par_total<DIV, SM>(e.range, m);
  if (SM) {  // r < 2^56, c, cum <= 2^16: low half by v_mad_u64_u32, high by v_mad_u32_u24
    const u32 rl = (u32)r, rh = hi32(r);
    const u64 R0 = (u64)rl * c;                   // range_coder.rs:65
    const u64 L0 = (u64)rl * cum + e.low;         // range_coder.rs:68-81 (no overflow, §3)
    // (the flat model: range = r * 1, written out: __umul24's operand mask would stay)
    e.range = SM == 3 ? r : ((u64)(hi32(R0) + __umul24(rh, c)) << 32) | (u32)R0;
    e.low = ((u64)(hi32(L0) + __umul24(rh, cum)) << 32) | (u32)L0;
  } else {
    e.range = r * (u64)c;
    e.low += r * (u64)cum;
  }
  // no_carry_expansion in closed form: k = clz(low ^ upper) / 8 bytes settle (<= 3 here;
  // equal high halves (ffbh = ~0) mean >= 4 and the rare path continues after these 3)
  const u32 lh = hi32(e.low);
  // (SM: the high halves differ, so clz of a nonzero value, as a builtin: asm would be padded)
  const u32 z = SM ? (u32)__builtin_clz(lh ^ hi32(e.low + e.range)) : ffbh(lh ^ hi32(e.low + e.range));
  const u32 nb = z & 24u;
  e.low <<= nb;
  e.range <<= nb;
  lh_out = lh;
  nb_out = nb;
  // SM: range >= 2^32 after narrowing, so the high halves differ (z <= 31) and at most 3 bytes
  // settle; only range_reduction_expansion can be pending
  if (SM) return hi32(e.range) < 0x10000u;
  return (z > 31u) | (hi32(e.range) < 0x10000u);
}

// a symbol's (cum, c): the model's table entry; SM 3, the flat model (256 symbols, every c = 1,
// total 256): (s, 1) with no table read
template <int SM>
static __device__ __forceinline__ uint2 enc_tab(const uint2* s_tab, u32 s) {
  return SM == 3 ? make_uint2(s, 1u) : s_tab[s];
}

// one symbol, output included
template <int DIV, int SM>
static __device__ __forceinline__ bool enc_step(Enc& e, const ModelArgs& m, uint2 t) {
  u32 lh, nb;
  const bool rare = enc_core<DIV, SM>(e, m, t, lh, nb);
  enc_out(e, lh, nb);
  return rare;
}

// one symbol (table entry t) for the lanes with `act`; the rare path (wave-uniform branch) may
// flush
template <int DIV, int SM>
static __device__ __forceinline__ void enc_sym(Enc& e, const ModelArgs& m, uint2 t, bool act,
                                               u32 lane, const u32* wring, const EncOut* wout,
                                               u32* wrank) {
  bool rare = false;
  if (act) rare = enc_step<DIV, SM>(e, m, t);
  if (__builtin_expect(__any((int)rare), 0)) {
    if (rare) enc_rare(e);
    enc_flush(e, lane, wring, wout, wrank);
  }
}

// Two symbols with ONE rare test (SM models; ENC_PAIR): the second symbol is coded from the
// first's state before its range_reduction_expansion, which is exact for every lane that did not
// need one; a lane that did restores the state after the first symbol (still in registers),
// expands it and codes the second again.  Its speculative ring store went to a slot the redo
// rewrites (the redo's bytes start at the same bit position), so nothing else needs undoing.
// Halves the per-symbol wave-uniform branches, which cost the encoder ~8%.
template <int DIV, int SM>
static __device__ __forceinline__ void enc_sym2(Enc& e, const ModelArgs& m, uint2 t0, uint2 t1,
                                                bool act, u32 lane, const u32* wring,
                                                const EncOut* wout, u32* wrank) {
  bool r0 = false, r1 = false;
  if (act) r0 = enc_step<DIV, SM>(e, m, t0);
  const Enc ea = e;
  if (act) r1 = enc_step<DIV, SM>(e, m, t1);
  if (__builtin_expect(__any((int)(r0 | r1)), 0)) {
    if (r0) {
      e = ea;
      enc_rare(e);
      r1 = enc_step<DIV, SM>(e, m, t1);
    }
    if (r1) enc_rare(e);
    enc_flush(e, lane, wring, wout, wrank);
  }
}

// 16 symbols from one 16-B load, a flush check after every 8 (wave-uniform).  The table entry
// of the next symbol is read before the current symbol is coded, so the LDS latency is off the
// range -> range dependency chain.
template <int DIV, int SM>
static __device__ __forceinline__ void enc16(Enc& e, const ModelArgs& m, const uint2* s_tab,
                                             uint4 v, bool act, u32 lane, const u32* wring,
                                             const EncOut* wout, u32* wrank) {
  // the words rotate down (w0 holds the current 4 symbols) instead of being indexed: a rolled
  // loop would select w[i >> 2] with v_cndmask_b32 on VCC (~13 extra SIMD cycles each)
  u32 w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
  uint2 t = enc_tab<SM>(s_tab, w0 & 255u);
  auto quarter = [&](int q) {
    if (ENC_PAIR && SM) {
      // table entries two symbols ahead (the pair's second and the next pair's first)
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const uint2 t1 = enc_tab<SM>(s_tab, (w0 >> (8 * (i + 1))) & 255u);
        const u32 sn = i < 2 ? (w0 >> (8 * (i + 2))) & 255u : w1 & 255u;
        const uint2 tn = enc_tab<SM>(s_tab, sn);  // (past the tile's end: a harmless extra read)
        enc_sym2<DIV, SM>(e, m, t, t1, act, lane, wring, wout, wrank);
        t = tn;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32 sn = i < 3 ? (w0 >> (8 * (i + 1))) & 255u : w1 & 255u;
        const uint2 tn = enc_tab<SM>(s_tab, sn);  // (past the tile's end: a harmless extra read)
        enc_sym<DIV, SM>(e, m, t, act, lane, wring, wout, wrank);
        t = tn;
      }
    }
    if (q & 1) enc_flush(e, lane, wring, wout, wrank);
    w0 = w1;
    w1 = w2;
    w2 = w3;
  };
  // Small models: all four quarters unrolled (the word rotation then costs nothing); wide models
  // hold more state, and unrolled four times their encoder spills, so they unroll by two
  if (SM) {
#pragma unroll
    for (int q = 0; q < 4; ++q) quarter(q);
  } else {
#pragma unroll 2
    for (int q = 0; q < 4; ++q) quarter(q);
  }
}

// one symbol fetched byte-wise (unaligned head / tail of a chunk)
template <int DIV, int SM>
static __device__ __forceinline__ void enc_byte_sym(Enc& e, const ModelArgs& m,
                                                    const uint2* s_tab, const uint8_t* sp, u64 i,
                                                    bool act, u32 lane, const u32* wring,
                                                    const EncOut* wout, u32* wrank) {
  const u32 sym = act ? (u32)sp[i] : 0u;
  enc_sym<DIV, SM>(e, m, enc_tab<SM>(s_tab, sym), act, lane, wring, wout, wrank);
}

// the first symbol of a chunk the reference cannot encode (rare: flagged chunks only)
static __device__ u32 enc_first_error(const ModelArgs& m, const uint8_t* sp, u64 n) {
  for (u64 i = 0; i < n; ++i) {
    const u32 s = sp[i];
    if (s >= m.n) return RC_F_BAD_SYMBOL;  // sample_impl.rs:19 (Vec::get().unwrap())
    if (m.tab[s].y == 0) return RC_F_ZERO_FREQ;  // range_coder.rs:83-85 (endless loop)
  }
  return 0;
}

template <int DIV, int SM>
__global__ __launch_bounds__(WG, ENC_WAVES) void k_encode_static(ModelArgs m, const uint8_t* __restrict__ syms,
                                                        const u64* __restrict__ sym_off,
                                                        u32 n_chunks, uint8_t* __restrict__ out,
                                                        const u64* __restrict__ out_off,
                                                        u64* __restrict__ out_len,
                                                        u32* __restrict__ flags) {
  RC_STAMP_BEGIN();
  rc_set_prio(m);
  __shared__ uint2 s_tab[256];
  // (1-KiB aligned: a column base has no bits in the row field, ENC_ROWS)
  __shared__ __attribute__((aligned(1024))) u32 s_ring[WAVES * ENC_RING * 64];
  __shared__ EncOut s_out[WG];
  __shared__ u32 s_rank[WG];  // per wave: the lanes holding a unit, by rank (flush rounds)
  const u32 tid = threadIdx.x;
  {
    // SM (cum < 2^16): a symbol the reference cannot encode (c == 0: endless loop; outside the
    // alphabet: panic) is staged as (flag << 24, c = 1), so the common path only ORs entries
    // together; a chunk whose OR shows a flag is re-scanned for its first error at the end
    uint2 t = m.tab[tid];
    if (SM == 1 && t.y == 0)
      t = make_uint2((t.x == 0xFFFFFFFFu ? RC_F_BAD_SYMBOL : RC_F_ZERO_FREQ) << 24, 1u);
    s_tab[tid] = t;
  }
  const u32 lane = tid & 63, wave = tid >> 6;
  const u32 k = blockIdx.x * WG + tid;
  const bool live = k < n_chunks;  // dead lanes still take part in the wave's flush rounds
#if ENC_WAVES == 4
  RC_VGPR_FLOOR_128();
#endif

  u64 s0 = 0, n = 0, o0 = 0, o1 = 0;
  if (live) {
    s0 = sym_off[k];
    n = sym_off[k + 1] - s0;
    o0 = out_off[k];
    o1 = out_off[k + 1];
  }
  // B (bit position) is 32-bit: a longer chunk is flagged, not read, and its slot not written
  const bool too_long = n > RC_MAX_CHUNK_SYMBOLS;
  if (too_long) {
    n = 0;
    o1 = o0;
  }
  const u32 a = (u32)(((uintptr_t)out + o0) & (ENC_UNIT - 1));
  u64 cap = o1 - o0;
  if (cap > 0xFFFFFF00ull - a) cap = 0xFFFFFF00ull - a;
  s_out[tid].gbase = out + o0 - a;
  s_out[tid].lo_ok = a;
  s_out[tid].hi_ok = a + (u32)cap;
  __syncthreads();
  const u32* wring = s_ring + wave * ENC_RING * 64;
  const EncOut* wout = s_out + wave * 64;
  u32* const wrank = s_rank + wave * 64;

  Enc e;
#ifdef RC_FILL
  e.fill = 0;
#endif
  e.low = 0;  // RangeCoder::default (range_coder.rs:13-20)
  e.range = ~0ull;
  e.acc = 0;
  e.B = 8 * a;  // pad bytes in front of the slot (never stored)
  e.fthr = 8u * FLUSH_AT;  // fpos = 0
  e.err = 0;
  e.ring = (u32)(uintptr_t)(__attribute__((address_space(3))) u32*)(s_ring + wave * ENC_RING * 64 +
                                                                     ring_col(lane));

  const uint8_t* sp = syms + s0;
  u64 head = (64 - ((uintptr_t)sp & 63)) & 63;  // symbols before the first 64-B aligned tile
  if (head > n) head = n;
  const u64 ntile = (n - head) >> 6;
  // head: byte-wise, all lanes in step (flush rounds are wave-wide)
  for (u64 i = 0; __any((int)(i < head)); ++i) {
    enc_byte_sym<DIV, SM>(e, m, s_tab, sp, i, i < head, lane, wring, wout, wrank);
    if ((i & 7) == 7) enc_flush(e, lane, wring, wout, wrank);
  }
  // body, part 1: the tiles every live lane of the wave has, with every lane active (no
  // per-symbol exec masking).  Dead lanes run along on a dummy tile (g_sink, zeros) and a slot
  // with no writable bytes; their results are dropped.
  u64 tm = live ? ntile : ~0ull;
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const u64 v = ((u64)(u32)__shfl_xor((int)hi32(tm), o) << 32) | (u32)__shfl_xor((int)(u32)tm, o);
    tm = v < tm ? v : tm;
  }
  if (tm == ~0ull) tm = 0;  // no live lane in this wave
  const u64 tmin = ((u64)__builtin_amdgcn_readfirstlane(hi32(tm)) << 32) |
                   __builtin_amdgcn_readfirstlane((u32)tm);  // wave-uniform (scalar) trip count
  const uint4* tp = live ? reinterpret_cast<const uint4*>(sp + head)
                         : reinterpret_cast<const uint4*>(g_sink);
  // 64-symbol tiles, 4 x 16 B per lane, the next tile in flight while the current one is coded
  // (explicit registers: as arrays the compiler put the tiles in scratch memory, round 5).
  // ENC_TILE_Q 2 (scratch builds): 32-symbol half tiles, 16 registers fewer.
  const u64 tstep = live ? ENC_TILE_Q : 0;  // uint4s per load
  const u64 trips = tmin * (4 / ENC_TILE_Q);
  uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, c2 = c0, c3 = c0;
  if (trips) {
    c0 = tp[0];
    c1 = tp[1];
    if (ENC_TILE_Q == 4) {
      c2 = tp[2];
      c3 = tp[3];
    }
  }
  for (u64 t = 0; t < trips; ++t) {
    rc_prio_rotate(m.prio_rot);
    uint4 n0 = c0, n1 = c1, n2 = c2, n3 = c3;
    if (t + 1 < trips) {
      const uint4* q = tp + (t + 1) * tstep;
      n0 = q[0];
      n1 = q[1];
      if (ENC_TILE_Q == 4) {
        n2 = q[2];
        n3 = q[3];
      }
    }
    enc16<DIV, SM>(e, m, s_tab, c0, true, lane, wring, wout, wrank);
    enc16<DIV, SM>(e, m, s_tab, c1, true, lane, wring, wout, wrank);
    if (ENC_TILE_Q == 4) {
      enc16<DIV, SM>(e, m, s_tab, c2, true, lane, wring, wout, wrank);
      enc16<DIV, SM>(e, m, s_tab, c3, true, lane, wring, wout, wrank);
    }
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
  }
  // body, part 2 (ragged waves): the remaining 16-symbol blocks of the tiles, lanes masked
  const u64 nblk = ntile * 4;
  for (u64 b = tmin * 4; __any((int)(b < nblk)); ++b) {
    const bool act = b < nblk;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (act) v = tp[b];
    enc16<DIV, SM>(e, m, s_tab, v, act, lane, wring, wout, wrank);
  }
  const u64 tail0 = head + (ntile << 6);
  for (u64 j = 0; __any((int)(tail0 + j < n)); ++j) {  // j is wave-uniform
    enc_byte_sym<DIV, SM>(e, m, s_tab, sp, tail0 + j, tail0 + j < n, lane, wring, wout,
                          wrank);
    if ((j & 7) == 7) enc_flush(e, lane, wring, wout, wrank);
  }

  // Encoder::finish (encoder.rs:40-46): 8 x left_shift
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    enc_emit_byte(e, (u32)(e.low >> 56));
    e.low <<= 8;
  }
  const u32 len = (e.B >> 3) - a;
  u32 wend = enc_wpos(e);
  if (e.B & 31) {  // the last, incomplete dword
    ring_put(e.ring, (e.B >> 5) & (ENC_RING - 1), (u32)(e.acc << (32 - (e.B & 31))));
    wend += 4;
  }
  // final rounds: the last (partial) units, clipped to the stream end
  const u32 end = a + len;
  if (end < s_out[tid].hi_ok) s_out[tid].hi_ok = end;
  while (__any((int)(enc_fpos(e) < wend)))
    enc_round(e, enc_fpos(e) < wend, lane, wring, wout, wrank);
  RC_STAMP_END(enc, blockIdx.x * WAVES + wave, lane, n);
  if (live) {
    if (SM == 1) e.err = (e.err >> 24) ? enc_first_error(m, sp, n) : 0u;
    if (!e.err && (u64)len > cap) e.err = RC_F_CAPACITY;
    out_len[k] = too_long ? 0u : len;
    flags[k] = too_long ? RC_F_TOO_LONG : e.err;
  }
}


u32 rc_resident_wgs(const void* kernel, int block, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, u32> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_tuple(dev, kernel, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return cache[key] = (u32)(per_cu * cus);
}

hipError_t rc_static_encode_launch(hipStream_t stream, const RcKnobs& k, const ModelArgs& a_in,
                                   int div, int smv, const uint8_t* syms, const u64* sym_off,
                                   u32 n_chunks, uint8_t* out, const u64* out_off, u64* out_len,
                                   u32* flags) {
  const dim3 grid((n_chunks + WG - 1) / WG), block(WG);
  ModelArgs a = a_in;
  // (the launch's wave priorities: rc_static.h)
  auto go = [&](auto kern) {
    rc_prio_policy(a, kPrioEncoder, grid.x,
                   rc_resident_wgs(reinterpret_cast<const void*>(kern), WG, 0), k);
    hipLaunchKernelGGL(kern, grid, block, 0, stream, a, syms, sym_off, n_chunks, out, out_off,
                       out_len, flags);
  };
#ifdef RC_DEV_ONLY  // scratch builds for kernel tuning: the headline variants only
  if (div != DIV_POW2 || smv == 0) return hipErrorInvalidValue;
  if (a.flat) go(k_encode_static<DIV_POW2, 3>);
  else if (smv == 2) go(k_encode_static<DIV_POW2, 2>); else go(k_encode_static<DIV_POW2, 1>);
#else
  if (div == DIV_POW2) {
    if (a.flat) go(k_encode_static<DIV_POW2, 3>);  // the flat model (SM 3: no table reads)
    else if (smv == 2) go(k_encode_static<DIV_POW2, 2>);
    else if (smv == 1) go(k_encode_static<DIV_POW2, 1>);
    else go(k_encode_static<DIV_POW2, 0>);
  } else {
    if (smv == 2) go(k_encode_static<DIV_MAGIC, 2>);
    else if (smv == 1) go(k_encode_static<DIV_MAGIC, 1>);
    else go(k_encode_static<DIV_MAGIC, 0>);
  }
#endif
  return hipGetLastError();
}
