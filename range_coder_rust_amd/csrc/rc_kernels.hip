// rc_kernels.hip — MI355X (gfx950) kernels of the batched range coder.
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
#include "rc_common.h"

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
#ifndef DEC_OUT_BURST
#define DEC_OUT_BURST 4      // 16-B symbol blocks per lane per output burst (4: 64 B)
#endif
#ifndef DEC_TAB_LDS
#define DEC_TAB_LDS 1        // direct-LUT decoders: keep the (cum, c) table in LDS too
#endif
#define LUT_BITS 12
#define LUT_MAX_ENTRIES (1u << LUT_BITS)

enum { DIV_POW2 = 0, DIV_MAGIC = 1 };

struct ModelArgs {
  const uint2* tab;  // [256] (cum, c); entries s >= n_symbols hold (0xFFFFFFFF, 0)
  const u32* lut;    // decoder buckets: s0 | s1 << 8 | split << 16
  u64 magic;         // floor((2^64 - 1) / total) for DIV_MAGIC
  u32 n;             // alphabet size (1..256)
  u32 total;         // total_freq
  u32 lg;            // log2(total) for DIV_POW2
  u32 lut_shift;     // bucket = q >> lut_shift
  u32 lut_max;       // number of buckets - 1
  float ftotal;      // (float)total
  u32 direct;        // 1: lut[q] = s | cum << 8 | c << 20 for every q < total (total <= 2048)
                     // 2: lut[4q..4q+3] = {cum, c, s, total/c as f32} (256 <= total <= 512)
};


// RangeCoder::range_par_total (range_coder.rs:38-40): range / total, exact.
template <int DIV>
static __device__ __forceinline__ u64 range_par_total(u64 range, const ModelArgs& m) {
  if (DIV == DIV_POW2) return range >> m.lg;
  u64 q = __umul64hi(range, m.magic);  // q in {floor - 1, floor}
  u64 rem = range - q * (u64)m.total;
  return rem >= (u64)m.total ? q + 1 : q;
}

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
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(hi32(r)), "v"(v), "v"(hi32(p)));
    return ((u64)h << 32) | (u32)p;
  }
  return r * (u64)v;
}

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
#define FLUSH_AT 88    // ring fill forcing a flush round: 88 + 7*3 + 3 + 11 (rare tail) < 124
#define SINK_SLOTS 65536
__device__ uint4 g_sink[SINK_SLOTS];  // dummy symbol tiles of dead lanes (contents irrelevant)

struct Enc {
  u64 low, range;  // RangeCoder state (range_coder.rs:7-12)
  u64 acc;         // settled bytes, newest in the low bits; the B & 31 lowest are not pushed
  u32 B;           // bit position of the next settled byte, from the 64-B aligned slot base:
                   // dword B >> 5 of the stream is the incomplete one (its ring slot is free)
  u32 fpos;        // byte position of the next unit to store
  u32 err;         // first RC_F_* error of this chunk (SM: OR of staged table flags)
  u32 ring;        // LDS byte address of this lane's ring column: dword j at ring + 256 * j.
                   // The ring holds stream dwords as values (first byte in the top bits);
                   // the flush rounds byte-swap them on the way out.
};

// ring dword `slot` of the lane whose column is at LDS byte address `col`
static __device__ __forceinline__ void ring_put(u32 col, u32 slot, u32 v) {
  *(__attribute__((address_space(3))) u32*)(uintptr_t)(col + (slot << 8)) = v;
}

// byte position of the incomplete dword (everything below it has been pushed to the ring)
static __device__ __forceinline__ u32 enc_wpos(const Enc& e) { return (e.B >> 5) << 2; }

// v_ffbh_u32 as the hardware defines it: 0xFFFFFFFF for 0 (the clz builtins are undefined there)
static __device__ __forceinline__ u32 ffbh(u32 v) {
  u32 r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// Per-chunk output geometry shared with the other lanes of the wave (flush rounds)
struct EncOut {
  uint8_t* gbase;  // 64-B aligned base of the slot
  u32 lo_ok, hi_ok;  // writable byte window [lo_ok, hi_ok) relative to gbase
};

// One flush round.  Lane L of the wave moves granule (L & 3) of the unit of chunk 16*i + L/4
// for i = 0..3; chunks with has == false are masked.  Granules touching the slot edges are
// written byte by byte (first unit of a misaligned slot, capacity end).
static __device__ __forceinline__ void enc_round(Enc& e, bool has, u32 lane, const u32* wring,
                                                 const EncOut* wout) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32 c = 16 * i + (lane >> 2), g = lane & 3;
    const bool hc = __shfl((int)has, c) != 0;
    const u32 fp = (u32)__shfl((int)e.fpos, c);
    if (hc) {
      const u32 slot = (fp >> 2) + 4 * g;
      const u32* rp = wring + c;
      const uint4 v = make_uint4(__builtin_bswap32(rp[((slot + 0) & (ENC_RING - 1)) * 64]),
                                 __builtin_bswap32(rp[((slot + 1) & (ENC_RING - 1)) * 64]),
                                 __builtin_bswap32(rp[((slot + 2) & (ENC_RING - 1)) * 64]),
                                 __builtin_bswap32(rp[((slot + 3) & (ENC_RING - 1)) * 64]));
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
        const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const u32 p = p0 + j;
          if (p >= o.lo_ok && p < o.hi_ok) gstore8(o.gbase + p, w[j >> 2] >> (8 * (j & 3)));
        }
      }
    }
  }
  e.fpos += has ? (u32)ENC_UNIT : 0u;
}

// flush rounds until no lane's ring is above the threshold (wave-uniform call sites only)
static __device__ __forceinline__ void enc_flush(Enc& e, u32 lane, const u32* wring,
                                                 const EncOut* wout) {
  while (__any((int)(enc_wpos(e) - e.fpos >= FLUSH_AT)))
    enc_round(e, enc_wpos(e) - e.fpos >= ENC_UNIT, lane, wring, wout);
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

// Encoder::encode (encoder.rs:24-37) -> RangeCoder::param_update (range_coder.rs:53-92),
// common path without branches.  Returns true when the lane needs enc_rare().  Written for the
// gfx950 VALU price list (profiles/r01/ubench_valu.txt): 64-bit ops, multiplies, compares and
// bit-field ops cost ~3.6 cycles per wave, plain 32-bit add/logic/right-shift ~2.
// SM: 0 wide model; 1 small model (256 <= total <= 2^16) that may hold entries the reference
// cannot encode; 2 small and complete (256 symbols, every c > 0: nothing to check)
template <int DIV, int SM>
static __device__ __forceinline__ bool enc_step(Enc& e, const ModelArgs& m, uint2 t) {
  u32 c, cum;
  if (SM == 2) {
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
  const u64 r = range_par_total<DIV>(e.range, m);
  if (SM) {  // r < 2^56, c, cum <= 2^16: low half by v_mad_u64_u32, high by v_mad_u32_u24
    const u32 rl = (u32)r, rh = hi32(r);
    const u64 R0 = (u64)rl * c;                   // range_coder.rs:65
    const u64 L0 = (u64)rl * cum + e.low;         // range_coder.rs:68-81 (no overflow, §3)
    e.range = ((u64)(hi32(R0) + __umul24(rh, c)) << 32) | (u32)R0;
    e.low = ((u64)(hi32(L0) + __umul24(rh, cum)) << 32) | (u32)L0;
  } else {
    e.range = r * (u64)c;
    e.low += r * (u64)cum;
  }
  // no_carry_expansion in closed form: k = clz(low ^ upper) / 8 bytes settle (<= 3 here;
  // equal high halves (ffbh = ~0) mean >= 4 and the rare path continues after these 3)
  const u32 lh = hi32(e.low);
  const u32 z = ffbh(lh ^ hi32(e.low + e.range));
  const u32 nb = z & 24u;
  const u32 bytes = __builtin_amdgcn_ubfe(lh, 32u - nb, nb);  // the top nb bits (0 if nb == 0)
  e.acc = (e.acc << nb) | bytes;
  e.low <<= nb;
  e.range <<= nb;
  // push: the slot of the dword that was incomplete before this symbol gets the 32 bits above
  // the (new) incomplete ones; if it is still incomplete the slot is rewritten later
  const u32 slot = __builtin_amdgcn_ubfe(e.B, 5, 5);  // (B >> 5) & (ENC_RING - 1): v_bfe_u32
  e.B += nb;
  ring_put(e.ring, slot, (u32)(e.acc >> (e.B & 31u)));
  // SM: range >= 2^32 after narrowing, so the high halves differ (z <= 31) and at most 3 bytes
  // settle; only range_reduction_expansion can be pending
  if (SM) return hi32(e.range) < 0x10000u;
  return (z > 31u) | (hi32(e.range) < 0x10000u);
}

// one symbol (table entry t) for the lanes with `act`; the rare path (wave-uniform branch) may
// flush
template <int DIV, int SM>
static __device__ __forceinline__ void enc_sym(Enc& e, const ModelArgs& m, uint2 t, bool act,
                                               u32 lane, const u32* wring, const EncOut* wout) {
  bool rare = false;
  if (act) rare = enc_step<DIV, SM>(e, m, t);
  if (__builtin_expect(__any((int)rare), 0)) {
    if (rare) enc_rare(e);
    enc_flush(e, lane, wring, wout);
  }
}

// 16 symbols from one 16-B load, a flush check after every 8 (wave-uniform).  The table entry
// of the next symbol is read before the current symbol is coded, so the LDS latency is off the
// range -> range dependency chain.
template <int DIV, int SM>
static __device__ __forceinline__ void enc16(Enc& e, const ModelArgs& m, const uint2* s_tab,
                                             uint4 v, bool act, u32 lane, const u32* wring,
                                             const EncOut* wout) {
  // the words rotate down (w0 holds the current 4 symbols) instead of being indexed: a rolled
  // loop would select w[i >> 2] with v_cndmask_b32 on VCC (~13 extra SIMD cycles each)
  u32 w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
  uint2 t = s_tab[w0 & 255u];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32 sn = i < 3 ? (w0 >> (8 * (i + 1))) & 255u : w1 & 255u;
      const uint2 tn = s_tab[sn];  // (past the tile's end: a harmless extra read)
      enc_sym<DIV, SM>(e, m, t, act, lane, wring, wout);
      t = tn;
    }
    if (q & 1) enc_flush(e, lane, wring, wout);
    w0 = w1;
    w1 = w2;
    w2 = w3;
  }
}

// one symbol fetched byte-wise (unaligned head / tail of a chunk)
template <int DIV, int SM>
static __device__ __forceinline__ void enc_byte_sym(Enc& e, const ModelArgs& m,
                                                    const uint2* s_tab, const uint8_t* sp, u64 i,
                                                    bool act, u32 lane, const u32* wring,
                                                    const EncOut* wout) {
  const u32 sym = act ? (u32)sp[i] : 0u;
  enc_sym<DIV, SM>(e, m, s_tab[sym], act, lane, wring, wout);
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
__global__ __launch_bounds__(WG, 4) void k_encode_static(ModelArgs m, const uint8_t* __restrict__ syms,
                                                        const u64* __restrict__ sym_off,
                                                        u32 n_chunks, uint8_t* __restrict__ out,
                                                        const u64* __restrict__ out_off,
                                                        u64* __restrict__ out_len,
                                                        u32* __restrict__ flags) {
  __shared__ uint2 s_tab[256];
  __shared__ u32 s_ring[WAVES * ENC_RING * 64];
  __shared__ EncOut s_out[WG];
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
  RC_VGPR_FLOOR_128();

  u64 s0 = 0, n = 0, o0 = 0, o1 = 0;
  if (live) {
    s0 = sym_off[k];
    n = sym_off[k + 1] - s0;
    o0 = out_off[k];
    o1 = out_off[k + 1];
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

  Enc e;
  e.low = 0;  // RangeCoder::default (range_coder.rs:13-20)
  e.range = ~0ull;
  e.acc = 0;
  e.B = 8 * a;  // pad bytes in front of the slot (never stored)
  e.fpos = 0;
  e.err = 0;
  e.ring = (u32)(uintptr_t)(__attribute__((address_space(3))) u32*)(s_ring + wave * ENC_RING * 64 + lane);

  const uint8_t* sp = syms + s0;
  u64 head = (64 - ((uintptr_t)sp & 63)) & 63;  // symbols before the first 64-B aligned tile
  if (head > n) head = n;
  const u64 ntile = (n - head) >> 6;
  // head: byte-wise, all lanes in step (flush rounds are wave-wide)
  for (u64 i = 0; __any((int)(i < head)); ++i) {
    enc_byte_sym<DIV, SM>(e, m, s_tab, sp, i, i < head, lane, wring, wout);
    if ((i & 7) == 7) enc_flush(e, lane, wring, wout);
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
  const u64 tstep = live ? 4 : 0;  // uint4s per tile
  uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, c2 = c0, c3 = c0;
  if (tmin) {
    c0 = tp[0];
    c1 = tp[1];
    c2 = tp[2];
    c3 = tp[3];
  }
  for (u64 t = 0; t < tmin; ++t) {
    uint4 n0 = c0, n1 = c1, n2 = c2, n3 = c3;
    if (t + 1 < tmin) {
      const uint4* q = tp + (t + 1) * tstep;
      n0 = q[0];
      n1 = q[1];
      n2 = q[2];
      n3 = q[3];
    }
    enc16<DIV, SM>(e, m, s_tab, c0, true, lane, wring, wout);
    enc16<DIV, SM>(e, m, s_tab, c1, true, lane, wring, wout);
    enc16<DIV, SM>(e, m, s_tab, c2, true, lane, wring, wout);
    enc16<DIV, SM>(e, m, s_tab, c3, true, lane, wring, wout);
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
    enc16<DIV, SM>(e, m, s_tab, v, act, lane, wring, wout);
  }
  const u64 tail0 = head + (ntile << 6);
  for (u64 j = 0; __any((int)(tail0 + j < n)); ++j) {  // j is wave-uniform
    enc_byte_sym<DIV, SM>(e, m, s_tab, sp, tail0 + j, tail0 + j < n, lane, wring, wout);
    if ((j & 7) == 7) enc_flush(e, lane, wring, wout);
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
  while (__any((int)(e.fpos < wend))) enc_round(e, e.fpos < wend, lane, wring, wout);
  if (live) {
    if (SM == 1) e.err = (e.err >> 24) ? enc_first_error(m, sp, n) : 0u;
    if (!e.err && (u64)len > cap) e.err = RC_F_CAPACITY;
    out_len[k] = len;
    flags[k] = e.err;
  }
}

// ------------------------------------------------------------------------------------------
// Decoder
//
// Per lane: one chunk.  The code stream is staged through a per-lane 128-B LDS ring (+4
// mirror dwords so a 20-byte window never wraps), refilled 64 B at a time: at each 16-symbol
// phase boundary a lane stores its 16 decoded symbols, moves its pending 64-B load into the
// ring and, if the ring has room, issues the next 64-B load.  The pending load is therefore
// waited for with vmcnt(1) one phase after it was issued.  Lanes that consume faster than the
// ring covers (rare renormalisation bursts) are refilled synchronously.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) u32 l_u32;

struct Dec {
  u64 low, range;  // RangeCoder (decoder.rs:6-12)
  // Decoder::data - lower_bound (mod 2^64): all find_index needs (sample_impl.rs:29).  Kept as
  // two 32-bit halves: as a u64 it must sit in an even-aligned VGPR pair, which costs a move
  // per symbol when its new halves are produced in other registers.
  u32 xlo, xhi;
  float G;  // 16-B direct tables: 16 * total / (range / 2^32), carried from symbol to symbol
  __device__ __forceinline__ u64 x() const { return ((u64)xhi << 32) | xlo; }
  __device__ __forceinline__ void set_x(u64 v) { xlo = (u32)v; xhi = hi32(v); }
  u32 cpos;   // bytes consumed, relative to the 16-B aligned base of the code stream
  u32 fill;   // bytes staged into the ring, same origin
  u32 lim;    // cpos > lim: more bytes consumed than the stream holds
  u32 err;
  u32 pend_ok;           // 32-B refills still held in pend[] (a load burst gives DEC_LD / DEC_PF)
  l_u32* ring;           // this lane's ring column: dword j at ring[j * 64] (LDS pointer)
  const uint4* gbase;    // 16-B aligned base of the stream
  u32 gnext;             // next 16-B block (index from gbase)
  u32 glast;             // last block holding a byte of this chunk (fetch clamp)
  uint4 pend[DEC_LD];
};

static __device__ __forceinline__ void dec_issue(Dec& d) {
#pragma unroll
  for (int q = 0; q < DEC_LD; ++q) {
    // 32-bit block index clamp (v_min_u32): a 64-bit pointer compare would select on VCC
    const uint4* p = d.gbase + min(d.gnext + q, d.glast);
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)p;  // global, not flat
    d.pend[q] = make_uint4(v.x, v.y, v.z, v.w);
  }
  d.gnext += DEC_LD;
  d.pend_ok = DEC_LD / DEC_PF;
}

// move the next DEC_PF pending blocks into the ring (pend[0..DEC_PF) hold them)
static __device__ __forceinline__ void dec_commit(Dec& d) {
  const u32 j = (d.fill >> 2) & (DEC_RING - 1);
  l_u32* rp = d.ring + j * 64;
#pragma unroll
  for (int q = 0; q < DEC_PF; ++q) {
    rp[(4 * q + 0) * 64] = d.pend[q].x;
    rp[(4 * q + 1) * 64] = d.pend[q].y;
    rp[(4 * q + 2) * 64] = d.pend[q].z;
    rp[(4 * q + 3) * 64] = d.pend[q].w;
  }
  if (j == 0) {  // mirror slots
    rp[DEC_RING * 64] = d.pend[0].x;
    rp[(DEC_RING + 1) * 64] = d.pend[0].y;
    if (DEC_MIRROR > 2) rp[(DEC_RING + 2) * 64] = d.pend[0].z;
    if (DEC_MIRROR > 3) rp[(DEC_RING + 3) * 64] = d.pend[0].w;
  }
#pragma unroll
  for (int q = 0; q + DEC_PF < DEC_LD; ++q) d.pend[q] = d.pend[q + DEC_PF];
  d.fill += 16 * DEC_PF;
  d.pend_ok -= 1;
}

// phase boundary: commit the pending load, issue the next one if the ring has room
// (the ring has room for a refill once at most 4 * DEC_RING - 16 * DEC_PF bytes are unread;
// a 64-B load burst feeds two refills, so every lane's global reads are whole 64-B segments)
static __device__ __forceinline__ void dec_phase(Dec& d) {
  if (d.pend_ok && (int)(d.fill - d.cpos) <= 4 * DEC_RING - 16 * DEC_PF) dec_commit(d);
  if (!d.pend_ok) dec_issue(d);
}

// a lane about to read past the staged bytes: commit / load synchronously (rare)
static __device__ __forceinline__ void dec_sync(Dec& d, u32 need) {
  while ((int)(d.fill - d.cpos) < (int)need) {
    if (!d.pend_ok) dec_issue(d);
    dec_commit(d);
  }
}

// the 8 code bytes ending at cpos, big-endian (Decoder::new's priming, decoder.rs:14-23)
static __device__ __forceinline__ u64 dec_read8_before(const Dec& d) {
  const u32 p = d.cpos - 8;
  const l_u32* rp = d.ring + ((p >> 2) & (DEC_RING - 1)) * 64;
  const u32 d0 = rp[0], d1 = rp[64], d2 = rp[128];
  const u32 sh = p & 3;
  const u32 w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const u32 w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  return ((u64)__builtin_bswap32(w0) << 32) | __builtin_bswap32(w1);
}

// range_reduction_expansion (range_coder.rs:126-135): each iteration settles one more byte,
// which Decoder::shift_left_buffer (decoder.rs:31-35) shifts into data (so into x = data-low)
static __device__ __forceinline__ void dec_rare(Dec& d, u32 need) {
  u32 m = 0;
  while (d.range < TOP16) {
    d.range = ~d.low & (TOP16 - 1);
    d.low <<= 8;
    d.range <<= 8;
    ++m;
  }
  dec_sync(d, m + need);
  for (u32 j = 0; j < m; ++j, ++d.cpos) {
    const u32 w = d.ring[((d.cpos >> 2) & (DEC_RING - 1)) * 64];
    d.set_x((d.x() << 8) | ((w >> (8 * (d.cpos & 3))) & 255u));
  }
}

// the exact index: s = #{ j in [1, n-1] : r * cum[j] <= x }  (FreqTable::find_index)
static __device__ __forceinline__ void dec_fix(u32& s, uint2& t, u64& A, u64& B, u64 x,
                                                        u64 r, const uint2* s_tab, u32 n) {
  s &= 255u;
  if (A > x) {
    do {
      --s;
      t = s_tab[s];
      A = r * (u64)t.x;
    } while (A > x);
    B = r * (u64)t.y;
  } else {
    while (s + 1 < n && x - A >= B) {
      ++s;
      t = s_tab[s];
      A = r * (u64)t.x;
      B = r * (u64)t.y;
    }
  }
}

// Decoder::decode (decoder.rs:38-54) with FreqTable::find_index (sample_impl.rs:27-45).
// SM: 256 <= total <= 2^16 (then range >= 2^32 after narrowing, so at most 3 bytes settle).
// u32 -> f32 as the single instruction; written out because hipcc otherwise widens a
// (float)hi32(v) back into its multi-instruction u64 -> f32 sequence
static __device__ __forceinline__ float cvt_f32(u32 v) {
  float f;
  asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"(v));
  return f;
}

// float -> u32 as the single instruction, which saturates (negative -> 0, >= 2^32 -> 2^32 - 1)
static __device__ __forceinline__ u32 cvt_u32_sat(float f) {
  u32 v;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(v) : "v"(f));
  return v;
}

// code bytes a symbol may consume before the next ring check: SM checks once per 4 symbols
// (<= 3 bytes each), otherwise every symbol (<= 7 bytes)
#define DEC_NEED_SM 12u
#define DEC_NEED_WIDE 8u

// byte j of w = byte 0 of v, other bytes kept (j = 0: cleared): one v_mov_b32_sdwa
static __device__ __forceinline__ u32 put_byte(u32 w, u32 v, int j) {
  switch (j) {
    case 0:
      asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0"
          : "=v"(w) : "v"(v));
      break;
    case 1:
      asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0"
          : "+v"(w) : "v"(v));
      break;
    case 2:
      asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0"
          : "+v"(w) : "v"(v));
      break;
    default:
      asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0"
          : "+v"(w) : "v"(v));
  }
  return w;
}

// the hint scale of 16-B direct tables, exactly (from the top 32 bits of range)
static __device__ __forceinline__ void dec_gexact(Dec& d, const ModelArgs& m) {
  d.G = (16.0f * m.ftotal) * __builtin_amdgcn_rcpf(cvt_f32(hi32(d.range)));
}

template <int DIV, int SM, int LUT>
static __device__ __forceinline__ u32 dec_sym(Dec& d, const ModelArgs& m, const uint2* s_tab,
                                              const u32* s_lut) {
  // the code bytes at cpos (the ring holds the ones this symbol can settle); they are shifted
  // into x at the end
  const l_u32* rp = d.ring + ((d.cpos >> 2) & (DEC_RING - 1)) * 64;
  const u32 D0 = rp[0], D1 = rp[64];
  const u32 D2 = SM ? 0u : rp[128];
  const u64 r = range_par_total<DIV>(d.range, m);
  // hint q ~ x / r ~ x * total / range from the top 32 bits of x and range.  Direct tables
  // (total <= 2048) take the high halves as they are: range >= 2^48, so the relative error is
  // <= 2^-15 (and ~2^-24 for the usual range >= 2^56), far inside one frequency step.  Bucket
  // tables (totals up to 2^32) first shift both by clz(range), for a relative error ~2^-22.
  float X, R;
  if (LUT == 2) {
    X = cvt_f32(d.xhi);
    R = 1.0f;  // unused: the scale G is carried
  } else if (LUT) {
    X = cvt_f32(d.xhi);
    R = cvt_f32(hi32(d.range));
  } else {
    const u32 e = (u32)__builtin_clz(hi32(d.range));
    X = cvt_f32(hi32(d.x() << e));
    R = cvt_f32(hi32(d.range << e));
  }
  // The table index is masked, not clamped: the tables are padded to a power of two with valid
  // entries, so an out-of-range hint (corrupt streams, x >= range; or rounding to q == total)
  // only starts the exact fix-up below from another symbol, whose result does not depend on
  // where it starts.  (A v_mul_f32 clamp modifier was tried instead and gave wrong hints.)
  const float rR = LUT == 2 ? 1.0f : __builtin_amdgcn_rcpf(R);
  u32 s;
  uint2 t;
  float tc = 0.0f;  // LUT == 2: total / c of the coded symbol, as a float
  if (LUT == 2) {  // 16-B direct entries {cum, c, s, total/c}: one ds_read_b128, no unpacking
    // G = 16 total / (range / 2^32) is not recomputed per symbol: range' = r c 2^k, so
    // G' = G (total / c) 2^-k (one multiply, one ldexp instead of a convert and a reciprocal);
    // it is recomputed exactly at every phase and after any rare path
    const u32 q16 = cvt_u32_sat(X * d.G) & (m.lut_max << 4);
    const u32x4 ent = *(const __attribute__((address_space(3))) u32x4*)(uintptr_t)q16;
    s = ent.z;
    t = make_uint2(ent.x, ent.y);
    tc = __uint_as_float(ent.w);
  } else if (LUT) {  // direct table: candidate symbol and its (cum, c) in one LDS read at byte 4q
    // the LUT is the kernel's first LDS object (address 0): q4 is its LDS byte address
    const u32 q4 = cvt_u32_sat(X * ((4.0f * m.ftotal) * rR)) & (m.lut_max << 2);
    const u32 ent = *(const __attribute__((address_space(3))) u32*)(uintptr_t)q4;
    s = ent;  // the symbol is its low byte (callers take byte 0; dec_fix masks it)
    t = make_uint2((ent >> 8) & 0xFFFu, ent >> 20);
  } else {  // bucket table, then the (cum, c) table
    const u32 qh = cvt_u32_sat(X * (m.ftotal * rR));
    const u32 b = (qh >> m.lut_shift) & m.lut_max;
    const u32 ent = s_lut[b];
    s = ((qh - (b << m.lut_shift)) >= (ent >> 16)) ? ((ent >> 8) & 255u) : (ent & 255u);
    t = s_tab[s];
  }
  u64 A = mul_rv<SM>(r, t.x);
  u64 B = mul_rv<SM>(r, t.y);
  // exact verification r*cum[s] <= x < r*cum[s+1] as ONE unsigned test: A + B <= range < 2^64,
  // so when A > x the wrapped difference x - A is >= 2^64 - A > B.  The hint is rarely off.
  // (At s = n - 1 the test fails only on corrupt input, x >= r * total: dec_fix keeps s = n-1.)
  u64 dx = sub64(d.xlo, d.xhi, A);
  if (__builtin_expect(__any((int)(dx >= B)), 0)) {
    if (dx >= B) {
      dec_fix(s, t, A, B, d.x(), r, s_tab, m.n);
      if (LUT == 2) tc = m.ftotal * __builtin_amdgcn_rcpf(cvt_f32(t.y));
      // the tables only hold symbols with c > 0, so c == 0 can only come from dec_fix: corrupt
      // input (the reference loops forever); an over-read, if any, came first
      if (t.y == 0) {
        d.err = d.err ? d.err : (d.cpos > d.lim ? RC_F_TRUNCATED : RC_F_CORRUPT);
        B = r;
      }
      dx = sub64(d.xlo, d.xhi, A);
    }
  }
  // param_update (range_coder.rs:53-92)
  d.low += A;
  d.range = B;
  // closed-form no_carry_expansion; SM: range >= 2^32 here, so the high halves
  // differ and k8 <= 24
  const u32 k8 = SM ? (ffbh(hi32(d.low) ^ hi32(d.low + d.range)) & 24u)
                    : ((u32)__clzll(d.low ^ (d.low + d.range)) & 56u);
  d.low <<= k8;
  d.range <<= k8;
  if (LUT == 2) d.G = __builtin_amdgcn_ldexpf(d.G * tc, -(int)k8);
  // data' = data << k8 | k settled bytes and low' = (low + A) << k8, so x' = ((x - A) << k8) |
  // those bytes (shift_left_buffer, decoder.rs:31-35): the high half of dx << k8, and the high
  // half of (dx_lo : next 4 code bytes) << k8 (alignbyte uses cpos & 3 only)
  if (SM) {  // k8 = 8n <= 24
    // xl = dx_lo << 8n | the n code bytes at cpos, first byte highest: ONE v_perm_b32 over
    // {dx_lo, W} (W = the 4 code bytes at cpos, first byte in byte 0) whose selector is
    // hi32(0x0706050400010203 << 8n): byte j takes dx_lo byte j - n (j >= n) or W byte
    // n - 1 - j (j < n).  (No byte swap, no register pair to assemble.)
    const u32 W = __builtin_amdgcn_alignbyte(D1, D0, d.cpos);
    const u32 sel = hi32(0x0706050400010203ull << k8);
    const u32 xl = __builtin_amdgcn_perm((u32)dx, W, sel);
    d.xhi = hi32(dx << k8);
    d.xlo = xl;
  } else {   // k8 <= 56
    const u32 w0 = __builtin_bswap32(__builtin_amdgcn_alignbyte(D1, D0, d.cpos));
    const u64 b = ((u64)w0 << 32) | __builtin_bswap32(__builtin_amdgcn_alignbyte(D2, D1, d.cpos));
    d.set_x((dx << k8) | (k8 ? b >> (64 - k8) : 0ull));
  }
  u32 nbytes;  // k8 >> 3 as a plain shift (the compiler's v_bfe from the ffbh result costs more)
  asm("v_lshrrev_b32 %0, 3, %1" : "=v"(nbytes) : "v"(k8));
  d.cpos += nbytes;
  // rare: range_reduction_expansion, or (wide models) the ring runs short for the next symbol
  const bool rare = SM ? (hi32(d.range) < 0x10000u)
                       : ((hi32(d.range) < 0x10000u) | ((int)(d.fill - d.cpos) < (int)DEC_NEED_WIDE));
  if (__builtin_expect(__any((int)rare), 0)) {
    if (rare) {
      dec_rare(d, SM ? DEC_NEED_SM : DEC_NEED_WIDE);
      if (LUT == 2) dec_gexact(d, m);
    }
  }
  return s;
}

// SM models: the ring check for the next 4 symbols (wave-uniform call sites)
template <int SM>
static __device__ __forceinline__ void dec_check4(Dec& d) {
  if (!SM) return;
  const bool low = (int)(d.fill - d.cpos) < (int)DEC_NEED_SM;
  if (__builtin_expect(__any((int)low), 0)) {
    if (low) dec_sync(d, DEC_NEED_SM);
  }
}

// 16 symbols into one 16-B block (byte j of word q = symbol 4q + j), with the ring checks
template <int DIV, int SM, int LUT>
static __device__ __forceinline__ uint4 dec_phase16(Dec& d, const ModelArgs& m,
                                                    const uint2* s_tab, const u32* s_lut) {
  if (LUT == 2) dec_gexact(d, m);  // bounds the drift of the carried scale to 16 symbols
  u32 w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int j = 0; j < 4; ++j) w[q] = put_byte(w[q], dec_sym<DIV, SM, LUT>(d, m, s_tab, s_lut), j);
    if (q < 3) dec_check4<SM>(d);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int DIV, int SM, int LUT>
__global__ __launch_bounds__(WG) void k_decode_static(
    ModelArgs m, const uint8_t* __restrict__ code, const u64* __restrict__ code_off,
    const u64* __restrict__ code_len, uint8_t* __restrict__ syms_out,
    const u64* __restrict__ sym_off, u32 n_chunks, u32* __restrict__ flags) {
  // All LDS is dynamic, sized at launch (the WG's footprint sets how many WGs share a CU):
  // the LUT (lut_max + 1 entries) first, at LDS address 0, so a table read is a ds_read at the
  // hint's byte offset with no base add; then the (cum, c) table and the code rings.
  extern __shared__ u32 s_dyn[];
  u32* s_lut = s_dyn;
  const u32 lut_n = (m.lut_max + 1) * (LUT == 2 ? 4u : 1u);  // LUT words
  const u32 lut_words = (lut_n + 1) & ~1u;                    // 8-B aligned s_tab
  // (direct tables hold (cum, c) themselves; then only the rare exact fix-up reads the table)
  constexpr bool tab_lds = !LUT || DEC_TAB_LDS;
  const uint2* s_tab = tab_lds ? reinterpret_cast<const uint2*>(s_dyn + lut_words) : m.tab;
  const u32 tid = threadIdx.x;
  if (tab_lds) reinterpret_cast<uint2*>(s_dyn + lut_words)[tid] = m.tab[tid];
  for (u32 j = tid; j < lut_n; j += WG) s_lut[j] = m.lut[j];
  __syncthreads();
  const u32 k = blockIdx.x * WG + tid;
  if (k >= n_chunks) return;
  RC_VGPR_FLOOR_64();
  const u32 lane = tid & 63, wave = tid >> 6;

  const u64 c0 = code_off[k];
  const u64 clen = code_len[k];
  const u64 n = sym_off[k + 1] - sym_off[k];
  uint8_t* op = syms_out + sym_off[k];
  if (clen < 8) {  // Decoder::new panics (decoder.rs:21, :33)
    flags[k] = RC_F_TRUNCATED;
    return;
  }
  const uint8_t* cp = code + c0;
  const u32 a = (u32)((uintptr_t)cp & 15);

  Dec d;
  d.low = 0;
  d.range = ~0ull;
  d.err = 0;
  d.fill = 0;
  d.pend_ok = 0;
  // the ring as a plain LDS address (s_dyn is at 0), one register: no per-access base math
  d.ring = (l_u32*)(uintptr_t)((lut_words + (tab_lds ? 512 : 0)) * 4) +
           wave * DEC_RING_ALLOC * 64 + lane;
  d.gbase = reinterpret_cast<const uint4*>(cp - a);
  d.gnext = 0;
  d.glast = (u32)((a + clen - 1) >> 4);
  d.cpos = a + 8;  // Decoder::new primes 8 bytes (decoder.rs:21)
  d.lim = (u32)(clen < 0xFFFFFF00ull - a ? a + clen : 0xFFFFFF00ull);
  // fill the whole ring, and have the next load burst in flight
#pragma unroll
  for (int h = 0; h < DEC_RING / (4 * DEC_PF); ++h) {
    if (!d.pend_ok) dec_issue(d);
    dec_commit(d);
  }
  if (!d.pend_ok) dec_issue(d);
  d.set_x(dec_read8_before(d));  // data - low with low = 0
  if (LUT == 2) dec_gexact(d, m);

  u64 i = 0;
  // head: single symbols until the output is 64-B aligned
  constexpr u32 OUT_ALIGN = 16 * DEC_OUT_BURST;  // (symbols before the first aligned burst)
  u64 head = (OUT_ALIGN - ((uintptr_t)op & (OUT_ALIGN - 1))) & (OUT_ALIGN - 1);
  if (head > n) head = n;
  dec_check4<SM>(d);
  for (; i < head; ++i) {
    op[i] = (uint8_t)dec_sym<DIV, SM, LUT>(d, m, s_tab, s_lut);
    dec_check4<SM>(d);
  }
  // body: 16-symbol phases (after each: commit a refill, maybe issue the next load burst).
  // Decoded symbols leave in 64-B bursts per lane (4 phases, four back-to-back 16-B stores to
  // one 64-B segment): HBM sees whole 64-B writes, not 16-B partial ones.
  uint4* ob = reinterpret_cast<uint4*>(op + i);
  const u64 nbu = DEC_OUT_BURST > 1 ? (n - i) / (16 * DEC_OUT_BURST) : 0;
  for (u64 b = 0; b < nbu; ++b) {
    // written out: the compiler declines to unroll a 64-symbol loop and would then index the
    // blocks through scratch
#define RC_DEC_PHASE(o)                                          \
  const uint4 o = dec_phase16<DIV, SM, LUT>(d, m, s_tab, s_lut); \
  dec_phase(d);                                                  \
  dec_check4<SM>(d);
    RC_DEC_PHASE(o0) RC_DEC_PHASE(o1) RC_DEC_PHASE(o2) RC_DEC_PHASE(o3)
    uint4* ob_b = ob + DEC_OUT_BURST * b;
    if (DEC_OUT_BURST == 8) {
      RC_DEC_PHASE(o4) RC_DEC_PHASE(o5) RC_DEC_PHASE(o6) RC_DEC_PHASE(o7)
      ob_b[0] = o0; ob_b[1] = o1; ob_b[2] = o2; ob_b[3] = o3;
      ob_b[4] = o4; ob_b[5] = o5; ob_b[6] = o6; ob_b[7] = o7;
    } else {
      ob_b[0] = o0; ob_b[1] = o1; ob_b[2] = o2; ob_b[3] = o3;
    }
#undef RC_DEC_PHASE
  }
  i += nbu * 16 * DEC_OUT_BURST;
  ob += DEC_OUT_BURST * nbu;
  const u64 nph = (n - i) >> 4;
  for (u64 b = 0; b < nph; ++b) {
    ob[b] = dec_phase16<DIV, SM, LUT>(d, m, s_tab, s_lut);
    dec_phase(d);
    dec_check4<SM>(d);
  }
  i += nph << 4;
  for (; i < n; ++i) {
    op[i] = (uint8_t)dec_sym<DIV, SM, LUT>(d, m, s_tab, s_lut);
    dec_check4<SM>(d);
  }
  // shift_left_buffer panics once more bytes are needed than the stream holds (decoder.rs:33)
  if (!d.err && d.cpos > d.lim) d.err = RC_F_TRUNCATED;
  flags[k] = d.err;
}

// ------------------------------------------------------------------------------------------
// Synthetic workload generator (inputs for bench/tests, generated directly in HBM)
// ------------------------------------------------------------------------------------------
static __device__ __forceinline__ u64 mix64(u64 z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(WG) void k_synth(u64 seed, const uint8_t* __restrict__ inv,
                                             uint8_t* __restrict__ dst, u64 chunk_len,
                                             u64 total_words) {
  // one item = 16 symbols = 4 splitmix words; grid-stride (a launch is capped at 2^32 items)
  RC_VGPR_FLOOR_64();
  const u64 words_per_chunk = chunk_len >> 4;
  for (u64 g = (u64)blockIdx.x * WG + threadIdx.x; g < total_words; g += (u64)gridDim.x * WG) {
    const u64 chunk = g / words_per_chunk;
    const u64 w16 = g - chunk * words_per_chunk;
    u32 o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u64 word = mix64(seed + 0x9E3779B97F4A7C15ull * ((chunk << 32) + w16 * 4 + q + 1));
      o[q] = (u32)inv[word & 0xFFFF] | ((u32)inv[(word >> 16) & 0xFFFF] << 8) |
             ((u32)inv[(word >> 32) & 0xFFFF] << 16) | ((u32)inv[(word >> 48) & 0xFFFF] << 24);
    }
    reinterpret_cast<uint4*>(dst + chunk * chunk_len)[w16] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(WG) void k_synth_generic(u64 seed, const uint8_t* __restrict__ inv,
                                                     uint8_t* __restrict__ dst, u64 chunk_len,
                                                     u32 n_chunks) {
  // one thread per chunk, byte stores: any chunk_len / alignment (small test inputs)
  RC_VGPR_FLOOR_64();
  const u32 chunk = blockIdx.x * WG + threadIdx.x;
  if (chunk >= n_chunks) return;
  for (u64 i = 0; i < chunk_len; ++i) {
    const u64 word = mix64(seed + 0x9E3779B97F4A7C15ull * (((u64)chunk << 32) + i / 4 + 1));
    dst[(u64)chunk * chunk_len + i] = inv[(word >> (16 * (i & 3))) & 0xFFFF];
  }
}

// ------------------------------------------------------------------------------------------
// Host side: contexts, models, launches
// ------------------------------------------------------------------------------------------
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

struct rc_ctx {
  int device;
  hipStream_t own;
  hipStream_t cur;
  uint8_t* inv;  // 64 KiB device scratch for rc_synth_fill's inverse CDF
};

struct rc_model {
  int kind;  // 0 static, 1 adaptive
  int device;
  int div;
  ModelArgs args;
  void* dmem;
  AdaptParams ap;      // kind 1
  u32 c_host[256];     // kind 0: the c_freq snapshot (container tables, entropy reports)
  u32 period;          // kind 1: as given
  bool complete;       // kind 0: 256 symbols, every c_freq > 0 (no symbol the coder can reject)
};

namespace {

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int now = -1;
    if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
  }
};

u32 bitlen(u32 v) { return v ? 32u - (u32)__builtin_clz(v) : 0u; }

thread_local char g_last_error[256] = "";

rc_status device_error(hipError_t e, const char* what) {
  snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
  return RC_E_DEVICE;
}

rc_status launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? RC_OK : device_error(e, "kernel launch");
}

}  // namespace

extern "C" {

const char* rc_last_error(void) { return g_last_error; }

const char* rc_status_string(rc_status s) {
  switch (s) {
    case RC_OK: return "ok";
    case RC_E_ARG: return "invalid argument";
    case RC_E_BAD_MODEL: return "frequency table rejected";
    case RC_E_DEVICE: return "HIP runtime error";
    case RC_E_NO_DEVICE: return "no usable gfx950 device";
    case RC_E_CHUNK: return "at least one chunk flagged";
    case RC_E_BAD_CONTAINER: return "malformed container";
    case RC_E_CAPACITY: return "destination too small";
    default: return "unknown status";
  }
}

rc_status rc_device_info(int device, char* buf, size_t buf_len) {
  if (!buf || !buf_len) return RC_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RC_E_NO_DEVICE;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return RC_E_DEVICE;
  snprintf(buf, buf_len, "%s CUs=%d LDS/CU=%zu", p.gcnArchName, p.multiProcessorCount,
           (size_t)p.maxSharedMemoryPerMultiProcessor);
  return RC_OK;
}

rc_status rc_ctx_create(int device, rc_ctx** out) {
  if (!out) return RC_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RC_E_NO_DEVICE;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return RC_E_DEVICE;
  if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return RC_E_NO_DEVICE;
  DeviceGuard g(device);
  if (!g.ok) return RC_E_DEVICE;
  rc_ctx* c = new rc_ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return RC_E_DEVICE;
  }
  c->cur = c->own;
  if (hipMalloc((void**)&c->inv, 65536) != hipSuccess) {
    (void)hipStreamDestroy(c->own);
    delete c;
    return RC_E_DEVICE;
  }
  *out = c;
  return RC_OK;
}

void rc_stream_release_(const rc_ctx* ctx);  // rc_stream.hip: the cached host pipeline

rc_status rc_ctx_destroy(rc_ctx* ctx) {
  if (!ctx) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  rc_stream_release_(ctx);
  (void)hipStreamSynchronize(ctx->own);
  (void)hipStreamSynchronize(ctx->cur);
  (void)hipFree(ctx->inv);
  (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return RC_OK;
}

// internal (not in the header): the context's device and current stream, for the other
// translation units of the library
rc_status rc_ctx_stream_(rc_ctx* ctx, hipStream_t* s, int* device) {
  if (!ctx || !s || !device) return RC_E_ARG;
  *s = ctx->cur;
  *device = ctx->device;
  return RC_OK;
}

// internal: what the container writer needs to know about a model
rc_status rc_model_describe_(const rc_model* m, int* kind, int* device, uint32_t* n_symbols,
                             uint32_t* total, const uint32_t** c_host, uint32_t* increment,
                             uint32_t* limit, uint32_t* period) {
  if (!m) return RC_E_ARG;
  *kind = m->kind;
  *device = m->device;
  *n_symbols = m->kind == 0 ? m->args.n : m->ap.n;
  *total = m->args.total;
  *c_host = m->c_host;
  *increment = m->ap.inc;
  *limit = m->ap.limit;
  *period = m->period;
  return RC_OK;
}

rc_status rc_ctx_set_stream(rc_ctx* ctx, void* hip_stream) {
  if (!ctx) return RC_E_ARG;
  ctx->cur = (hipStream_t)hip_stream;
  return RC_OK;
}

rc_status rc_ctx_reset_stream(rc_ctx* ctx) {
  if (!ctx) return RC_E_ARG;
  ctx->cur = ctx->own;
  return RC_OK;
}

rc_status rc_ctx_synchronize(rc_ctx* ctx) {
  if (!ctx) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  return hipStreamSynchronize(ctx->cur) == hipSuccess ? RC_OK : RC_E_DEVICE;
}

rc_status rc_model_create_static(rc_ctx* ctx, uint32_t n_symbols, const uint32_t* c_freq,
                                 const uint32_t* cum_freq, uint32_t total_freq, rc_model** out) {
  if (!ctx || !c_freq || !cum_freq || !out) return RC_E_ARG;
  *out = nullptr;
  if (n_symbols < 1 || n_symbols > 256 || total_freq < 1) return RC_E_BAD_MODEL;
  u64 acc = 0;
  for (u32 i = 0; i < n_symbols; ++i) {
    if ((u64)cum_freq[i] != acc) return RC_E_BAD_MODEL;
    acc += c_freq[i];
  }
  if (acc != (u64)total_freq) return RC_E_BAD_MODEL;

  std::vector<uint2> tab(256);
  for (u32 i = 0; i < 256; ++i)
    tab[i] = i < n_symbols ? make_uint2(cum_freq[i], c_freq[i]) : make_uint2(0xFFFFFFFFu, 0u);

  ModelArgs a;
  memset(&a, 0, sizeof a);
  a.n = n_symbols;
  a.total = total_freq;
  a.ftotal = (float)total_freq;
  const bool pow2 = (total_freq & (total_freq - 1)) == 0;
  a.lg = pow2 ? (u32)__builtin_ctz(total_freq) : 0u;
  a.magic = ~0ull / (u64)total_freq;
  const u32 bl = bitlen(total_freq - 1);
  a.lut_shift = bl > LUT_BITS ? bl - LUT_BITS : 0u;
  a.lut_max = (total_freq - 1) >> a.lut_shift;
  // bucket table: s0 = symbol containing the bucket's first frequency, s1 = the next symbol
  // with c > 0 starting inside the bucket, split = its offset (0xFFFF: none)
  std::vector<u32> lut(a.lut_max + 1);
  u32 s = 0;
  for (u32 b = 0; b <= a.lut_max; ++b) {
    const u64 f0 = (u64)b << a.lut_shift;
    const u64 f1 = std::min<u64>((u64)(b + 1) << a.lut_shift, total_freq);
    while (s + 1 < n_symbols && (u64)cum_freq[s + 1] <= f0) ++s;
    u32 s1 = s, split = 0xFFFFu;
    for (u32 t = s + 1; t < n_symbols; ++t) {
      if ((u64)cum_freq[t] >= f1) break;
      if (c_freq[t] > 0) {
        if ((u64)cum_freq[t] - f0 <= 0xFFFFu) {
          s1 = t;
          split = (u32)((u64)cum_freq[t] - f0);
        }
        break;
      }
    }
    lut[b] = s | (s1 << 8) | (split << 16);
  }
  // pad to a power of two (the kernel masks the bucket index) with the last bucket
  while (lut.size() & (lut.size() - 1)) lut.push_back(lut.back());
  a.lut_max = (u32)lut.size() - 1;

  if (total_freq <= 2048) {  // direct table: q -> s | cum << 8 | c << 20
    a.direct = 1;
    a.lut_shift = 0;
    a.lut_max = total_freq - 1;
    lut.assign(total_freq, 0);
    u32 sym = 0;
    for (u32 q = 0; q < total_freq; ++q) {
      while (sym + 1 < n_symbols && cum_freq[sym + 1] <= q) ++sym;
      lut[q] = sym | (cum_freq[sym] << 8) | (c_freq[sym] << 20);
    }
    while (lut.size() & (lut.size() - 1)) lut.push_back(lut.back());  // pow2 (masked index)
    a.lut_max = (u32)lut.size() - 1;
    if (total_freq >= 256 && total_freq <= 512) {  // 16-B entries {cum, c, s, 0}
      a.direct = 2;
      std::vector<u32> wide(4 * lut.size());
      for (size_t q = 0; q < lut.size(); ++q) {
        const u32 sq = lut[q] & 255u;
        wide[4 * q + 0] = cum_freq[sq];
        wide[4 * q + 1] = c_freq[sq];
        wide[4 * q + 2] = sq;
        const float tcf = (float)total_freq / (float)c_freq[sq];
        memcpy(&wide[4 * q + 3], &tcf, sizeof tcf);
      }
      lut.swap(wide);
    }
  }
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const size_t tab_bytes = 256 * sizeof(uint2);
  const size_t lut_bytes = lut.size() * sizeof(u32);
  void* d = nullptr;
  if (hipMalloc(&d, tab_bytes + lut_bytes) != hipSuccess) return RC_E_DEVICE;
  if (hipMemcpy(d, tab.data(), tab_bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((char*)d + tab_bytes, lut.data(), lut_bytes, hipMemcpyHostToDevice) !=
          hipSuccess) {
    (void)hipFree(d);
    return RC_E_DEVICE;
  }
  a.tab = (const uint2*)d;
  a.lut = (const u32*)((char*)d + tab_bytes);
  rc_model* mm = new rc_model;
  mm->kind = 0;
  mm->device = ctx->device;
  mm->div = pow2 ? DIV_POW2 : DIV_MAGIC;
  mm->args = a;
  mm->dmem = d;
  mm->ap = AdaptParams{};
  memset(mm->c_host, 0, sizeof mm->c_host);
  for (u32 i = 0; i < n_symbols; ++i) mm->c_host[i] = c_freq[i];
  mm->complete = n_symbols == 256;
  for (u32 i = 0; i < n_symbols; ++i) mm->complete = mm->complete && c_freq[i] > 0;
  mm->period = 0;
  *out = mm;
  return RC_OK;
}

rc_status rc_model_create_adaptive(rc_ctx* ctx, uint32_t n_symbols, uint32_t increment,
                                   uint32_t limit, uint32_t period, rc_model** out) {
  if (!ctx || !out) return RC_E_ARG;
  *out = nullptr;
  const u64 grow = (u64)increment * period;  // total growth between two halving checks
  if (n_symbols < 1 || n_symbols > 256 || increment < 1 || period < 1 || period > 65536 ||
      (period & (period - 1)) != 0 || grow + n_symbols > limit || limit + grow > 65535)
    return RC_E_BAD_MODEL;
  rc_model* mm = new rc_model;
  memset(mm, 0, sizeof *mm);
  mm->kind = 1;
  mm->device = ctx->device;
  mm->ap = AdaptParams{n_symbols, increment, limit, period - 1};
  mm->period = period;
  *out = mm;
  return RC_OK;
}

rc_status rc_model_destroy(rc_model* m) {
  if (!m) return RC_E_ARG;
  DeviceGuard g(m->device);
  if (m->dmem) (void)hipFree(m->dmem);
  delete m;
  return RC_OK;
}

rc_status rc_encode_batch(rc_ctx* ctx, const rc_model* m, const uint8_t* syms,
                          const uint64_t* sym_off, uint32_t n_chunks, uint8_t* out,
                          const uint64_t* out_off, uint64_t* out_len, uint32_t* flags) {
  if (!ctx || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!syms || !sym_off || !out || !out_off || !out_len || !flags) return RC_E_ARG;
  if (m->device != ctx->device) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  if (m->kind == 1) {
    const hipError_t e = rc_adaptive_encode_launch(ctx->cur, m->ap, syms, sym_off, n_chunks,
                                                   out, out_off, out_len, flags);
    return e == hipSuccess ? RC_OK : device_error(e, "adaptive encode launch");
  }
  const dim3 grid((n_chunks + WG - 1) / WG), block(WG);
  const bool sm = m->args.total >= 256 && m->args.total <= 65536;
  const int smv = sm ? (m->complete ? 2 : 1) : 0;
#define RC_ENC_LAUNCH(D, S)                                                                \
  hipLaunchKernelGGL((k_encode_static<D, S>), grid, block, 0, ctx->cur, m->args, syms,    \
                     sym_off, n_chunks, out, out_off, out_len, flags)
#ifdef RC_DEV_ONLY  // scratch builds for kernel tuning: the headline variants only
  if (m->div != DIV_POW2 || !sm) return RC_E_ARG;
  if (smv == 2) RC_ENC_LAUNCH(DIV_POW2, 2); else RC_ENC_LAUNCH(DIV_POW2, 1);
#else
  if (m->div == DIV_POW2) {
    if (smv == 2) RC_ENC_LAUNCH(DIV_POW2, 2);
    else if (smv == 1) RC_ENC_LAUNCH(DIV_POW2, 1);
    else RC_ENC_LAUNCH(DIV_POW2, 0);
  } else {
    if (smv == 2) RC_ENC_LAUNCH(DIV_MAGIC, 2);
    else if (smv == 1) RC_ENC_LAUNCH(DIV_MAGIC, 1);
    else RC_ENC_LAUNCH(DIV_MAGIC, 0);
  }
#endif
#undef RC_ENC_LAUNCH
  return launch_status();
}

rc_status rc_decode_batch(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                          const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                          const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags) {
  if (!ctx || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!code || !code_off || !code_len || !syms_out || !sym_off || !flags) return RC_E_ARG;
  if (m->device != ctx->device) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  if (m->kind == 1) {
    const hipError_t e = rc_adaptive_decode_launch(ctx->cur, m->ap, code, code_off, code_len,
                                                   syms_out, sym_off, n_chunks, flags);
    return e == hipSuccess ? RC_OK : device_error(e, "adaptive decode launch");
  }
  const dim3 grid((n_chunks + WG - 1) / WG), block(WG);
  const bool sm = m->args.total >= 256 && m->args.total <= 65536;
#define RC_DEC_LAUNCH(D, S, L)                                                             \
  hipLaunchKernelGGL((k_decode_static<D, S, L>), grid, block, lut_bytes, ctx->cur, m->args, \
                     code, code_off, code_len, syms_out, sym_off, n_chunks, flags)
  const bool dl = m->args.direct != 0, dl2 = m->args.direct == 2;
  // dynamic LDS of k_decode_static: LUT (8-B aligned), the (cum, c) table, the code rings
  const size_t lut_n = ((size_t)m->args.lut_max + 1) * (dl2 ? 4 : 1);
  const size_t lut_bytes = ((lut_n + 1) & ~(size_t)1) * sizeof(u32) +
                           (!dl || DEC_TAB_LDS ? 256 * sizeof(uint2) : 0) +
                           WAVES * DEC_RING_ALLOC * 64 * sizeof(u32);
#ifdef RC_DEV_ONLY
  if (m->div != DIV_POW2 || !sm) return RC_E_ARG;
  if (dl2) RC_DEC_LAUNCH(DIV_POW2, 1, 2);
  else if (dl) RC_DEC_LAUNCH(DIV_POW2, 1, 1); else RC_DEC_LAUNCH(DIV_POW2, 1, 0);
#else
  // (direct == 2 implies sm)
  if (m->div == DIV_POW2) {
    if (dl2) RC_DEC_LAUNCH(DIV_POW2, 1, 2);
    else if (sm) { if (dl) RC_DEC_LAUNCH(DIV_POW2, 1, 1); else RC_DEC_LAUNCH(DIV_POW2, 1, 0); }
    else    { if (dl) RC_DEC_LAUNCH(DIV_POW2, 0, 1); else RC_DEC_LAUNCH(DIV_POW2, 0, 0); }
  } else {
    if (dl2) RC_DEC_LAUNCH(DIV_MAGIC, 1, 2);
    else if (sm) { if (dl) RC_DEC_LAUNCH(DIV_MAGIC, 1, 1); else RC_DEC_LAUNCH(DIV_MAGIC, 1, 0); }
    else    { if (dl) RC_DEC_LAUNCH(DIV_MAGIC, 0, 1); else RC_DEC_LAUNCH(DIV_MAGIC, 0, 0); }
  }
#endif
#undef RC_DEC_LAUNCH
  return launch_status();
}

// rc_encode_host / rc_decode_host: the pipelined host path lives in rc_stream.hip

rc_status rc_synth_fill(rc_ctx* ctx, uint64_t seed, const uint8_t* inv_cdf_host,
                        uint8_t* syms_dev, uint64_t chunk_len, uint32_t n_chunks) {
  if (!ctx || !inv_cdf_host || !syms_dev) return RC_E_ARG;
  if (n_chunks == 0 || chunk_len == 0) return RC_OK;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const uint8_t* dinv = ctx->inv;
  hipError_t e = hipMemcpyAsync(ctx->inv, inv_cdf_host, 65536, hipMemcpyHostToDevice, ctx->cur);
  if (e != hipSuccess) return device_error(e, "rc_synth_fill copy");
  if ((chunk_len & 15) == 0 && ((uintptr_t)syms_dev & 15) == 0) {
    const u64 words = (chunk_len >> 4) * (u64)n_chunks;
    const u64 blocks = std::min<u64>((words + WG - 1) / WG, 1u << 16);
    hipLaunchKernelGGL(k_synth, dim3((u32)blocks), dim3(WG), 0, ctx->cur, seed,
                       dinv, syms_dev, chunk_len, words);
  } else {
    hipLaunchKernelGGL(k_synth_generic, dim3((n_chunks + WG - 1) / WG), dim3(WG), 0, ctx->cur,
                       seed, dinv, syms_dev, chunk_len, n_chunks);
  }
  rc_status st = launch_status();
  // the host table may be freed once the call returns: wait for the copy
  if (st == RC_OK && (e = hipStreamSynchronize(ctx->cur)) != hipSuccess)
    return device_error(e, "rc_synth_fill sync");
  return st;
}

}  // extern "C"
