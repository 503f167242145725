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
// 255-node tree of u16 (32 KiB per wave).  Node 256 — the total — lives in a register.  The
// tree is interleaved by lane, so one node row is one conflict-free 128-B access:
//     node j (1..255) = the counts of symbols [j - lowbit(j), j).
// Read top-down, that is the left-subtree-sum tree over the 256 symbols:
//   * the encoder's (cum[s], c[s]) is a root-to-leaf walk of 8 independent loads;
//   * the decoder's FreqTable::find_index (sample_impl.rs:27-45) is the same walk, steered by
//     the target frequency (8 dependent loads); it also yields cum[s] and c[s];
//   * c[s] += inc adds inc to the nodes where the walk went left (packed ds_add_u32).
// Read as a Fenwick tree, it turns into counts and back in place for the halving.
// Node values stay below 2^16 because the total does: limit + inc * period <= 65535.
// range / total (range_coder.rs:38-40) uses a float64 reciprocal and an exact integer
// correction.  Symbols and code move through per-lane dword loads and stores; L2 merges each
// lane's partial lines.
#include "rc_common.h"

#define AWG 64                  // one wave per workgroup
#define TREE_BYTES (255 * 64 * 2)

// ~1/t to well under 2^-40 relative error: v_rcp_f64 plus one Newton step
static __device__ __forceinline__ double recip(u32 t) {
  const double d = (double)t;
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}

// range_par_total (range_coder.rs:38-40): floor(v / t) for 1 <= t < 2^16, exact.  Each
// quotient half is floor or floor - 1 from the float64 product, then corrected.
static __device__ __forceinline__ u64 div_total(u64 v, u32 t, double rt) {
  const u32 hi = hi32(v), lo = (u32)v;
  u32 qh = (u32)((double)hi * rt);
  u32 rh = hi - qh * t;
  const bool fh = rh >= t;
  qh += fh ? 1u : 0u;
  rh -= fh ? t : 0u;
  const double num = fma((double)rh, 4294967296.0, (double)lo);  // < 2^48: exact
  u32 ql = (u32)(num * rt);
  const u64 rl = (((u64)rh << 32) | lo) - (u64)ql * t;
  ql += rl >= t ? 1u : 0u;
  return ((u64)qh << 32) + ql;
}

// ---- the per-lane count tree: node j at t[(j - 1) * 64] ----

static __device__ __forceinline__ void tree_init(uint16_t* t, u32 n) {
  for (u32 j = 1; j < 256; ++j) {
    const u32 lo = j - (j & (0u - j));
    t[(j - 1) * 64] = (uint16_t)(n > lo ? min(n, j) - lo : 0u);
  }
}

// cum[s] and c[s]: the walk to leaf s goes right at level l iff bit 7-l of s is set
static __device__ __forceinline__ void tree_query(const uint16_t* t, u32 s, u32 total, u32& cum,
                                                  u32& c) {
  u32 v[8];
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const u32 step = 128u >> l;
    v[l] = t[(((s & ~(2 * step - 1)) | step) - 1) * 64];
  }
  u32 a = 0, b = total;
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const bool right = (s & (128u >> l)) != 0;
    a += right ? v[l] : 0u;
    b = right ? b - v[l] : v[l];
  }
  cum = a;
  c = b;
}

// FreqTable::find_index for q < total: the s with cum[s] <= q < cum[s] + c[s]
static __device__ __forceinline__ u32 tree_find(const uint16_t* t, u32 q, u32 total, u32& cum,
                                                u32& c) {
  u32 pos = 0, rem = q, b = total;
#pragma unroll
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

// c[s] += inc: every node whose left subtree holds s.  tw: this lane's dword column (the
// lane pair's u16s share a dword; incv = inc in this lane's half, no carry: nodes < 2^16)
static __device__ __forceinline__ void tree_add(u32* tw, u32 s, u32 incv) {
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const u32 step = 128u >> l;
    // unconditional (adding 0 where the walk went right): no exec-mask branch per level
    atomicAdd(&tw[(((s & ~(2 * step - 1)) | step) - 1) * 32], (s & step) ? 0u : incv);
  }
}

// every c = (c + 1) >> 1: Fenwick -> counts (reverse pass), halve, counts -> Fenwick
static __device__ void tree_halve(uint16_t* t, u32& total) {
  for (u32 j = 255; j >= 1; --j) {
    const u32 k = j + (j & (0u - j));
    if (k < 256) t[(k - 1) * 64] = (uint16_t)(t[(k - 1) * 64] - t[(j - 1) * 64]);
  }
  u32 sum = 0, nt = 0;
  for (u32 j = 1; j < 256; ++j) {
    const u32 v = t[(j - 1) * 64];
    sum += v;
    nt += (v + 1) >> 1;
    t[(j - 1) * 64] = (uint16_t)((v + 1) >> 1);
  }
  nt += (total - sum + 1) >> 1;  // c[255] lives only in the total
  for (u32 j = 1; j < 256; ++j) {
    const u32 k = j + (j & (0u - j));
    if (k < 256) t[(k - 1) * 64] = (uint16_t)(t[(k - 1) * 64] + t[(j - 1) * 64]);
  }
  total = nt;
}

// ------------------------------------------------------------------------------------------
// I/O.  Memory traffic happens only at phase boundaries (every 16 symbols, at the same symbol
// index in every lane): first the block loaded one boundary earlier is consumed (the only
// wait), then this phase's stores are issued, then the next load.  So no wait ever covers a
// recent memory operation.  A conditional per-lane prefetch does not achieve this: the value
// merge at the branch join makes the compiler wait for the load right after issuing it.
// ------------------------------------------------------------------------------------------

__device__ u32x4 g_zero16;  // load target of lanes without input (never written)


// 4 bytes at byte offset (dsh * 4 + bsh) of the 8-dword window v: v[dsh], v[dsh + 1] funnel
static __device__ __forceinline__ u32 pick4(const u32 (&v)[8], u32 k, u32 dsh, u32 bsh) {
  // v[dsh + k] and v[dsh + k + 1] for a per-lane dsh in 0..3
  u32 a = v[k], b = v[k + 1];
  a = dsh == 1 ? v[k + 1] : a;
  b = dsh == 1 ? v[k + 2] : b;
  a = dsh == 2 ? v[k + 2] : a;
  b = dsh == 2 ? v[k + 3] : b;
  a = dsh == 3 ? v[k + 3] : a;
  b = dsh == 3 ? v[k + 4] : b;
  return __builtin_amdgcn_alignbyte(b, a, bsh);
}

// ------------------------------------------------------------------------------------------
// Encoder
// ------------------------------------------------------------------------------------------

// A settled dword (stream order, first byte in the top bits) at dp, clipped to [lo, hi).  dp
// is 4-B aligned because the stream starts with (slot address & 3) phantom bytes.
static __device__ __forceinline__ void put_dword(uint8_t*& dp, u32 be, const uint8_t* lo,
                                                 const uint8_t* hi) {
  const u32 d = __builtin_bswap32(be);
  if (dp >= lo && dp + 4 <= hi) {
    gstore32(dp, d);
  } else {
    for (u32 j = 0; j < 4; ++j)
      if (dp + j >= lo && dp + j < hi) gstore8(dp + j, d >> (8 * j));
  }
  dp += 4;
}

struct AEnc {
  u64 low, range, acc, len;
  u32 nbits;
  u32 q0, q1, q2, q3, qn;  // settled dwords waiting for the phase boundary
  uint8_t* dp;             // where q0 goes
};

static __device__ __forceinline__ void aenc_flush(AEnc& e, const uint8_t* lo,
                                                  const uint8_t* hi) {
  if (e.qn > 0) put_dword(e.dp, e.q0, lo, hi);
  if (e.qn > 1) put_dword(e.dp, e.q1, lo, hi);
  if (e.qn > 2) put_dword(e.dp, e.q2, lo, hi);
  if (e.qn > 3) put_dword(e.dp, e.q3, lo, hi);
  e.qn = 0;
}

static __device__ __forceinline__ void aenc_push(AEnc& e, u32 be, const uint8_t* lo,
                                                 const uint8_t* hi) {
  if (e.qn == 4) aenc_flush(e, lo, hi);  // more than 16 B settled within one phase (rare)
  e.q0 = e.qn == 0 ? be : e.q0;
  e.q1 = e.qn == 1 ? be : e.q1;
  e.q2 = e.qn == 2 ? be : e.q2;
  e.q3 = e.qn == 3 ? be : e.q3;
  e.qn += 1;
}

static __device__ __forceinline__ void aenc_byte(AEnc& e, u32 b, const uint8_t* lo,
                                                 const uint8_t* hi) {
  e.acc = (e.acc << 8) | b;
  e.nbits += 8;
  e.len += 1;
  if (e.nbits >= 32) {
    e.nbits -= 32;
    aenc_push(e, (u32)(e.acc >> e.nbits), lo, hi);
  }
}

__global__ __launch_bounds__(AWG) void k_encode_adaptive(
    AdaptParams p, const uint8_t* __restrict__ syms, const u64* __restrict__ sym_off,
    u32 n_chunks, uint8_t* __restrict__ out, const u64* __restrict__ out_off,
    u64* __restrict__ out_len, u32* __restrict__ flags) {
  extern __shared__ uint16_t s_tree[];
  const u32 lane = threadIdx.x;
  const u32 k = blockIdx.x * AWG + lane;
  const bool live = k < n_chunks;
  RC_VGPR_FLOOR_64();
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
  const uint8_t* hi = lo + cap;
  uint16_t* t = s_tree + lane;
  u32* tw = (u32*)(s_tree + (lane & ~1u));
  const u32 incv = p.inc << (16 * (lane & 1));
  tree_init(t, p.n);
  u32 total = p.n, err = 0;

  AEnc e;
  e.low = 0;
  e.range = ~0ull;  // RangeCoder::default (range_coder.rs:13-20)
  e.acc = 0;
  e.len = 0;
  e.nbits = 8 * (u32)((uintptr_t)lo & 3);
  e.q0 = e.q1 = e.q2 = e.q3 = e.qn = 0;
  e.dp = (uint8_t*)((uintptr_t)lo & ~(uintptr_t)3);

  // input window: 16-B blocks cur, nxt (landed) and pend (in flight); a phase's 16 symbols
  // start at byte (sp & 15) of cur
  const bool has = live && n > 0;
  const u32x4* bp = has ? (const u32x4*)((uintptr_t)sp & ~(uintptr_t)15) : &g_zero16;
  const u32x4* blast = has ? (const u32x4*)((uintptr_t)(sp + n - 1) & ~(uintptr_t)15) : bp;
  const u32 dsh = ((u32)(uintptr_t)sp >> 2) & 3u, bsh = (u32)(uintptr_t)sp & 3u;
  u32x4 cur = gload16(bp);
  bp = bp < blast ? bp + 1 : blast;
  u32x4 nxt = gload16(bp);
  bp = bp < blast ? bp + 1 : blast;
  u32x4 pend = gload16(bp);

  for (u64 i0 = 0;; i0 += 16) {
    if (!__any((int)(live && i0 < n && err == 0))) break;  // wave-uniform exit
    // this phase's 16 symbols, then the boundary I/O: rotate (waits for pend), store, load
    u32 sw[4];
    {
      const u32 v[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
#pragma unroll
      for (u32 q = 0; q < 4; ++q) sw[q] = pick4(v, q, dsh, bsh);
    }
    cur = nxt;
    nxt = pend;
    aenc_flush(e, lo, hi);
    bp = bp < blast ? bp + 1 : blast;
    pend = gload16(bp);

    for (u32 q = 0; q < 4; ++q) {
      u32 w = sw[0];
      w = q == 1 ? sw[1] : w;
      w = q == 2 ? sw[2] : w;
      w = q == 3 ? sw[3] : w;
#pragma unroll
      for (u32 jj = 0; jj < 4; ++jj) {
        const u64 i = i0 + 4 * q + jj;
        const bool act = live && i < n && err == 0;
        bool rare = false;
        if (act) {
          const u32 sym = (w >> (8 * jj)) & 255u;
          if (sym >= p.n) {
            err = RC_F_BAD_SYMBOL;  // the reference panics (sample_impl.rs:19)
          } else {
            u32 cum, c;
            tree_query(t, sym, total, cum, c);
            const u64 r = div_total(e.range, total, recip(total));
            e.range = r * c;   // range_coder.rs:65
            e.low += r * cum;  // :68-81 (no overflow: r * total <= range)
            // no_carry_expansion in closed form; range >= 2^32 here, so <= 3 bytes settle
            const u32 x = hi32(e.low) ^ hi32(e.low + e.range);
            const u32 nb = (u32)__builtin_clz(x) & 24u;
            e.acc = (e.acc << nb) | (u32)(((u64)hi32(e.low) << nb) >> 32);
            e.low <<= nb;
            e.range <<= nb;
            e.nbits += nb;
            e.len += nb >> 3;
            if (e.nbits >= 32) {
              e.nbits -= 32;
              aenc_push(e, (u32)(e.acc >> e.nbits), lo, hi);
            }
            rare = hi32(e.range) < 0x10000u;
            tree_add(tw, sym, incv);
            total += p.inc;
          }
        }
        if (__builtin_expect(__any((int)rare), 0)) {
          if (rare) {
            while (e.range < TOP16) {  // range_reduction_expansion (range_coder.rs:126-135)
              e.range = ~e.low & (TOP16 - 1);
              aenc_byte(e, (u32)(e.low >> 56), lo, hi);
              e.low <<= 8;
              e.range <<= 8;
            }
          }
        }
        if (((u32)i & p.pmask) == p.pmask) {  // wave-uniform: the period's halving check
          const bool h = act && err == 0 && total > p.limit;
          if (__any((int)h)) {
            if (h) tree_halve(t, total);
          }
        }
      }
    }
  }

  if (live) {
    if (err == 0) {
      for (u32 j = 0; j < 8; ++j) {  // Encoder::finish (encoder.rs:40-46): 8 x left_shift
        aenc_byte(e, (u32)(e.low >> 56), lo, hi);
        e.low <<= 8;
      }
      aenc_flush(e, lo, hi);
      for (u32 m = 0; m < e.nbits / 8; ++m) {  // the last partial dword
        uint8_t* a = e.dp + m;
        if (a >= lo && a < hi) gstore8(a, (u32)(e.acc >> (e.nbits - 8 * (m + 1))));
      }
      err = e.len > cap ? RC_F_CAPACITY : 0u;
    }
    out_len[k] = e.len;
    flags[k] = err;
  }
}

// ------------------------------------------------------------------------------------------
// Decoder
// ------------------------------------------------------------------------------------------

// The code of one lane: r[0..fill) are stream dwords (memory order), byte cpos at offset off
// of r[0]; pend is the 16-B block after them, loaded one phase ahead.
struct Win {
  u32 r[8];
  u32 off, fill;
  u32x4 pend;
  const u32x4* pnx;    // address of pend
  const u32x4* plast;  // last 16-B block holding a code byte
};

// the next kb (0..4) code bytes, big-endian (Decoder::shift_left_buffer, decoder.rs:31-35);
// needs fill >= 2
static __device__ __forceinline__ u32 win_take(Win& w, u32 kb) {
  const u32 v = __builtin_bswap32(__builtin_amdgcn_alignbyte(w.r[1], w.r[0], w.off));
  const u32 res = kb ? v >> (32 - 8 * kb) : 0u;
  w.off += kb;
  const bool sh = w.off >= 4;
#pragma unroll
  for (int i = 0; i < 7; ++i) w.r[i] = sh ? w.r[i + 1] : w.r[i];
  w.off -= sh ? 4u : 0u;
  w.fill -= sh ? 1u : 0u;
  return res;
}

// r[fill .. fill + 4) = pend (fill <= 4), and advance to the next block
static __device__ __forceinline__ void win_append(Win& w) {
  const u32 pv[4] = {w.pend.x, w.pend.y, w.pend.z, w.pend.w};
#pragma unroll
  for (u32 i = 0; i < 8; ++i) {
    const u32 d = i - w.fill;  // wraps for i < fill
    u32 v = pv[0];
    v = d == 1 ? pv[1] : v;
    v = d == 2 ? pv[2] : v;
    v = d == 3 ? pv[3] : v;
    w.r[i] = d < 4 ? v : w.r[i];
  }
  w.fill += 4;
  w.pnx = w.pnx < w.plast ? w.pnx + 1 : w.plast;
}

// the ~x * total / range hint (relative error ~2^-21): both shifted by clz(range)
static __device__ __forceinline__ u32 freq_hint(u64 x, u64 range, u32 total) {
  const u32 sh = (u32)__builtin_clz(hi32(range));
  const float X = (float)hi32(x << sh), R = (float)hi32(range << sh);
  return (u32)fminf(X * ((float)total * __builtin_amdgcn_rcpf(R)), 4.0e9f);
}

struct ADec {
  u64 low, range, data, used;
  u32 total, err;
};

// Decoder::decode (decoder.rs:38-54) with FreqTable::find_index (sample_impl.rs:27-45) and
// the model update; returns the symbol.  Wave-uniform call sites only (rare branches).
static __device__ __forceinline__ u32 adec_sym(ADec& d, Win& w, bool act, const uint16_t* t,
                                               u32* tw, u32 incv, const AdaptParams& p,
                                               u64 clen) {
  if (__builtin_expect(__any((int)(act && w.fill < 2)), 0)) {  // the window ran short (rare)
    if (act && w.fill < 2) {
      win_append(w);
      w.pend = gload16(w.pnx);
    }
  }
  bool rare = false, bad = false;
  u32 sym = 0, cum = 0, c = 0;
  u64 r = 0, x = 0;
  if (act) {
    x = d.data - d.low;
    // walk from the hint while the exact division runs; the interval check decides
    sym = tree_find(t, min(freq_hint(x, d.range, d.total), d.total - 1), d.total, cum, c);
    r = div_total(d.range, d.total, recip(d.total));
    const u64 a = r * cum;
    bad = a > x || x - a >= r * c;  // (for x >= r * total the answer is n - 1: exact path)
  }
  if (__builtin_expect(__any((int)bad), 0)) {
    if (bad) {  // exact rfreq = min(x / r, total - 1), then the walk
      u32 q = d.total - 1;
      if (x < r * d.total) {
        q = min(freq_hint(x, d.range, d.total), d.total - 1);
        u64 a = r * q;
        while (a > x) {
          --q;
          a -= r;
        }
        while (x - a >= r) {
          ++q;
          a += r;
        }
      }
      sym = tree_find(t, q, d.total, cum, c);
    }
  }
  if (act) {
    d.low += r * cum;
    d.range = r * c;
    const u32 kb = (u32)__clzll(d.low ^ (d.low + d.range)) >> 3;  // <= 3: range >= 2^32
    d.low <<= 8 * kb;
    d.range <<= 8 * kb;
    d.data = kb ? (d.data << (8 * kb)) | win_take(w, kb) : d.data;
    d.used += kb;
    rare = d.range < TOP16;
  }
  if (__builtin_expect(__any((int)rare), 0)) {
    if (rare) {
      while (d.range < TOP16) {  // range_reduction_expansion (range_coder.rs:126-135)
        d.range = ~d.low & (TOP16 - 1);
        d.low <<= 8;
        d.range <<= 8;
        if (w.fill < 2) {
          win_append(w);
          w.pend = gload16(w.pnx);
        }
        d.data = (d.data << 8) | win_take(w, 1);
        d.used += 1;
      }
    }
  }
  if (act) {
    if (d.used > clen) {
      d.err = RC_F_TRUNCATED;  // shift_left_buffer's pop_front panics (decoder.rs:33)
    } else {
      tree_add(tw, sym, incv);
      d.total += p.inc;
    }
  }
  return sym;
}

__global__ __launch_bounds__(AWG) void k_decode_adaptive(
    AdaptParams p, const uint8_t* __restrict__ code, const u64* __restrict__ code_off,
    const u64* __restrict__ code_len, uint8_t* __restrict__ syms_out,
    const u64* __restrict__ sym_off, u32 n_chunks, u32* __restrict__ flags) {
  extern __shared__ uint16_t s_tree[];
  const u32 lane = threadIdx.x;
  const u32 k = blockIdx.x * AWG + lane;
  const bool live = k < n_chunks;
  RC_VGPR_FLOOR_112();
  u64 n = 0, clen = 0;
  const uint8_t* cp = code;
  uint8_t* op = syms_out;
  if (live) {
    cp = code + code_off[k];
    clen = code_len[k];
    const u64 a = sym_off[k];
    n = sym_off[k + 1] - a;
    op = syms_out + a;
  }
  ADec d;
  d.err = live && clen < 8 ? RC_F_TRUNCATED : 0u;  // Decoder::new panics (decoder.rs:21)
  uint16_t* t = s_tree + lane;
  u32* tw = (u32*)(s_tree + (lane & ~1u));
  const u32 incv = p.inc << (16 * (lane & 1));
  tree_init(t, p.n);
  d.total = p.n;
  d.low = 0;
  d.range = ~0ull;
  d.data = 0;
  d.used = 8;

  // code window: the first two 16-B blocks, from the dword holding the first byte
  const bool has = live && d.err == 0;
  Win w;
  const u32x4* b0 = has ? (const u32x4*)((uintptr_t)cp & ~(uintptr_t)15) : &g_zero16;
  w.plast = has ? (const u32x4*)((uintptr_t)(cp + clen - 1) & ~(uintptr_t)15) : b0;
  {
    const u32x4 B0 = gload16(b0);
    const u32x4 B1 = gload16(b0 < w.plast ? b0 + 1 : w.plast);
    const u32 sh = ((u32)(uintptr_t)cp >> 2) & 3u;
    // r = (B0, B1) shifted down by sh dwords: a barrel shifter (by 1, then by 2)
    const bool s1 = (sh & 1u) != 0, s2 = (sh & 2u) != 0;
    const u32 a0 = s1 ? B0.y : B0.x, a1 = s1 ? B0.z : B0.y, a2 = s1 ? B0.w : B0.z;
    const u32 a3 = s1 ? B1.x : B0.w, a4 = s1 ? B1.y : B1.x, a5 = s1 ? B1.z : B1.y;
    const u32 a6 = s1 ? B1.w : B1.z, a7 = s1 ? 0u : B1.w;
    w.r[0] = s2 ? a2 : a0;
    w.r[1] = s2 ? a3 : a1;
    w.r[2] = s2 ? a4 : a2;
    w.r[3] = s2 ? a5 : a3;
    w.r[4] = s2 ? a6 : a4;
    w.r[5] = s2 ? a7 : a5;
    w.r[6] = s2 ? 0u : a6;
    w.r[7] = s2 ? 0u : a7;
    w.fill = 8 - sh;
    w.off = (u32)(uintptr_t)cp & 3u;
    w.pnx = b0 + 2 <= w.plast ? b0 + 2 : w.plast;
    w.pend = gload16(w.pnx);
    const u32 d0 = win_take(w, 4);
    d.data = ((u64)d0 << 32) | win_take(w, 4);
  }

  // output: head bytes until op is 8-B aligned, 8-symbol phases, then the tail bytes.  (A
  // phase of 8 keeps the 8-dword window fed without the short-window path up to ~1.5 B per
  // symbol: an append needs fill <= 4, and a phase then consumes at most 3 dwords.)
  const u64 head = min((u64)((8 - ((uintptr_t)op & 7)) & 7), n);
  u64 i = 0;
  for (; __any((int)(live && i < head && d.err == 0)); ++i) {
    const bool act = live && i < head && d.err == 0;
    const u32 sym = adec_sym(d, w, act, t, tw, incv, p, clen);
    if (act && d.err == 0) gstore8(op + i, sym);
    const bool h = act && d.err == 0 && ((u32)i & p.pmask) == p.pmask && d.total > p.limit;
    if (__any((int)h)) {
      if (h) tree_halve(t, d.total);
    }
  }
  i = head;  // every lane, at its own symbol index from here on
  while (__any((int)(live && i + 8 <= n && d.err == 0))) {
    const bool lact = live && i + 8 <= n && d.err == 0;
    u32 o0 = 0, o1 = 0;
    u32 nv = 0;  // symbols decoded in this phase before any error
    for (u32 q = 0; q < 2; ++q) {
      u32 wd = 0;
#pragma unroll
      for (u32 jj = 0; jj < 4; ++jj) {
        const u64 ii = i + 4 * q + jj;
        const bool act = lact && d.err == 0;
        wd |= adec_sym(d, w, act, t, tw, incv, p, clen) << (8 * jj);
        const bool ok = act && d.err == 0;
        nv += ok ? 1u : 0u;
        const bool h = ok && ((u32)ii & p.pmask) == p.pmask && d.total > p.limit;
        if (__any((int)h)) {
          if (h) tree_halve(t, d.total);
        }
      }
      o0 = q == 0 ? wd : o0;
      o1 = q == 1 ? wd : o1;
    }
    // boundary: consume pend (the only wait), store the block, load the next one
    if (lact && w.fill <= 4) win_append(w);
    if (lact && nv == 8) {
      *(__attribute__((address_space(1))) u64*)(op + i) = ((u64)o1 << 32) | o0;
    } else if (lact) {  // truncated inside the phase: the symbols before the error
      for (u32 j = 0; j < nv; ++j) gstore8(op + i + j, (j < 4 ? o0 : o1) >> (8 * (j & 3)));
    }
    w.pend = gload16(w.pnx);
    i += lact ? 8u : 0u;
  }
  for (; __any((int)(live && i < n && d.err == 0)); ++i) {  // tail
    const bool act = live && i < n && d.err == 0;
    const u32 sym = adec_sym(d, w, act, t, tw, incv, p, clen);
    if (act && d.err == 0) gstore8(op + i, sym);
    const bool h = act && d.err == 0 && ((u32)i & p.pmask) == p.pmask && d.total > p.limit;
    if (__any((int)h)) {
      if (h) tree_halve(t, d.total);
    }
  }
  if (live) flags[k] = d.err;
}

hipError_t rc_adaptive_encode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* syms, const u64* sym_off, u32 n_chunks,
                                     uint8_t* out, const u64* out_off, u64* out_len,
                                     u32* flags) {
  hipLaunchKernelGGL(k_encode_adaptive, dim3((n_chunks + AWG - 1) / AWG), dim3(AWG),
                     TREE_BYTES, stream, p, syms, sym_off, n_chunks, out, out_off, out_len,
                     flags);
  return hipGetLastError();
}

hipError_t rc_adaptive_decode_launch(hipStream_t stream, const AdaptParams& p,
                                     const uint8_t* code, const u64* code_off,
                                     const u64* code_len, uint8_t* syms_out, const u64* sym_off,
                                     u32 n_chunks, u32* flags) {
  hipLaunchKernelGGL(k_decode_adaptive, dim3((n_chunks + AWG - 1) / AWG), dim3(AWG),
                     TREE_BYTES, stream, p, code, code_off, code_len, syms_out, sym_off,
                     n_chunks, flags);
  return hipGetLastError();
}
