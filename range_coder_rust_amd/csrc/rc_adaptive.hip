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
    if ((s & step) == 0) atomicAdd(&tw[(((s & ~(2 * step - 1)) | step) - 1) * 32], incv);
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
// Encoder
// ------------------------------------------------------------------------------------------

// A settled dword (stream order, first byte in the top bits) at dp, clipped to [lo, hi): dp is
// 4-B aligned because the stream starts with (slot address & 3) phantom bytes.
static __device__ __forceinline__ void put_dword(uint8_t*& dp, u32 be, const uint8_t* lo,
                                                 const uint8_t* hi) {
  const u32 d = __builtin_bswap32(be);
  if (dp >= lo && dp + 4 <= hi) {
    *(u32*)dp = d;
  } else {
    for (u32 j = 0; j < 4; ++j)
      if (dp + j >= lo && dp + j < hi) dp[j] = (uint8_t)(d >> (8 * j));
  }
  dp += 4;
}

struct AEnc {
  u64 low, range, acc, len;
  u32 nbits;
  uint8_t* dp;
};

static __device__ __forceinline__ void aenc_byte(AEnc& e, u32 b, const uint8_t* lo,
                                                 const uint8_t* hi) {
  e.acc = (e.acc << 8) | b;
  e.nbits += 8;
  e.len += 1;
  if (e.nbits >= 32) {
    e.nbits -= 32;
    put_dword(e.dp, (u32)(e.acc >> e.nbits), lo, hi);
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
  e.dp = (uint8_t*)((uintptr_t)lo & ~(uintptr_t)3);

  // symbols: the dword holding symbol i, the next one, and a load in flight
  const u32* ip = (const u32*)((uintptr_t)sp & ~(uintptr_t)3);
  const u32* ilast = (const u32*)((uintptr_t)(sp + (n ? n - 1 : 0)) & ~(uintptr_t)3);
  const u32 b0 = (u32)((uintptr_t)sp & 3);
  u32 w0 = 0, w1 = 0;
  if (live && n) {
    w0 = ip[0];
    w1 = ip + 1 <= ilast ? ip[1] : 0u;
    ip = ip + 2 <= ilast ? ip + 2 : ilast;
  }

  for (u64 i = 0;; ++i) {
    const bool act = live && i < n && err == 0;
    if (!__any((int)act)) break;  // wave-uniform exit
    bool rare = false;
    if (act) {
      const u32 bpos = (b0 + (u32)i) & 3u;
      const u32 sym = (w0 >> (8 * bpos)) & 255u;
      if (bpos == 3u) {
        w0 = w1;
        w1 = *ip;
        ip = ip < ilast ? ip + 1 : ilast;
      }
      if (sym >= p.n) {
        err = RC_F_BAD_SYMBOL;  // the reference panics (sample_impl.rs:19)
      } else {
        u32 cum, c;
        tree_query(t, sym, total, cum, c);
        const u64 r = div_total(e.range, total, recip(total));
        e.range = r * c;    // range_coder.rs:65
        e.low += r * cum;   // :68-81 (no overflow: r * total <= range)
        // no_carry_expansion in closed form; range >= 2^32 here, so at most 3 bytes settle
        const u32 x = hi32(e.low) ^ hi32(e.low + e.range);
        const u32 nb = (u32)__builtin_clz(x) & 24u;
        e.acc = (e.acc << nb) | (u32)(((u64)hi32(e.low) << nb) >> 32);
        e.low <<= nb;
        e.range <<= nb;
        e.nbits += nb;
        e.len += nb >> 3;
        if (e.nbits >= 32) {
          e.nbits -= 32;
          put_dword(e.dp, (u32)(e.acc >> e.nbits), lo, hi);
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

  if (live) {
    if (err == 0) {
      for (u32 j = 0; j < 8; ++j) {  // Encoder::finish (encoder.rs:40-46): 8 x left_shift
        aenc_byte(e, (u32)(e.low >> 56), lo, hi);
        e.low <<= 8;
      }
      for (u32 m = 0; m < e.nbits / 8; ++m) {  // the last partial dword
        uint8_t* a = e.dp + m;
        if (a >= lo && a < hi) *a = (uint8_t)(e.acc >> (e.nbits - 8 * (m + 1)));
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

// The code stream of one lane: the dword holding byte cpos, the next one, one load in flight.
struct ACode {
  u32 c0, c1, c2, off;  // off: byte offset of cpos in c0
  const u32* nx;        // next dword to load
  const u32* last;      // last dword holding a code byte (loads are clamped to it)
};

static __device__ __forceinline__ void acode_rotate(ACode& s) {
  s.c0 = s.c1;
  s.c1 = s.c2;
  s.c2 = *s.nx;
  s.nx = s.nx < s.last ? s.nx + 1 : s.last;
}

// the next kb (0..4) code bytes, big-endian (Decoder::shift_left_buffer, decoder.rs:31-35)
static __device__ __forceinline__ u32 acode_take(ACode& s, u32 kb) {
  const u32 w = __builtin_bswap32(__builtin_amdgcn_alignbyte(s.c1, s.c0, s.off));
  const u32 v = kb ? w >> (32 - 8 * kb) : 0u;
  s.off += kb;
  if (s.off >= 4) {
    s.off -= 4;
    acode_rotate(s);
  }
  return v;
}

// the ~x * total / range hint (relative error ~2^-21): both shifted by clz(range)
static __device__ __forceinline__ u32 freq_hint(u64 x, u64 range, u32 total) {
  const u32 sh = (u32)__builtin_clz(hi32(range));
  const float X = (float)hi32(x << sh), R = (float)hi32(range << sh);
  return (u32)fminf(X * ((float)total * __builtin_amdgcn_rcpf(R)), 4.0e9f);
}

__global__ __launch_bounds__(AWG) void k_decode_adaptive(
    AdaptParams p, const uint8_t* __restrict__ code, const u64* __restrict__ code_off,
    const u64* __restrict__ code_len, uint8_t* __restrict__ syms_out,
    const u64* __restrict__ sym_off, u32 n_chunks, u32* __restrict__ flags) {
  extern __shared__ uint16_t s_tree[];
  const u32 lane = threadIdx.x;
  const u32 k = blockIdx.x * AWG + lane;
  const bool live = k < n_chunks;
  RC_VGPR_FLOOR_64();
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
  u32 err = live && clen < 8 ? RC_F_TRUNCATED : 0u;  // Decoder::new panics (decoder.rs:21)
  uint16_t* t = s_tree + lane;
  u32* tw = (u32*)(s_tree + (lane & ~1u));
  const u32 incv = p.inc << (16 * (lane & 1));
  tree_init(t, p.n);
  u32 total = p.n;
  u64 low = 0, range = ~0ull, data = 0, used = 8;

  ACode s;
  s.c0 = s.c1 = s.c2 = 0;
  s.off = (u32)((uintptr_t)cp & 3);
  s.nx = s.last = (const u32*)((uintptr_t)cp & ~(uintptr_t)3);
  if (live && err == 0) {
    const u32* w = s.nx;
    s.last = (const u32*)((uintptr_t)(cp + clen - 1) & ~(uintptr_t)3);
    s.c0 = w[0];
    s.c1 = w + 1 <= s.last ? w[1] : 0u;
    s.c2 = w + 2 <= s.last ? w[2] : 0u;
    s.nx = w + 3 <= s.last ? w + 3 : s.last;
    const u32 d0 = acode_take(s, 4);
    data = ((u64)d0 << 32) | acode_take(s, 4);
  }

  for (u64 i = 0;; ++i) {
    const bool act = live && i < n && err == 0;
    if (!__any((int)act)) break;  // wave-uniform exit
    bool rare = false;
    u32 sym = 0;
    if (act) {
      const u64 x = data - low;
      const u64 r = div_total(range, total, recip(total));
      // rfreq = x / r clamped to total - 1: sample_impl.rs:29-44 then picks n - 1
      u32 q = total - 1;
      if (x < r * total) {
        q = min(freq_hint(x, range, total), total - 1);
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
      u32 cum, c;
      sym = tree_find(t, q, total, cum, c);
      low += r * cum;
      range = r * c;
      const u32 kb = (u32)__clzll(low ^ (low + range)) >> 3;  // <= 3: range >= 2^32 here
      low <<= 8 * kb;
      range <<= 8 * kb;
      data = kb ? (data << (8 * kb)) | acode_take(s, kb) : data;
      used += kb;
      rare = range < TOP16;
    }
    if (__builtin_expect(__any((int)rare), 0)) {
      if (rare) {
        while (range < TOP16) {  // range_reduction_expansion (range_coder.rs:126-135)
          range = ~low & (TOP16 - 1);
          low <<= 8;
          range <<= 8;
          data = (data << 8) | acode_take(s, 1);
          used += 1;
        }
      }
    }
    if (act) {
      if (used > clen) {
        err = RC_F_TRUNCATED;  // shift_left_buffer's pop_front panics (decoder.rs:33)
      } else {
        op[i] = (uint8_t)sym;
        tree_add(tw, sym, incv);
        total += p.inc;
      }
    }
    if (((u32)i & p.pmask) == p.pmask) {  // wave-uniform: the period's halving check
      const bool h = act && err == 0 && total > p.limit;
      if (__any((int)h)) {
        if (h) tree_halve(t, total);
      }
    }
  }
  if (live) flags[k] = err;
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
