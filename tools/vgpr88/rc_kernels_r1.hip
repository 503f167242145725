// tools/vgpr88/rc_kernels_r1.hip — the round-1 coder (commit 5f3e404) kept for the 88-VGPR
// repro (tools/vgpr88/README.md).  Not built into the library.
// rc_kernels.hip — MI355X (gfx950) kernels of the batched range coder.
//
// One independent stream ("chunk", a fresh reference Encoder/Decoder) per lane; 64 chunks per
// wave run the reference's sequential per-symbol loop in lock-step.  The arithmetic restates
// src/range_coder.rs (param_update :53-92, left_shift :95-100, no_carry_expansion :110-116,
// range_reduction_expansion :126-135), src/encoder.rs (encode :24-37, finish :40-46) and
// src/decoder.rs (new :14-23, decode :38-54) bit-exactly, with these MI355X-specific choices:
//  * coder state (lower_bound, range, decoder data window) lives in VGPR pairs;
//  * the PModel snapshot (cum, c) and the decoder's inverse-CDF bucket table live in LDS;
//  * the no-carry loop (range_coder.rs:83-85) is evaluated in closed form: it settles exactly
//    k = clz64(low ^ (low + range)) / 8 bytes (proof in DESIGN.md §3), so the wave does not
//    diverge on it;
//  * range / total (range_coder.rs:38-40) is a shift for power-of-two totals and an exact
//    multiply-high by a host-computed reciprocal otherwise (no 64-bit divide on the VALU);
//  * the decoder's find_index division + binary search (sample_impl.rs:27-45) is replaced by a
//    float hint -> LDS bucket table -> exact integer verification r*cum[s] <= data-low <
//    r*cum[s+1], which yields the same index for every input, valid or corrupt;
//  * input symbols are read 16 B per lane per load, output bytes are staged through a per-lane
//    LDS ring and written back 16 B per lane per store.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "range_coder_r1.h"

typedef uint64_t u64;
typedef uint32_t u32;

#define TOP16 (1ull << 48)
#define WG 256
#define WAVES (WG / 64)
#define ENC_RING 16          // dwords per lane in the encoder's output ring (64 B)
#define DEC_RING 16          // dwords per lane in the decoder's input ring (64 B)
#define DEC_RING_ALLOC 18    // + 2 mirror slots so a 12-byte window never wraps
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
};


#ifdef RC_PROBE
// Diagnostic side buffers: per wave {HW_ID, GPR_ALLOC, LDS_ALLOC, XCC_ID,
// t_start lo/hi, t_end lo/hi}; per chunk {changed-canary mask, first changed value}.
__device__ u32 g_probe[(1u << 17) / 64 * 8 * 4];
__device__ u32 g_canary[(1u << 17) * 2 * 4];
#define PROBE_BEGIN()                                                              \
  if ((tid & 63) == 0) {                                                           \
    const u64 pr_t0 = wall_clock64();                                              \
    u32* pp = g_probe + ((blockIdx.x * WG + tid) >> 6) * 8;                        \
    pp[0] = __builtin_amdgcn_s_getreg(0xF804);                                     \
    pp[1] = __builtin_amdgcn_s_getreg(0xF805);                                     \
    pp[2] = __builtin_amdgcn_s_getreg(0xF806);                                     \
    pp[3] = __builtin_amdgcn_s_getreg(0xF814);                                     \
    pp[4] = (u32)pr_t0; pp[5] = (u32)(pr_t0 >> 32);                                \
  }
#define PROBE_END(k)                                                               \
  if (((k) & 63) == 0) {                                                           \
    const u64 pr_t1 = wall_clock64();                                              \
    u32* pp = g_probe + ((k) >> 6) * 8;                                            \
    pp[6] = (u32)pr_t1; pp[7] = (u32)(pr_t1 >> 32);                                \
  }
#else
#define PROBE_BEGIN()
#define PROBE_END(k)
#endif
#ifdef RC_CANARY
// Fill v88..v95 (inside a 96-VGPR allocation, above every register the code names) and read
// them back at the end: any change means the wave wrote past the registers it names.
#define CANARY_SET()                                                               \
  asm volatile("v_mov_b32 v88, 0xca000058\n\tv_mov_b32 v89, 0xca000059\n\t"        \
               "v_mov_b32 v90, 0xca00005a\n\tv_mov_b32 v91, 0xca00005b\n\t"        \
               "v_mov_b32 v92, 0xca00005c\n\tv_mov_b32 v93, 0xca00005d\n\t"        \
               "v_mov_b32 v94, 0xca00005e\n\tv_mov_b32 v95, 0xca00005f" ::          \
                   : "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95")
#define CANARY_CHECK(k)                                                            \
  {                                                                                \
    u32 cv[8];                                                                     \
    asm volatile("v_mov_b32 %0, v88\n\tv_mov_b32 %1, v89\n\tv_mov_b32 %2, v90\n\t"  \
                 "v_mov_b32 %3, v91\n\tv_mov_b32 %4, v92\n\tv_mov_b32 %5, v93\n\t"   \
                 "v_mov_b32 %6, v94\n\tv_mov_b32 %7, v95"                             \
                 : "=v"(cv[0]), "=v"(cv[1]), "=v"(cv[2]), "=v"(cv[3]), "=v"(cv[4]),      \
                   "=v"(cv[5]), "=v"(cv[6]), "=v"(cv[7])::"v88", "v89", "v90", "v91",  \
                   "v92", "v93", "v94", "v95");                                       \
    u32 mask = 0, first = 0;                                                       \
    for (int j = 7; j >= 0; --j)                                                   \
      if (cv[j] != 0xca000058u + j) mask |= 1u << j, first = cv[j];                \
    if ((k) < (1u << 17) * 4) g_canary[2 * (k)] = mask, g_canary[2 * (k) + 1] = first; \
  }
#else
#define CANARY_SET()
#define CANARY_CHECK(k)
#endif

static __device__ __forceinline__ u32 hi32(u64 v) { return (u32)(v >> 32); }

// RangeCoder::range_par_total (range_coder.rs:38-40): range / total, exact.
template <int DIV>
static __device__ __forceinline__ u64 range_par_total(u64 range, const ModelArgs& m) {
  if (DIV == DIV_POW2) return range >> m.lg;
  u64 q = __umul64hi(range, m.magic);  // q in {floor - 1, floor}
  u64 rem = range - q * (u64)m.total;
  return rem >= (u64)m.total ? q + 1 : q;
}

// ------------------------------------------------------------------------------------------
// Encoder
// ------------------------------------------------------------------------------------------
struct EncState {
  u64 low, range;  // RangeCoder state (range_coder.rs:7-12)
  u64 acc;         // settled bytes not yet in the ring (newest byte in the low bits)
  u32 nbits;       // 8 * bytes held in acc (< 32 between symbols)
  u32 wpos;        // byte position (from the 16-B aligned slot base) of the next ring dword
  u32 fpos;        // byte position of the next 16-B granule to store to HBM
  u32 lo_ok, hi_ok;  // writable byte window [lo_ok, hi_ok) relative to the aligned base
  u32 flag;
};

struct EncIO {
  uint8_t* gbase;  // 16-B aligned base of the output slot
  u32* ring;       // this lane's ring column: dword j at ring[j * 64]
};

static __device__ __forceinline__ void enc_push_dword(EncState& st, const EncIO& io, u32 be) {
  io.ring[((st.wpos >> 2) & (ENC_RING - 1)) * 64] = __builtin_bswap32(be);
  st.wpos += 4;
}

// Store granule [fpos, fpos + 16) from the ring; bytes outside [lo_ok, hi_ok) are skipped.
static __device__ __forceinline__ void enc_flush_one(EncState& st, const EncIO& io) {
  const u32* rp = io.ring + ((st.fpos >> 2) & (ENC_RING - 1)) * 64;
  uint4 v = make_uint4(rp[0], rp[64], rp[128], rp[192]);
  if (st.fpos >= st.lo_ok && st.fpos + 16 <= st.hi_ok) {
    *reinterpret_cast<uint4*>(io.gbase + st.fpos) = v;
  } else {
    u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      u32 p = st.fpos + j;
      if (p >= st.lo_ok && p < st.hi_ok) io.gbase[p] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
  }
  st.fpos += 16;
}

static __device__ __forceinline__ void enc_flush_ready(EncState& st, const EncIO& io) {
  while (st.wpos - st.fpos >= 16) enc_flush_one(st, io);
}

// One settled byte (left_shift, range_coder.rs:95-100, done by the caller).
static __device__ __forceinline__ void enc_emit_byte(EncState& st, const EncIO& io, u32 b) {
  st.acc = (st.acc << 8) | b;
  st.nbits += 8;
  if (st.nbits >= 32) {
    st.nbits -= 32;
    enc_push_dword(st, io, (u32)(st.acc >> st.nbits));
  }
}

// Rare paths: the no-carry loop settling >= 4 bytes, and range_reduction_expansion.
static __device__ __forceinline__ void enc_rare(EncState& st, const EncIO& io,
                                                          bool loop1) {
  if (loop1) {
    // no_carry_expansion (range_coder.rs:110-116), byte by byte
    while (((st.low ^ (st.low + st.range)) >> 56) == 0) {
      enc_emit_byte(st, io, (u32)(st.low >> 56));
      st.low <<= 8;
      st.range <<= 8;
    }
  }
  // range_reduction_expansion (range_coder.rs:126-135)
  while (st.range < TOP16) {
    st.range = ~st.low & (TOP16 - 1);
    enc_emit_byte(st, io, (u32)(st.low >> 56));
    st.low <<= 8;
    st.range <<= 8;
  }
  enc_flush_ready(st, io);
}

// Encoder::encode (encoder.rs:24-37) -> RangeCoder::param_update (range_coder.rs:53-92)
template <int DIV>
static __device__ __forceinline__ void enc_symbol(EncState& st, const EncIO& io,
                                                  const ModelArgs& m, const uint2* s_tab,
                                                  u32 sym) {
  uint2 e = s_tab[sym];
  u32 cum = e.x, c = e.y;
  if (c == 0) {  // zero-frequency or out-of-alphabet symbol: flag, keep the lane finite
    if (!st.flag) st.flag = (cum == 0xFFFFFFFFu) ? RC_F_BAD_SYMBOL : RC_F_ZERO_FREQ;
    c = 1;
    cum = 0;
  }
  u64 r = range_par_total<DIV>(st.range, m);
  st.range = r * (u64)c;   // range_coder.rs:65
  st.low += r * (u64)cum;  // range_coder.rs:68-81 (overflow unreachable)
  u32 x = hi32(st.low) ^ hi32(st.low + st.range);
  bool rare = (x == 0);
  if (!rare) {
    // no-carry loop in closed form: k = clz(x) / 8 <= 3 bytes settle
    u32 nb = __clz(x) & 24u;
    u32 lh = hi32(st.low);
    st.acc = (st.acc << nb) | (u64)(u32)(((u64)lh << nb) >> 32);
    st.nbits += nb;
    st.low <<= nb;
    st.range <<= nb;
    if (st.nbits >= 32) {
      st.nbits -= 32;
      enc_push_dword(st, io, (u32)(st.acc >> st.nbits));
    }
  }
  if (rare || st.range < TOP16) enc_rare(st, io, rare);
}

template <int DIV>
__global__ __launch_bounds__(WG) void k_encode_static(ModelArgs m, const uint8_t* __restrict__ syms,
                                                     const u64* __restrict__ sym_off,
                                                     u32 n_chunks, uint8_t* __restrict__ out,
                                                     const u64* __restrict__ out_off,
                                                     u64* __restrict__ out_len,
                                                     u32* __restrict__ flags) {
  __shared__ uint2 s_tab[256];
  __shared__ u32 s_ring[WAVES * ENC_RING * 64];
  const u32 tid = threadIdx.x;
  s_tab[tid] = m.tab[tid];
  __syncthreads();
  const u32 k = blockIdx.x * WG + tid;
#ifdef RC_R1_FLOOR96
  asm volatile("; vgpr floor 96" ::: "v95");
#endif
  CANARY_SET();
  PROBE_BEGIN();
  if (k >= n_chunks) return;

  const u32 lane = tid & 63, wave = tid >> 6;
  EncIO io;
  io.ring = s_ring + wave * ENC_RING * 64 + lane;

  const u64 s0 = sym_off[k], s1 = sym_off[k + 1];
  const u64 o0 = out_off[k], o1 = out_off[k + 1];
  const u32 a = (u32)(((uintptr_t)out + o0) & 15);
  io.gbase = out + o0 - a;
  u64 cap = o1 - o0;
  if (cap > 0xFFFFFF00ull - a) cap = 0xFFFFFF00ull - a;

  EncState st;
  st.low = 0;           // RangeCoder::default (range_coder.rs:13-20)
  st.range = ~0ull;
  st.acc = 0;
  st.nbits = 8 * (a & 3);  // pad bytes ahead of the slot (never stored)
  st.wpos = a & ~3u;
  st.fpos = 0;
  st.lo_ok = a;
  st.hi_ok = a + (u32)cap;
  st.flag = 0;

  const uint8_t* sp = syms + s0;
  const u64 n = s1 - s0;
  u64 i = 0;
  // head: symbols until the input pointer is 16-B aligned
  u64 head = (16 - ((uintptr_t)sp & 15)) & 15;
  if (head > n) head = n;
  for (; i < head; ++i) {
    enc_symbol<DIV>(st, io, m, s_tab, sp[i]);
    enc_flush_ready(st, io);
  }
  // body: 16 symbols per 16-B load, next block prefetched
  const u64 nblk = (n - i) >> 4;
  const uint4* bp = reinterpret_cast<const uint4*>(sp + i);
  uint4 cur = nblk ? bp[0] : make_uint4(0, 0, 0, 0);
  for (u64 b = 0; b < nblk; ++b) {
    uint4 nxt = bp[b + 1 < nblk ? b + 1 : b];
    u32 w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) enc_symbol<DIV>(st, io, m, s_tab, (w[q] >> (8 * j)) & 255u);
      enc_flush_ready(st, io);
    }
    cur = nxt;
  }
  i += nblk << 4;
  for (; i < n; ++i) {
    enc_symbol<DIV>(st, io, m, s_tab, sp[i]);
    enc_flush_ready(st, io);
  }

  // Encoder::finish (encoder.rs:40-46): 8 x left_shift
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    enc_emit_byte(st, io, (u32)(st.low >> 56));
    st.low <<= 8;
  }
  const u32 len = st.wpos + (st.nbits >> 3) - a;
  if (st.nbits) enc_push_dword(st, io, (u32)(st.acc << (32 - st.nbits)));
  const u32 end = a + len;
  if (end < st.hi_ok) st.hi_ok = end;
  while (st.fpos < st.wpos) enc_flush_one(st, io);
  if (!st.flag && (u64)len > cap) st.flag = RC_F_CAPACITY;
  out_len[k] = len;
  flags[k] = st.flag;
  CANARY_CHECK(k);
  PROBE_END(k);
}

// ------------------------------------------------------------------------------------------
// Decoder
// ------------------------------------------------------------------------------------------
struct DecState {
  u64 low, range, data;  // RangeCoder + Decoder::data (decoder.rs:6-12)
  u32 cpos;  // bytes consumed, relative to the 16-B aligned base of the code stream
  u32 fill;  // bytes staged into the ring, same origin
  u32 lim;   // cpos beyond lim == more bytes consumed than the stream holds
  u32 flag;
};

struct DecIO {
  const uint8_t* gnext;  // next 16-B block to fetch
  const uint8_t* glast;  // last block holding a byte of this chunk (fetch clamp)
  uint4 pend;            // in-flight block
  u32* ring;             // this lane's ring column: dword j at ring[j * 64]
};

static __device__ __forceinline__ void dec_refill_one(DecState& st, DecIO& io) {
  const u32 j = (st.fill >> 2) & (DEC_RING - 1);
  u32* rp = io.ring + j * 64;
  rp[0] = io.pend.x;
  rp[64] = io.pend.y;
  rp[128] = io.pend.z;
  rp[192] = io.pend.w;
  if (j == 0) {  // mirror slots 16, 17
    rp[DEC_RING * 64] = io.pend.x;
    rp[(DEC_RING + 1) * 64] = io.pend.y;
  }
  st.fill += 16;
  io.pend = *reinterpret_cast<const uint4*>(io.gnext);
  io.gnext = io.gnext < io.glast ? io.gnext + 16 : io.glast;
}

static __device__ __forceinline__ void dec_refill_ready(DecState& st, DecIO& io) {
  while ((int)(st.fill - st.cpos) < 24) dec_refill_one(st, io);
}

// data = the 8 code bytes ending at cpos, big-endian (Decoder::shift_left_buffer, :31-35)
static __device__ __forceinline__ void dec_window(DecState& st, const DecIO& io) {
  const u32 p = st.cpos - 8;
  const u32* rp = io.ring + ((p >> 2) & (DEC_RING - 1)) * 64;
  const u32 d0 = rp[0], d1 = rp[64], d2 = rp[128];
  const u32 sh = p & 3;
  const u32 w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const u32 w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  st.data = ((u64)__builtin_bswap32(w0) << 32) | __builtin_bswap32(w1);
}

static __device__ __forceinline__ void dec_rare(DecState& st, DecIO& io) {
  // range_reduction_expansion (range_coder.rs:126-135); the decoder only counts the bytes
  while (st.range < TOP16) {
    st.range = ~st.low & (TOP16 - 1);
    st.low <<= 8;
    st.range <<= 8;
    st.cpos += 1;
  }
  dec_refill_ready(st, io);
}

// Decoder::decode (decoder.rs:38-54) with FreqTable::find_index (sample_impl.rs:27-45)
template <int DIV>
static __device__ __forceinline__ u32 dec_symbol(DecState& st, DecIO& io, const ModelArgs& m,
                                                 const uint2* s_tab, const u32* s_lut) {
  const u64 x = st.data - st.low;
  const u64 r = range_par_total<DIV>(st.range, m);
  // hint: q ~ x / r = x * total / range, from the top 32 bits of both (range >= 2^48)
  const u32 e = __clz(hi32(st.range));
  const u32 X = hi32(x << e), R = hi32(st.range << e);
  float qf = (float)X * (m.ftotal * __builtin_amdgcn_rcpf((float)R));
  qf = fminf(qf, 4.0e9f);
  const u32 qh = (u32)qf;
  u32 b = qh >> m.lut_shift;
  b = b < m.lut_max ? b : m.lut_max;
  const u32 ent = s_lut[b];
  u32 s = ((qh - (b << m.lut_shift)) >= (ent >> 16)) ? ((ent >> 8) & 255u) : (ent & 255u);
  uint2 t = s_tab[s];
  u64 A = r * (u64)t.x;
  u64 B = r * (u64)t.y;
  // exact verification: s = #{ j in [1, n-1] : r * cum[j] <= x }  (== the reference's index)
  if (A > x) {
    do {
      --s;
      t = s_tab[s];
      A = r * (u64)t.x;
    } while (A > x);
    B = r * (u64)t.y;
  }
  while (s + 1 < m.n && x - A >= B) {
    ++s;
    t = s_tab[s];
    A = r * (u64)t.x;
    B = r * (u64)t.y;
  }
  if (t.y == 0) {  // only reachable on corrupt input (reference: infinite loop)
    // a stream already over-read would have panicked first (decoder.rs:33)
    if (!st.flag) st.flag = st.cpos > st.lim ? RC_F_TRUNCATED : RC_F_CORRUPT;
    B = r;
  }
  // param_update (range_coder.rs:53-92)
  st.low += A;
  st.range = B;
  const u64 xx = st.low ^ (st.low + st.range);
  const u32 k8 = __clzll(xx) & 56u;  // bytes settled by no_carry_expansion, x 8
  st.low <<= k8;
  st.range <<= k8;
  st.cpos += k8 >> 3;
  if (st.range < TOP16) dec_rare(st, io);
  dec_window(st, io);
  return s;
}

template <int DIV>
__global__ __launch_bounds__(WG) void k_decode_static(
    ModelArgs m, const uint8_t* __restrict__ code, const u64* __restrict__ code_off,
    const u64* __restrict__ code_len, uint8_t* __restrict__ syms_out,
    const u64* __restrict__ sym_off, u32 n_chunks, u32* __restrict__ flags) {
  __shared__ uint2 s_tab[256];
  __shared__ u32 s_lut[LUT_MAX_ENTRIES];
  __shared__ u32 s_ring[WAVES * DEC_RING_ALLOC * 64];
  const u32 tid = threadIdx.x;
  s_tab[tid] = m.tab[tid];
  for (u32 j = tid; j <= m.lut_max; j += WG) s_lut[j] = m.lut[j];
  __syncthreads();
  const u32 k = blockIdx.x * WG + tid;
#ifdef RC_R1_FLOOR96
  asm volatile("; vgpr floor 96" ::: "v95");
#endif
  if (k >= n_chunks) return;

  const u32 lane = tid & 63, wave = tid >> 6;
  DecIO io;
  io.ring = s_ring + wave * DEC_RING_ALLOC * 64 + lane;

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
  const uint8_t* gb = cp - a;
  io.glast = (const uint8_t*)((uintptr_t)(cp + clen - 1) & ~(uintptr_t)15);
  io.gnext = gb;

  DecState st;
  st.low = 0;
  st.range = ~0ull;
  st.flag = 0;
  st.fill = 0;
  st.cpos = a + 8;  // Decoder::new primes 8 bytes (decoder.rs:21)
  st.lim = (u32)(clen < 0xFFFFFF00ull - a ? a + clen : 0xFFFFFF00ull);
  io.pend = *reinterpret_cast<const uint4*>(io.gnext);
  io.gnext = io.gnext < io.glast ? io.gnext + 16 : io.glast;
  dec_refill_ready(st, io);
  dec_window(st, io);

  u64 i = 0;
  u64 head = (16 - ((uintptr_t)op & 15)) & 15;
  if (head > n) head = n;
  for (; i < head; ++i) {
    op[i] = (uint8_t)dec_symbol<DIV>(st, io, m, s_tab, s_lut);
    dec_refill_ready(st, io);
  }
  const u64 nblk = (n - i) >> 4;
  uint4* ob = reinterpret_cast<uint4*>(op + i);
  for (u64 b = 0; b < nblk; ++b) {
    u32 w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) w[q] |= dec_symbol<DIV>(st, io, m, s_tab, s_lut) << (8 * j);
      dec_refill_ready(st, io);
    }
    ob[b] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  i += nblk << 4;
  for (; i < n; ++i) {
    op[i] = (uint8_t)dec_symbol<DIV>(st, io, m, s_tab, s_lut);
    dec_refill_ready(st, io);
  }
  // shift_left_buffer panics once more bytes are needed than the stream holds (decoder.rs:33)
  if (!st.flag && st.cpos > st.lim) st.flag = RC_F_TRUNCATED;
  flags[k] = st.flag;
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
  // one thread = 16 symbols = 4 splitmix words
  const u64 g = (u64)blockIdx.x * WG + threadIdx.x;
  const u64 words_per_chunk = chunk_len >> 4;
  if (g >= total_words) return;
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

__global__ __launch_bounds__(WG) void k_synth_generic(u64 seed, const uint8_t* __restrict__ inv,
                                                     uint8_t* __restrict__ dst, u64 chunk_len,
                                                     u32 n_chunks) {
  // one thread per chunk, byte stores: any chunk_len / alignment (small test inputs)
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
};

struct rc_model {
  int kind;  // 0 static, 1 adaptive
  int device;
  int div;
  ModelArgs args;
  void* dmem;
  u32 inc, limit;  // adaptive parameters
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

rc_status launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? RC_OK : RC_E_DEVICE;
}

}  // namespace

extern "C" {

const char* rc_status_string(rc_status s) {
  switch (s) {
    case RC_OK: return "ok";
    case RC_E_ARG: return "invalid argument";
    case RC_E_BAD_MODEL: return "frequency table rejected";
    case RC_E_DEVICE: return "HIP runtime error";
    case RC_E_NO_DEVICE: return "no usable gfx950 device";
    case RC_E_CHUNK: return "at least one chunk flagged";
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
  *out = c;
  return RC_OK;
}

rc_status rc_ctx_destroy(rc_ctx* ctx) {
  if (!ctx) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  (void)hipStreamSynchronize(ctx->own);
  (void)hipStreamDestroy(ctx->own);
  delete ctx;
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
  mm->inc = mm->limit = 0;
  *out = mm;
  return RC_OK;
}

rc_status rc_model_create_adaptive(rc_ctx* ctx, uint32_t n_symbols, uint32_t increment,
                                   uint32_t limit, rc_model** out) {
  (void)ctx;
  (void)n_symbols;
  (void)increment;
  (void)limit;
  if (out) *out = nullptr;
  return RC_E_ARG;  // implemented in rc_adaptive (next milestone)
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
  if (m->kind != 0 || m->device != ctx->device) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const dim3 grid((n_chunks + WG - 1) / WG), block(WG);
  if (m->div == DIV_POW2)
    hipLaunchKernelGGL(k_encode_static<DIV_POW2>, grid, block, 0, ctx->cur, m->args, syms,
                       sym_off, n_chunks, out, out_off, out_len, flags);
  else
    hipLaunchKernelGGL(k_encode_static<DIV_MAGIC>, grid, block, 0, ctx->cur, m->args, syms,
                       sym_off, n_chunks, out, out_off, out_len, flags);
  return launch_status();
}

rc_status rc_decode_batch(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                          const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                          const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags) {
  if (!ctx || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!code || !code_off || !code_len || !syms_out || !sym_off || !flags) return RC_E_ARG;
  if (m->kind != 0 || m->device != ctx->device) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const dim3 grid((n_chunks + WG - 1) / WG), block(WG);
  if (m->div == DIV_POW2)
    hipLaunchKernelGGL(k_decode_static<DIV_POW2>, grid, block, 0, ctx->cur, m->args, code,
                       code_off, code_len, syms_out, sym_off, n_chunks, flags);
  else
    hipLaunchKernelGGL(k_decode_static<DIV_MAGIC>, grid, block, 0, ctx->cur, m->args, code,
                       code_off, code_len, syms_out, sym_off, n_chunks, flags);
  return launch_status();
}

namespace {
// Synchronous staging through device memory for the host-pointer helpers.
struct DevBuf {
  void* p = nullptr;
  hipStream_t s;
  explicit DevBuf(hipStream_t st) : s(st) {}
  bool alloc(size_t n) { return hipMallocAsync(&p, n ? n : 16, s) == hipSuccess; }
  ~DevBuf() {
    if (p) (void)hipFreeAsync(p, s);
  }
};

rc_status any_flag(const uint32_t* flags, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (flags[i]) return RC_E_CHUNK;
  return RC_OK;
}
}  // namespace

rc_status rc_encode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* syms,
                         const uint64_t* sym_off, uint32_t n_chunks, uint8_t* out,
                         const uint64_t* out_off, uint64_t* out_len, uint32_t* flags) {
  if (!ctx || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!syms || !sym_off || !out || !out_off || !out_len || !flags) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const size_t nsym = sym_off[n_chunks], nout = out_off[n_chunks], noff = 8 * (n_chunks + 1);
  hipStream_t s = ctx->cur;
  DevBuf dsyms(s), dsoff(s), dout(s), doo(s), dlen(s), dfl(s);
  if (!dsyms.alloc(nsym) || !dsoff.alloc(noff) || !dout.alloc(nout) || !doo.alloc(noff) ||
      !dlen.alloc(8 * n_chunks) || !dfl.alloc(4 * n_chunks))
    return RC_E_DEVICE;
  if (hipMemcpyAsync(dsyms.p, syms, nsym, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dsoff.p, sym_off, noff, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(doo.p, out_off, noff, hipMemcpyHostToDevice, s) != hipSuccess)
    return RC_E_DEVICE;
  rc_status st = rc_encode_batch(ctx, m, (const uint8_t*)dsyms.p, (const uint64_t*)dsoff.p,
                                 n_chunks, (uint8_t*)dout.p, (const uint64_t*)doo.p,
                                 (uint64_t*)dlen.p, (uint32_t*)dfl.p);
  if (st != RC_OK) return st;
  if (hipMemcpyAsync(out, dout.p, nout, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(out_len, dlen.p, 8 * n_chunks, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(flags, dfl.p, 4 * n_chunks, hipMemcpyDeviceToHost, s) != hipSuccess)
    return RC_E_DEVICE;
  if (hipStreamSynchronize(s) != hipSuccess) return RC_E_DEVICE;
  return any_flag(flags, n_chunks);
}

rc_status rc_decode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                         const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                         const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags) {
  if (!ctx || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!code || !code_off || !code_len || !syms_out || !sym_off || !flags) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  size_t ncode = 0;
  for (uint32_t i = 0; i < n_chunks; ++i)
    ncode = std::max<size_t>(ncode, (size_t)(code_off[i] + code_len[i]));
  const size_t nsym = sym_off[n_chunks], noff = 8 * (n_chunks + 1);
  hipStream_t s = ctx->cur;
  DevBuf dcode(s), dcoff(s), dclen(s), dsyms(s), dsoff(s), dfl(s);
  if (!dcode.alloc(ncode + 16) || !dcoff.alloc(8 * n_chunks) || !dclen.alloc(8 * n_chunks) ||
      !dsyms.alloc(nsym) || !dsoff.alloc(noff) || !dfl.alloc(4 * n_chunks))
    return RC_E_DEVICE;
  if (hipMemcpyAsync(dcode.p, code, ncode, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dcoff.p, code_off, 8 * n_chunks, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dclen.p, code_len, 8 * n_chunks, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dsoff.p, sym_off, noff, hipMemcpyHostToDevice, s) != hipSuccess)
    return RC_E_DEVICE;
  rc_status st = rc_decode_batch(ctx, m, (const uint8_t*)dcode.p, (const uint64_t*)dcoff.p,
                                 (const uint64_t*)dclen.p, (uint8_t*)dsyms.p,
                                 (const uint64_t*)dsoff.p, n_chunks, (uint32_t*)dfl.p);
  if (st != RC_OK) return st;
  if (hipMemcpyAsync(syms_out, dsyms.p, nsym, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(flags, dfl.p, 4 * n_chunks, hipMemcpyDeviceToHost, s) != hipSuccess)
    return RC_E_DEVICE;
  if (hipStreamSynchronize(s) != hipSuccess) return RC_E_DEVICE;
  return any_flag(flags, n_chunks);
}

rc_status rc_synth_fill(rc_ctx* ctx, uint64_t seed, const uint8_t* inv_cdf_host,
                        uint8_t* syms_dev, uint64_t chunk_len, uint32_t n_chunks) {
  if (!ctx || !inv_cdf_host || !syms_dev) return RC_E_ARG;
  if (n_chunks == 0 || chunk_len == 0) return RC_OK;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  void* dinv = nullptr;
  if (hipMallocAsync(&dinv, 65536, ctx->cur) != hipSuccess) return RC_E_DEVICE;
  if (hipMemcpyAsync(dinv, inv_cdf_host, 65536, hipMemcpyHostToDevice, ctx->cur) !=
      hipSuccess)
    return RC_E_DEVICE;
  if ((chunk_len & 15) == 0 && ((uintptr_t)syms_dev & 15) == 0) {
    const u64 words = (chunk_len >> 4) * (u64)n_chunks;
    const u64 blocks = (words + WG - 1) / WG;
    hipLaunchKernelGGL(k_synth, dim3((u32)blocks), dim3(WG), 0, ctx->cur, seed,
                       (const uint8_t*)dinv, syms_dev, chunk_len, words);
  } else {
    hipLaunchKernelGGL(k_synth_generic, dim3((n_chunks + WG - 1) / WG), dim3(WG), 0, ctx->cur,
                       seed, (const uint8_t*)dinv, syms_dev, chunk_len, n_chunks);
  }
  rc_status st = launch_status();
  (void)hipFreeAsync(dinv, ctx->cur);
  return st;
}

#ifdef RC_PROBE
int rc_probe_read(void* probe, size_t probe_bytes, void* canary, size_t canary_bytes) {
  if (hipMemcpyFromSymbol(probe, HIP_SYMBOL(g_probe), probe_bytes) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(canary, HIP_SYMBOL(g_canary), canary_bytes) != hipSuccess) return -1;
  return 0;
}
#endif
}  // extern "C"
