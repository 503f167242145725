// rc_resume.hip — resumable streams: the reference's per-call Encoder::encode / Decoder::decode
// with the model read on every call (include/range_coder.h, rc_stream_*).
//
// The batch kernels (rc_encode.hip, rc_decode.inc) code whole chunks against one table held in
// LDS.  The reference's public surface is per call instead: Encoder::encode reads the caller's
// (c_freq(i), cum_freq(i), total_freq()) at that moment (encoder.rs:24-31) and Decoder::decode
// runs find_index and reads the table again (decoder.rs:38-50), so a caller may change its
// PModel between calls.  These kernels keep one stream's state (RangeCoder, decoder data window,
// 64-bit stream position) in rc_stream_state between launches, and take per-symbol triples
// (encode) or the table of the next n symbols (decode).  One lane per stream: the host mirrors
// (api.py Encoder / Decoder, range_coder.hpp) run one stream, so this path is latency-, not
// bandwidth-bound; the arithmetic is the reference's, branch for branch, with its panics and
// endless loops turned into sticky flags:
//   total == 0                       -> RC_F_BAD_MODEL (u64 / 0, range_coder.rs:38-40)
//   low + r*cum overflows            -> RC_F_BAD_MODEL (LowerBoundOverflow, :68-81)
//   range == r*c == 0                -> RC_F_ZERO_FREQ / RC_F_CORRUPT (:83-85 never ends)
//   low + range overflows            -> RC_F_BAD_MODEL (upper_bound().unwrap(), :138-146)
//   decoder needs a byte past the end -> RC_F_TRUNCATED (pop_front().unwrap(), decoder.rs:33)
// u64 products wrap (release-build semantics of the reference).
#include "rc_common.h"
#include "rc_udiv.h"

#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <unordered_map>

#define RWG 64
#define TOP8 (1ull << 56)  // range_coder.rs:23

static_assert(sizeof(rc_stream_state) == 48, "rc_stream_state layout");

namespace {

// RangeCoder::param_update up to the renormalisation loops: the narrowed interval, or a flag
struct Narrow {
  u64 low, range;
  u32 err;
};

// (r = range_par_total, range_coder.rs:38-40)
static __device__ __forceinline__ Narrow narrow_r(u64 low, u64 range, u64 r, u32 c, u32 cum,
                                                  u32 zero_flag) {
  Narrow o{low, range, 0u};
  const u64 nr = r * (u64)c;     // range_coder.rs:65
  const u64 add = r * (u64)cum;  // :68
  const u64 nl = low + add;
  if (nl < add) o.err = RC_F_BAD_MODEL;          // overflowing_add -> Err (:68-81)
  else if (nr == 0) o.err = zero_flag;           // no_carry_expansion never terminates
  else if (nl + nr < nr) o.err = RC_F_BAD_MODEL;  // upper_bound() overflow (:138-146)
  o.low = nl;
  o.range = nr;
  return o;
}
static __device__ __forceinline__ Narrow narrow(u64 low, u64 range, u32 c, u32 cum, u32 total,
                                                u32 zero_flag) {
  if (total == 0) return Narrow{low, range, RC_F_BAD_MODEL};  // range_par_total divides by 0
  return narrow_r(low, range, rc_udiv64(range, total), c, cum, zero_flag);
}

// bytes the two renormalisation loops settle from (low, range), without applying them
static __device__ __forceinline__ u32 settle_count(u64 low, u64 range) {
  u32 k = 0;
  while (((low ^ (low + range)) >> 56) == 0) {  // no_carry_expansion (:110-116)
    low <<= 8;
    range <<= 8;
    ++k;
  }
  while (range < TOP16) {  // range_reduction_expansion (:126-135)
    range = ~low & (TOP16 - 1);
    low <<= 8;
    range <<= 8;
    ++k;
  }
  return k;
}

// byte store into the body's block: global memory (the launch path) or LDS (the service; the
// pointer is generic, derived from the LDS block, and the compiler infers the address space)
template <bool kLds>
static __device__ __forceinline__ void bstore(uint8_t* p, u32 v) {
  if constexpr (kLds) *p = (uint8_t)v;
  else gstore8(p, v);
}

// Encoder::encode x n (+ finish) for stream k (the body of k_stream_encode and of the service)
template <bool kLds>
static __device__ void stream_encode_one(
    u32 k, rc_stream_state* __restrict__ st, const u32* __restrict__ trip,
    const u64* __restrict__ sym_off, uint8_t* __restrict__ out, const u64* __restrict__ out_off,
    u64* __restrict__ out_len, uint8_t* __restrict__ nbytes, u32 finish,
    u32* __restrict__ flags) {
  rc_stream_state S = st[k];
  const u64 s0 = sym_off[k], n = sym_off[k + 1] - s0;
  uint8_t* o = out + out_off[k];
  const u64 cap = out_off[k + 1] - out_off[k];
  out_len[k] = 0;
  if (S.flags) {  // the reference panicked (or hung) at an earlier call
    flags[k] = S.flags;
    return;
  }
  if (S.stage == 2) {  // Encoder::finish took the encoder by value (encoder.rs:40)
    S.flags = RC_F_FINISHED;
    st[k] = S;
    flags[k] = S.flags;
    return;
  }
  if (cap < RC_STREAM_MAX_BYTES(n, finish)) {  // not sticky: the caller retries, nothing changed
    flags[k] = RC_F_CAPACITY;
    return;
  }
  u64 low = S.lower_bound, range = S.range, w = 0;
  for (u64 i = 0; i < n; ++i) {  // Encoder::encode (encoder.rs:24-37)
    const u32* t = trip + 3 * (s0 + i);
    const Narrow q = narrow(low, range, t[0], t[1], t[2], RC_F_ZERO_FREQ);
    if (q.err) {
      S.flags = q.err;
      break;
    }
    low = q.low;
    range = q.range;
    u32 nb = 0;
    while (((low ^ (low + range)) >> 56) == 0) {  // no_carry_expansion (:110-116)
      bstore<kLds>(o + w++, (u32)(low >> 56));  // left_shift (:95-100)
      low <<= 8;
      range <<= 8;
      ++nb;
    }
    while (range < TOP16) {  // range_reduction_expansion (:126-135)
      range = ~low & (TOP16 - 1);
      bstore<kLds>(o + w++, (u32)(low >> 56));
      low <<= 8;
      range <<= 8;
      ++nb;
    }
    if (nbytes) bstore<kLds>(nbytes + s0 + i, nb);  // encode()'s return value (encoder.rs:34-36)
    S.n += 1;
  }
  if (finish && !S.flags) {  // Encoder::finish: 8 x left_shift (encoder.rs:40-46)
    for (int j = 0; j < 8; ++j) {
      bstore<kLds>(o + w++, (u32)(low >> 56));
      low <<= 8;
      range <<= 8;
    }
    S.stage = 2;
  } else if (S.stage == 0) {
    S.stage = 1;
  }
  S.lower_bound = low;
  S.range = range;
  S.pos += w;
  st[k] = S;
  out_len[k] = w;
  flags[k] = S.flags;
}

__global__ __launch_bounds__(RWG) void k_stream_encode(
    rc_stream_state* __restrict__ st, const u32* __restrict__ trip, const u64* __restrict__ sym_off,
    u32 n_streams, uint8_t* __restrict__ out, const u64* __restrict__ out_off,
    u64* __restrict__ out_len, uint8_t* __restrict__ nbytes, u32 finish,
    u32* __restrict__ flags) {
  const u32 k = blockIdx.x * RWG + threadIdx.x;
  if (k >= n_streams) return;
  RC_VGPR_FLOOR_48();
  stream_encode_one<false>(k, st, trip, sym_off, out, out_off, out_len, nbytes, finish, flags);
}

// Decoder::decode x n for stream k against the table in LDS (the body of k_stream_decode and of
// the service)
template <bool kLds>
static __device__ void stream_decode_one(
    u32 k, const u32* s_c, const u32* s_cum, u32 n_alpha, u32 total,
    rc_stream_state* __restrict__ st, const uint8_t* __restrict__ code,
    const u64* __restrict__ code_off, const u64* __restrict__ code_len,
    uint8_t* __restrict__ syms, const u64* __restrict__ sym_off, u32* __restrict__ flags) {
  rc_stream_state S = st[k];
  const uint8_t* cp = code + code_off[k];
  const u64 clen = code_len[k];
  const u64 s0 = sym_off[k], n = sym_off[k + 1] - s0;
  if (S.flags) {
    flags[k] = S.flags;
    return;
  }
  if (S.stage == 0) {  // Decoder::new: the first 8 bytes (decoder.rs:14-23)
    if (clen < 8) {
      S.flags = RC_F_TRUNCATED;
      st[k] = S;
      flags[k] = S.flags;
      return;
    }
    u64 d = 0;
    for (int j = 0; j < 8; ++j) d = (d << 8) | cp[j];
    S.data = d;
    S.pos = 8;
    S.stage = 1;
  }
  u64 low = S.lower_bound, range = S.range, data = S.data, pos = S.pos;
  for (u64 i = 0; i < n; ++i) {  // Decoder::decode (decoder.rs:38-54)
    if (total == 0) {            // find_index's range_par_total divides by zero
      S.flags = RC_F_BAD_MODEL;
      break;
    }
    // FreqTable::find_index (sample_impl.rs:27-45): rfreq, then the binary search over cum.
    // (r == 0 divides by zero there; param_update below then flags the step, r * c == 0.)
    const u64 r = rc_udiv64(range, total);
    const u64 rfreq = r ? rc_udiv64(data - low, r) : 0;
    u32 left = 0, right = n_alpha - 1;
    if constexpr (kLds) {
      // the service: the whole wave runs this body on the same values, so every comparison
      // the search could make (cum[j + 1] <= rfreq, j < n_alpha - 1) is taken at once, four
      // per lane, into a 256-bit mask; the search then walks the mask, step for step the same
      // bisection, without an LDS round trip per step
      const u32 lane = threadIdx.x;
      u64 m[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const u32 j = lane + 64 * h;
        m[h] = __ballot(j + 1 < n_alpha && (u64)s_cum[j + 1] <= rfreq);
      }
      while (left < right) {
        const u32 mid = (left + right) >> 1;
        const u64 w = mid < 64 ? m[0] : mid < 128 ? m[1] : mid < 192 ? m[2] : m[3];
        if ((w >> (mid & 63)) & 1) left = mid + 1;
        else right = mid;
      }
    } else {
      while (left < right) {
        const u32 mid = (left + right) >> 1;
        if ((u64)s_cum[mid + 1] <= rfreq) left = mid + 1;
        else right = mid;
      }
    }
    const Narrow q = narrow_r(low, range, r, s_c[left], s_cum[left], RC_F_CORRUPT);
    if (q.err) {
      S.flags = q.err;
      break;
    }
    const u32 nb = settle_count(q.low, q.range);
    if (pos + nb > clen) {  // shift_left_buffer pops past the end (decoder.rs:31-35)
      S.flags = RC_F_TRUNCATED;
      break;
    }
    low = q.low;
    range = q.range;
    while (((low ^ (low + range)) >> 56) == 0) {
      low <<= 8;
      range <<= 8;
    }
    while (range < TOP16) {
      range = ~low & (TOP16 - 1);
      low <<= 8;
      range <<= 8;
    }
    for (u32 j = 0; j < nb; ++j) data = (data << 8) | cp[pos++];
    bstore<kLds>(syms + s0 + i, left);
    S.n += 1;
  }
  S.lower_bound = low;
  S.range = range;
  S.data = data;
  S.pos = pos;
  st[k] = S;
  flags[k] = S.flags;
}

__global__ __launch_bounds__(RWG) void k_stream_decode(
    const u32* __restrict__ c_tab, const u32* __restrict__ cum_tab, u32 n_alpha, u32 total,
    rc_stream_state* __restrict__ st, const uint8_t* __restrict__ code,
    const u64* __restrict__ code_off, const u64* __restrict__ code_len,
    uint8_t* __restrict__ syms, const u64* __restrict__ sym_off, u32 n_streams,
    u32* __restrict__ flags) {
  __shared__ u32 s_c[256], s_cum[256];
  for (u32 j = threadIdx.x; j < n_alpha; j += RWG) {
    s_c[j] = c_tab[j];
    s_cum[j] = cum_tab[j];
  }
  __syncthreads();
  const u32 k = blockIdx.x * RWG + threadIdx.x;
  if (k >= n_streams) return;
  RC_VGPR_FLOOR_64();
  stream_decode_one<false>(k, s_c, s_cum, n_alpha, total, st, code, code_off, code_len, syms,
                           sym_off, flags);
}

// ------------------------------------------------------------------------------------------
// The stream service: one persistent wave per context that takes the one-stream host calls
// (rc_stream_encode_host / rc_stream_decode_host) from a mailbox in host memory, so a call is
// a store of its request block plus a poll, not a copy, a launch, a copy and a stream
// synchronisation (caller-adaptive Decoder::decode, decoder.rs:38-54, paid a
// launch and two pinned round trips per symbol).
//
// The mailbox is pinned, coherent, device-mapped host memory.  The host writes the request
// block (the same layout the launch path copies to the device) and then `seq` (release); the
// wave polls `seq` (system-scope acquire), reads the header and block into LDS with all 64
// lanes, runs the same per-stream body as the launch path on lane 0 against the block in LDS
// (so the body's loads and stores cost LDS latency, not device-memory round trips), writes the
// result ranges back into the mailbox and sets `ack` (release).  It leaves on `stop`, after
// SVC_IDLE_US without a request, after SVC_LIFE_US in all, or when a launch of the library asks
// it to yield (`yield_ep` = its epoch: rc_svc_yield_all_), so it never outlives its caller
// for long: a later call starts a new one (an epoch: `alive` is 2 epoch + 1 while epoch's wave
// runs and 2 epoch + 2 once it left).  Every exit condition is checked on every poll.
// ------------------------------------------------------------------------------------------
// (short on purpose: a resident wave holds its hardware queue, and HIP maps the process's
// streams onto 4 queues, so a kernel on another stream may sit behind the wave until it leaves;
// the library's own launches ask it to leave first, rc_svc_yield_all_)
#define SVC_IDLE_US 250
#define SVC_LIFE_US 1000
#define SVC_BLOCK (64u << 10)  // request / result block bytes (larger calls take the launch path)
#define SVC_STOP 0xFFFFFFFFu   // a seq value: leave now (a request number never reaches it)
enum { SVC_ENCODE = 1, SVC_DECODE = 2 };

struct alignas(64) SvcBox {
  u32 seq;            // host -> wave: request number (written last)
  u32 yield_ep;       // host -> wave: the wave of this epoch leaves (read with seq, one load)
  u32 p0[14];
  u32 ack, p1[15];    // wave -> host: the last request done
  u32 alive, p2[15];  // wave: 2 epoch + 1 running, 2 epoch + 2 left
  u32 stop, p3[15];   // host: leave now
  u32 op, n_alpha, total, finish;
  u64 in_bytes;               // block bytes the wave reads (a multiple of 16)
  u64 head_bytes;             // result head [0, head_bytes) copied back (multiple of 16)
  u64 tail_off, tail_bytes;   // result tail [tail_off, + tail_bytes) copied back (multiples of 16)
  u64 o[8];                   // byte offsets of the body's arguments inside the block
  u32 probe[4];  // wave -> host: 10-ns ticks from seeing seq to: block in LDS, body done,
                 // results written (rc_svc_probe_)
};
static_assert(sizeof(SvcBox) == 384, "mailbox header layout");
// header + block in LDS (one workgroup may hold up to 160 KiB on gfx950)
static_assert(sizeof(SvcBox) + SVC_BLOCK <= 96u << 10, "service LDS block");

static __device__ __forceinline__ u32 sys_load(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static __device__ __forceinline__ u64 sys_load64(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static __device__ __forceinline__ void sys_store(u32* p, u32 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// copy [off, off + bytes) (16-B multiples) from src to dst with the wave's 64 lanes, eight
// 16-B loads in flight per lane before the first store
static __device__ __forceinline__ void svc_copy(char* dst, const char* src, u64 off, u64 bytes,
                                                u32 lane) {
  const u64 end = off + bytes;
  u64 i = off + 16 * lane;
  for (; i + 7 * 16 * RWG < end; i += 8 * 16 * RWG) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *(const u32x4*)(src + i + j * 16 * RWG);
#pragma unroll
    for (int j = 0; j < 8; ++j) *(u32x4*)(dst + i + j * 16 * RWG) = v[j];
  }
  for (; i < end; i += 16 * RWG) *(u32x4*)(dst + i) = *(const u32x4*)(src + i);
}

#define SVC_BURST 4096u  // bytes of the mailbox read in one burst (header + the block's start)
// field at byte `off` of the burst held by the lanes (lane l holds bytes 16 (l + 64 j) ..)
static __device__ __forceinline__ u32 burst32(const u32x4* v, u32 off) {
  const u32x4& q = v[off / 1024];
  const u32 w = (off / 4) % 4;
  const u32 x = w == 0 ? q.x : w == 1 ? q.y : w == 2 ? q.z : q.w;
  return __builtin_amdgcn_readlane(x, (off / 16) % 64);
}
static __device__ __forceinline__ u64 burst64(const u32x4* v, u32 off) {
  return ((u64)burst32(v, off + 4) << 32) | burst32(v, off);
}

__global__ __launch_bounds__(RWG) void k_stream_service(SvcBox* box, u32 epoch, u64 idle_ticks,
                                                        u64 life_ticks) {
  __shared__ __attribute__((aligned(16))) char s_box[sizeof(SvcBox) + SVC_BLOCK];
  const u32 lane = threadIdx.x;
  char* const hbox = (char*)box;
  char* const sblk = s_box + sizeof(SvcBox);
  u32 done = __builtin_amdgcn_readfirstlane(sys_load(&box->ack));
  if (lane == 0) sys_store(&box->alive, 2 * epoch + 1);
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  u64 tl = t0;
  u32 polls = 0;
  for (;;) {
    // one load per poll: `stop` is rc_ctx_destroy's (checked every 64 polls), seq == SVC_STOP
    // is the same request from a caller that holds the mailbox
    const u64 sy = sys_load64((const u64*)&box->seq);  // {seq, yield_ep}
    const u32 seq = __builtin_amdgcn_readfirstlane((u32)sy);
    const u32 ye = __builtin_amdgcn_readfirstlane((u32)(sy >> 32));
    const u64 now = __builtin_amdgcn_s_memrealtime();
    if (seq == SVC_STOP || ye == epoch || now - t0 > life_ticks) break;
    if ((++polls & 63) == 0 && __builtin_amdgcn_readfirstlane(sys_load(&box->stop))) break;
    if (seq == done) {
      if (now - tl > idle_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const u64 td = now;
    // The request in one burst: the first 4 KiB of the mailbox (header and block), every load
    // in flight before the first is used, so a one-symbol call costs one PCIe round trip; the
    // header fields come out of the lanes' registers.  (Plain loads: the acquire of seq orders
    // them after the host's stores.)
    u32x4 v[SVC_BURST / 1024];
#pragma unroll
    for (u32 j = 0; j < SVC_BURST / 1024; ++j) v[j] = *(const u32x4*)(hbox + 16 * (lane + 64 * j));
    const u32 op = burst32(v, offsetof(SvcBox, op));
    const u64 in_b = burst64(v, offsetof(SvcBox, in_bytes));
    const u64 head_b = burst64(v, offsetof(SvcBox, head_bytes));
    const u64 t_off = burst64(v, offsetof(SvcBox, tail_off));
    const u64 t_b = burst64(v, offsetof(SvcBox, tail_bytes));
    u64 o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = burst64(v, offsetof(SvcBox, o) + 8 * j);
#pragma unroll
    for (u32 j = 0; j < SVC_BURST / 1024; ++j) *(u32x4*)(s_box + 16 * (lane + 64 * j)) = v[j];
    if (sizeof(SvcBox) + in_b > SVC_BURST)
      svc_copy(s_box, hbox, SVC_BURST, sizeof(SvcBox) + in_b - SVC_BURST, lane);
    __syncthreads();
    const u64 t1 = __builtin_amdgcn_s_memrealtime();
    if (op == SVC_DECODE) {
      const u32 na = burst32(v, offsetof(SvcBox, n_alpha)), tot = burst32(v, offsetof(SvcBox, total));
      // block: state | offsets (code_off, code_len, sym_off[0..1]) | flags | c | cum | window | syms
      // (all lanes: the search is wave-wide; every lane computes and stores the same values)
      stream_decode_one<true>(0, (const u32*)(sblk + o[2]), (const u32*)(sblk + o[3]), na, tot,
                                (rc_stream_state*)sblk, (const uint8_t*)(sblk + o[4]),
                                (const u64*)(sblk + o[0]), (const u64*)(sblk + o[0] + 8),
                                (uint8_t*)(sblk + o[5]), (const u64*)(sblk + o[0] + 16),
                                (u32*)(sblk + o[1]));
    } else if (op == SVC_ENCODE) {
      const u32 fin = burst32(v, offsetof(SvcBox, finish));
      // block: state | offsets (sym_off[0..1], out_off[0..1]) | out_len | flags | triples | nb | out
      if (lane == 0)
        stream_encode_one<true>(0, (rc_stream_state*)sblk, (const u32*)(sblk + o[3]),
                                (const u64*)(sblk + o[0]), (uint8_t*)(sblk + o[5]),
                                (const u64*)(sblk + o[0] + 16), (u64*)(sblk + o[1]),
                                o[6] ? (uint8_t*)(sblk + o[4]) : (uint8_t*)nullptr, fin,
                                (u32*)(sblk + o[2]));
    }
    __syncthreads();
    const u64 t2 = __builtin_amdgcn_s_memrealtime();
    char* const hblk = hbox + sizeof(SvcBox);
    svc_copy(hblk, sblk, 0, head_b, lane);
    svc_copy(hblk, sblk, t_off, t_b, lane);
    if (lane == 0) {
      const u64 t3 = __builtin_amdgcn_s_memrealtime();
      u32x4 pr = {(u32)(t1 - td), (u32)(t2 - td), (u32)(t3 - td), 0u};
      *(u32x4*)box->probe = pr;
    }
    // (the release below waits for every store of this one-wave workgroup, all lanes: vmcnt
    // counts per wave, so no separate system fence)
    if (lane == 0) sys_store(&box->ack, seq);
    done = seq;
    tl = __builtin_amdgcn_s_memrealtime();
  }
  __threadfence_system();
  if (lane == 0) sys_store(&box->alive, 2 * epoch + 2);
}

struct Dev {
  int prev = -1;
  explicit Dev(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~Dev() {
    int now = -1;
    if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
  }
};

// The host variants' staging: one pinned host block and its device mirror per context, grown on
// demand and kept until rc_ctx_destroy.  Every transfer is one DMA between the two (pageable
// caller memory is only touched by host memcpy), so copies and the kernel are plainly ordered
// on the context's stream.  (Small async copies to and from pageable memory returned wrong
// bytes intermittently on this stack; pinned staging is also the faster path.)  The block is
// held under its own mutex for the whole call: the Python mirrors share one default context
// between threads, and ctypes releases the GIL inside the call.  A call keeps its Stage alive
// by a shared_ptr, so an rc_ctx_destroy racing with it cannot free the mutex under it; the
// release marks the block dead, and a call that already held the shared_ptr and locks it
// afterwards fails instead of re-growing a block nobody would free.  (A call that starts after
// rc_ctx_destroy uses a destroyed context: a caller contract violation, as with every rc_*
// entry point.)
struct Stage {
  std::mutex mu;
  char* host = nullptr;
  char* dev = nullptr;
  size_t cap = 0;
  bool dead = false;
};
std::mutex g_stage_mu;
std::unordered_map<const rc_ctx*, std::shared_ptr<Stage>> g_stages;

// Locks the context's block (released when `lk` goes out of scope; `keep` holds the block
// alive until then, so declare it before `lk`) and grows it to `bytes`.
char* stage_acquire(const rc_ctx* ctx, size_t bytes, char** dev, std::shared_ptr<Stage>* keep,
                    std::unique_lock<std::mutex>* lk) {
  {
    std::lock_guard<std::mutex> g(g_stage_mu);
    auto& slot = g_stages[ctx];
    if (!slot) slot = std::make_shared<Stage>();
    *keep = slot;
  }
  Stage* st = keep->get();
  *lk = std::unique_lock<std::mutex>(st->mu);
  if (st->dead) return nullptr;  // the context is being destroyed
  if (st->cap < bytes) {
    if (st->host) (void)hipHostFree(st->host);
    if (st->dev) (void)hipFree(st->dev);
    st->host = st->dev = nullptr;
    st->cap = 0;
    const size_t cap = std::max<size_t>(bytes + bytes / 2, 1u << 16);
    if (hipHostMalloc((void**)&st->host, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    if (hipMalloc((void**)&st->dev, cap) != hipSuccess) {
      (void)hipHostFree(st->host);
      st->host = nullptr;
      return nullptr;
    }
    st->cap = cap;
  }
  *dev = st->dev;
  return st->host;
}

// Above this many worst-case output bytes, rc_stream_encode_host reads back the state first and
// then only the bytes written (two waits); below it one copy of the whole region is cheaper.
constexpr u64 kTwoPhaseBytes = 256u << 10;

// The context's stream service (host side): the mailbox, the wave's own
// non-blocking stream.  Held under its mutex for a whole call, like the staging block.
struct Svc {
  std::mutex mu;
  SvcBox* box = nullptr;  // host address of the mailbox (header, then the block)
  SvcBox* dbox_host = nullptr;  // device address of the mailbox (mapped host memory)
  hipStream_t stream = nullptr;
  u32 epoch = 0, seq = 0;
  bool launched = false, dead = false, broken = false;
  u64 probe[5] = {0, 0, 0, 0, 0};  // calls, the wave's three intervals, the host's wait (ns)
};
std::mutex g_svc_mu;
std::unordered_map<const rc_ctx*, std::shared_ptr<Svc>> g_svcs;
// at process exit, tell any running wave to leave (no HIP calls: the runtime may be going too;
// a wave leaves within one poll, and by SVC_IDLE_US in any case).  The box is written only under
// its service's lock, which a call that times out holds while it frees the box; a service whose
// lock another thread holds is skipped (its wave leaves by itself after SVC_IDLE_US).
struct SvcAtExit {
  ~SvcAtExit() {
    std::lock_guard<std::mutex> g(g_svc_mu);
    for (auto& kv : g_svcs) {
      if (!kv.second) continue;
      std::unique_lock<std::mutex> lk(kv.second->mu, std::try_to_lock);
      if (lk.owns_lock() && kv.second->box)
        __atomic_store_n(&kv.second->box->stop, 1u, __ATOMIC_RELEASE);
    }
  }
} g_svc_at_exit;

// RC_STREAM_SERVICE=0 in the environment of rc_ctx_create sends every call of that context down
// the launch path (RcKnobs, rc_common.h)
bool svc_enabled(const rc_ctx* ctx) { return rc_ctx_knobs_(ctx).stream_service; }

// Test hook (tests/test_gpu_stream.py, not in include/range_coder.h): the wave's idle time in
// 10-ns ticks for the waves launched from now on (0: SVC_IDLE_US), so a test can make waves
// leave at the moment requests are published.
std::atomic<u64> g_svc_idle_ticks{0};
std::atomic<bool> g_svc_any{false};  // some service wave was ever launched (rc_svc_yield_all_)
u64 idle_ticks() {
  const u64 t = g_svc_idle_ticks.load(std::memory_order_relaxed);
  return t ? t : (u64)SVC_IDLE_US * 100ull;
}

std::shared_ptr<Svc> svc_get(const rc_ctx* ctx) {
  // (the calling thread's last context, without the global lock and map: a per-symbol caller
  // comes here at every call; a context destroyed since, or a new one at the same address,
  // finds its entry dead or gone and looks it up again)
  thread_local const rc_ctx* last_ctx = nullptr;
  thread_local std::weak_ptr<Svc> last_sv;
  if (ctx == last_ctx) {
    std::shared_ptr<Svc> sv = last_sv.lock();
    if (sv && !__atomic_load_n(&sv->dead, __ATOMIC_ACQUIRE)) return sv;
  }
  std::lock_guard<std::mutex> g(g_svc_mu);
  auto& slot = g_svcs[ctx];
  if (!slot) slot = std::make_shared<Svc>();
  last_ctx = ctx;
  last_sv = slot;
  return slot;
}

// stop the wave (if any) and free everything; the caller holds sv->mu
void svc_teardown(Svc* sv) {
  if (sv->box) {
    __atomic_store_n(&sv->box->stop, 1u, __ATOMIC_RELEASE);
    if (sv->stream) (void)hipStreamSynchronize(sv->stream);
  }
  if (sv->stream) (void)hipStreamDestroy(sv->stream);
  if (sv->box) (void)hipHostFree(sv->box);
  sv->stream = nullptr;
  sv->box = nullptr;
  sv->dbox_host = nullptr;
  sv->launched = false;
}

// One request through the service.  fill(h) writes the request block at h (in the mailbox) and
// the header fields; after the wave acknowledged it, the results are in the same block.
// Returns false (and the call takes the launch path) when the service is off, broken, or
// cannot be set up; RC_E_DEVICE in *err when the wave did not answer.
template <class Fill>
bool svc_call(const rc_ctx* ctx, Svc* sv, int dev, Fill fill, rc_status* err) {
  if (sv->dead || sv->broken) return false;
  if (!sv->box) {
    Dev g(dev);
    void* hb = nullptr;
    if (hipHostMalloc(&hb, sizeof(SvcBox) + SVC_BLOCK,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      sv->broken = true;
      return false;
    }
    memset(hb, 0, sizeof(SvcBox));
    sv->box = (SvcBox*)hb;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hb, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&sv->stream, hipStreamNonBlocking) != hipSuccess) {
      svc_teardown(sv);
      sv->broken = true;
      return false;
    }
    sv->dbox_host = (SvcBox*)dp;
  }
  SvcBox* b = sv->box;
  fill((char*)(b + 1), b);
  if (++sv->seq == SVC_STOP) sv->seq = 1;  // (SVC_STOP is the stop request, never a number)
  const u32 s = sv->seq;
  __atomic_store_n(&b->seq, s, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  auto t_run = t0;  // (the last time the current epoch's wave was seen not running)
  for (u32 spin = 0;; ++spin) {
    if (__atomic_load_n(&b->ack, __ATOMIC_ACQUIRE) == s) {
      sv->probe[0] += 1;
      for (int j = 0; j < 3; ++j) sv->probe[1 + j] += b->probe[j];
      sv->probe[4] += (u64)std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now() - t0).count();
      return true;
    }
    // no wave of the current epoch running: start one (it takes the pending request)
    if (!sv->launched || __atomic_load_n(&b->alive, __ATOMIC_ACQUIRE) == 2 * sv->epoch + 2) {
      Dev g(dev);
      ++sv->epoch;
      hipLaunchKernelGGL(k_stream_service, dim3(1), dim3(RWG), 0, sv->stream, sv->dbox_host,
                         sv->epoch, idle_ticks(),
                         (u64)SVC_LIFE_US * 100ull);
      if (hipGetLastError() != hipSuccess) {
        sv->broken = true;
        *err = RC_E_DEVICE;
        return true;
      }
      sv->launched = true;
      g_svc_any.store(true, std::memory_order_relaxed);
    }
    if ((spin & 1023) == 1023) {
      // The timeout runs only while the current epoch's wave runs: a wave still waiting for a
      // CU (another long kernel holding the LDS it needs) is waited for, as a launch would be;
      // a wave that cannot start because the device failed shows in the stream query below.
      const auto now = std::chrono::steady_clock::now();
      if (__atomic_load_n(&b->alive, __ATOMIC_ACQUIRE) != 2 * sv->epoch + 1) t_run = now;
      if (now - t_run > std::chrono::seconds(10)) {
        svc_teardown(sv);  // (waits for the wave to leave: every exit is bounded)
        sv->broken = true;
        *err = RC_E_DEVICE;
        return true;
      }
      // (one query: a wave that leaves between two queries would read as a fault)
      const hipError_t q = hipStreamQuery(sv->stream);
      if (q != hipSuccess && q != hipErrorNotReady) {
        sv->broken = true;
        *err = RC_E_DEVICE;
        return true;
      }
    }
    __builtin_ia32_pause();
  }
}

}  // namespace

// Every launch of a batch kernel by the library first asks the process's running service waves
// to leave (their yield_ep := their epoch): such a wave may hold the hardware queue that the
// batch kernel's stream maps to, and the batch kernel would otherwise wait up to SVC_LIFE_US
// behind it.  The next per-call request launches a new wave.  A service whose lock a call
// holds is skipped (its wave is serving that call, and leaves by SVC_LIFE_US at the latest).
void rc_svc_yield_all_() {
  if (!g_svc_any.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> g(g_svc_mu);
  for (auto& kv : g_svcs) {
    Svc* sv = kv.second.get();
    if (!sv) continue;
    std::unique_lock<std::mutex> lk(sv->mu, std::try_to_lock);
    if (lk.owns_lock() && sv->box && sv->launched)
      __atomic_store_n(&sv->box->yield_ep, sv->epoch, __ATOMIC_RELEASE);
  }
}

extern "C" {

rc_status rc_ctx_stream_(rc_ctx* ctx, hipStream_t* s, int* device);  // rc_kernels.hip

rc_status rc_stream_encode(rc_ctx* ctx, rc_stream_state* states, const uint32_t* triples,
                           const uint64_t* sym_off, uint32_t n_streams, uint8_t* out,
                           const uint64_t* out_off, uint64_t* out_len, uint8_t* nbytes,
                           uint32_t finish, uint32_t* flags) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || n_streams > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_streams == 0) return RC_OK;
  if (!states || !triples || !sym_off || !out || !out_off || !out_len || !flags) return RC_E_ARG;
  Dev g(dev);
  rc_svc_yield_all_();
  hipLaunchKernelGGL(k_stream_encode, dim3((n_streams + RWG - 1) / RWG), dim3(RWG), 0, s,
                     states, triples, sym_off, n_streams, out, out_off, out_len, nbytes, finish,
                     flags);
  return hipGetLastError() == hipSuccess ? RC_OK : RC_E_DEVICE;
}

rc_status rc_stream_decode(rc_ctx* ctx, const uint32_t* c, const uint32_t* cum,
                           uint32_t n_symbols, uint32_t total_freq, rc_stream_state* states,
                           const uint8_t* code, const uint64_t* code_off,
                           const uint64_t* code_len, uint8_t* syms, const uint64_t* sym_off,
                           uint32_t n_streams, uint32_t* flags) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || n_streams > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_symbols < 1 || n_symbols > 256) return RC_E_BAD_MODEL;
  if (n_streams == 0) return RC_OK;
  if (!c || !cum || !states || !code || !code_off || !code_len || !syms || !sym_off || !flags)
    return RC_E_ARG;
  Dev g(dev);
  rc_svc_yield_all_();
  hipLaunchKernelGGL(k_stream_decode, dim3((n_streams + RWG - 1) / RWG), dim3(RWG), 0, s, c,
                     cum, n_symbols, total_freq, states, code, code_off, code_len, syms, sym_off,
                     n_streams, flags);
  return hipGetLastError() == hipSuccess ? RC_OK : RC_E_DEVICE;
}

rc_status rc_stream_encode_host(rc_ctx* ctx, rc_stream_state* state, const uint32_t* triples,
                                uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                uint8_t* nbytes, uint32_t finish, uint32_t* flags_out) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || !state || !out_len || (n && !triples))
    return RC_E_ARG;
  const u64 need = RC_STREAM_MAX_BYTES(n, finish);
  *out_len = 0;
  if (out_cap < need || (need && !out)) {
    if (flags_out) *flags_out = RC_F_CAPACITY;
    return RC_E_CAPACITY;
  }
  // block: state | offsets (4 x u64) | out_len | flags | triples || nbytes | out
  const size_t o_off = 64, o_len = o_off + 32, o_fl = o_len + 16, o_tr = o_fl + 16;
  const size_t o_nb = o_tr + ((12 * n + 15) & ~15ull), o_out = o_nb + ((n + 15) & ~15ull);
  const size_t tail = (o_out + need - o_nb + 15) & ~15ull;
  if (svc_enabled(ctx) && o_nb + tail <= SVC_BLOCK) {  // a small call: through the stream service
    auto sv = svc_get(ctx);
    std::lock_guard<std::mutex> slk(sv->mu);
    rc_status err = RC_OK;
    if (svc_call(ctx, sv.get(), dev, [&](char* h, SvcBox* b) {
          memcpy(h, state, sizeof *state);
          const u64 offs[4] = {0, n, 0, need};
          memcpy(h + o_off, offs, sizeof offs);
          if (n) memcpy(h + o_tr, triples, 12 * n);
          b->op = SVC_ENCODE;
          b->finish = finish;
          b->in_bytes = o_nb;
          b->head_bytes = o_tr;
          b->tail_off = o_nb;
          b->tail_bytes = tail;
          const u64 o[8] = {o_off, o_len, o_fl, o_tr, o_nb, o_out, nbytes ? 1u : 0u, 0};
          memcpy(b->o, o, sizeof o);
        }, &err)) {
      if (err != RC_OK) return err;
      const char* h = (const char*)(sv->box + 1);
      rc_stream_state nst;
      memcpy(&nst, h, sizeof nst);
      u64 w;
      u32 fl;
      memcpy(&w, h + o_len, 8);
      memcpy(&fl, h + o_fl, 4);
      if (w > need || nst.n - state->n > n) return RC_E_DEVICE;
      if (w) memcpy(out, h + o_out, w);
      if (nbytes && n) memcpy(nbytes, h + o_nb, nst.n - state->n);
      *state = nst;
      *out_len = w;
      if (flags_out) *flags_out = fl;
      return fl ? RC_E_CHUNK : RC_OK;
    }
  }
  Dev g(dev);  // (the service path makes no HIP call but its wave's launch, guarded there)
  char* d = nullptr;
  std::shared_ptr<Stage> keep;
  std::unique_lock<std::mutex> lk;
  char* h = stage_acquire(ctx, o_out + need, &d, &keep, &lk);
  if (!h) return RC_E_DEVICE;
  memcpy(h, state, sizeof *state);
  const u64 offs[4] = {0, n, 0, need};  // sym_off[0..1], out_off[0..1]
  memcpy(h + o_off, offs, sizeof offs);
  if (n) memcpy(h + o_tr, triples, 12 * n);
  if (hipMemcpyAsync(d, h, o_nb, hipMemcpyHostToDevice, s) != hipSuccess) return RC_E_DEVICE;
  hipLaunchKernelGGL(k_stream_encode, dim3(1), dim3(RWG), 0, s, (rc_stream_state*)d,
                     (const u32*)(d + o_tr), (const u64*)(d + o_off), 1u, (uint8_t*)(d + o_out),
                     (const u64*)(d + o_off + 16), (u64*)(d + o_len),
                     nbytes ? (uint8_t*)(d + o_nb) : (uint8_t*)nullptr, finish,
                     (u32*)(d + o_fl));
  if (hipGetLastError() != hipSuccess) return RC_E_DEVICE;
  // state, out_len and flags, then the new bytes (and the counts, when asked for).  A large
  // call reads the state first and then only the w bytes written, not the 12n + 8 worst case.
  const bool two_phase = need > kTwoPhaseBytes;
  if (hipMemcpyAsync(h, d, o_tr, hipMemcpyDeviceToHost, s) != hipSuccess) return RC_E_DEVICE;
  if (!two_phase) {
    if ((nbytes && n &&
         hipMemcpyAsync(h + o_nb, d + o_nb, n, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (need && hipMemcpyAsync(h + o_out, d + o_out, need, hipMemcpyDeviceToHost, s) !=
                     hipSuccess))
      return RC_E_DEVICE;
  }
  if (hipStreamSynchronize(s) != hipSuccess) return RC_E_DEVICE;
  rc_stream_state nst;
  memcpy(&nst, h, sizeof nst);
  u64 w;
  u32 fl;
  memcpy(&w, h + o_len, 8);
  memcpy(&fl, h + o_fl, 4);
  if (w > need || nst.n - state->n > n) return RC_E_DEVICE;
  if (two_phase) {
    const u64 got = nst.n - state->n;
    if ((nbytes && got &&
         hipMemcpyAsync(h + o_nb, d + o_nb, got, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (w && hipMemcpyAsync(h + o_out, d + o_out, w, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess)
      return RC_E_DEVICE;
  }
  if (w) memcpy(out, h + o_out, w);
  if (nbytes && n) memcpy(nbytes, h + o_nb, nst.n - state->n);
  *state = nst;
  *out_len = w;
  if (flags_out) *flags_out = fl;
  return fl ? RC_E_CHUNK : RC_OK;
}

rc_status rc_stream_decode_host(rc_ctx* ctx, const uint32_t* c, const uint32_t* cum,
                                uint32_t n_symbols, uint32_t total_freq, rc_stream_state* state,
                                const uint8_t* code, uint64_t code_len, uint8_t* syms,
                                uint64_t n, uint32_t* flags_out) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || !state || !c || !cum || (n && !syms) ||
      (code_len && !code))
    return RC_E_ARG;
  if (n_symbols < 1 || n_symbols > 256) return RC_E_BAD_MODEL;
  // the window this call can read: Decoder::new's 8 bytes and <= 12 per symbol
  const u64 p0 = state->stage == 0 ? 0 : state->pos;
  if (p0 > code_len) return RC_E_ARG;
  const u64 wlen = std::min<u64>(code_len - p0, (state->stage == 0 ? 8 : 0) + 12 * n);
  // block: state | offsets: code_off, code_len, sym_off[0..1] | flags | c | cum | window || syms
  const size_t o_off = 64, o_fl = o_off + 32, o_c = o_fl + 16, o_cum = o_c + 1024;
  const size_t o_win = o_cum + 1024, o_sym = o_win + ((wlen + 15) & ~15ull);
  const size_t tail = (n + 15) & ~15ull;
  if (svc_enabled(ctx) && o_sym + tail <= SVC_BLOCK) {  // a small call: through the stream service
    auto sv = svc_get(ctx);
    std::lock_guard<std::mutex> slk(sv->mu);
    rc_status err = RC_OK;
    if (svc_call(ctx, sv.get(), dev, [&](char* h, SvcBox* b) {
          rc_stream_state rel = *state;
          rel.pos -= p0;  // the window starts at p0 (stage 0: at the stream start)
          memcpy(h, &rel, sizeof rel);
          const u64 offs[4] = {0, wlen, 0, n};
          memcpy(h + o_off, offs, sizeof offs);
          memcpy(h + o_c, c, 4ull * n_symbols);
          memcpy(h + o_cum, cum, 4ull * n_symbols);
          if (wlen) memcpy(h + o_win, code + p0, wlen);
          b->op = SVC_DECODE;
          b->n_alpha = n_symbols;
          b->total = total_freq;
          b->in_bytes = o_sym;
          b->head_bytes = o_c;
          b->tail_off = o_sym;
          b->tail_bytes = tail;
          const u64 o[8] = {o_off, o_fl, o_c, o_cum, o_win, o_sym, 0, 0};
          memcpy(b->o, o, sizeof o);
        }, &err)) {
      if (err != RC_OK) return err;
      const char* h = (const char*)(sv->box + 1);
      rc_stream_state nst;
      u32 fl;
      memcpy(&nst, h, sizeof nst);
      memcpy(&fl, h + o_fl, 4);
      const u64 got = nst.n - state->n;
      if (got > n) return RC_E_DEVICE;
      if (got) memcpy(syms, h + o_sym, got);
      nst.pos += p0;
      *state = nst;
      if (flags_out) *flags_out = fl;
      return fl ? RC_E_CHUNK : RC_OK;
    }
  }
  Dev g(dev);
  char* d = nullptr;
  std::shared_ptr<Stage> keep;
  std::unique_lock<std::mutex> lk;
  char* h = stage_acquire(ctx, o_sym + n, &d, &keep, &lk);
  if (!h) return RC_E_DEVICE;
  rc_stream_state rel = *state;
  rel.pos -= p0;  // the window starts at p0 (stage 0: at the stream start)
  memcpy(h, &rel, sizeof rel);
  const u64 offs[4] = {0, wlen, 0, n};
  memcpy(h + o_off, offs, sizeof offs);
  memcpy(h + o_c, c, 4ull * n_symbols);
  memcpy(h + o_cum, cum, 4ull * n_symbols);
  if (wlen) memcpy(h + o_win, code + p0, wlen);
  if (hipMemcpyAsync(d, h, o_win + wlen, hipMemcpyHostToDevice, s) != hipSuccess)
    return RC_E_DEVICE;
  hipLaunchKernelGGL(k_stream_decode, dim3(1), dim3(RWG), 0, s, (const u32*)(d + o_c),
                     (const u32*)(d + o_cum), n_symbols, total_freq, (rc_stream_state*)d,
                     (const uint8_t*)(d + o_win), (const u64*)(d + o_off),
                     (const u64*)(d + o_off + 8), (uint8_t*)(d + o_sym),
                     (const u64*)(d + o_off + 16), 1u, (u32*)(d + o_fl));
  if (hipGetLastError() != hipSuccess) return RC_E_DEVICE;
  if (hipMemcpyAsync(h, d, o_c, hipMemcpyDeviceToHost, s) != hipSuccess ||
      (n && hipMemcpyAsync(h + o_sym, d + o_sym, n, hipMemcpyDeviceToHost, s) != hipSuccess) ||
      hipStreamSynchronize(s) != hipSuccess)
    return RC_E_DEVICE;
  rc_stream_state nst;
  u32 fl;
  memcpy(&nst, h, sizeof nst);
  memcpy(&fl, h + o_fl, 4);
  const u64 got = nst.n - state->n;
  if (got > n) return RC_E_DEVICE;
  if (got) memcpy(syms, h + o_sym, got);
  nst.pos += p0;
  *state = nst;
  if (flags_out) *flags_out = fl;
  return fl ? RC_E_CHUNK : RC_OK;
}

// Internal (not in include/range_coder.h; tools/percall_native.cpp): the context's stream-service
// timings since the last call, then reset: out[0] calls; out[1..3] the wave's 10-ns ticks summed
// from seeing a request to its block in LDS, to the body done, to the results written back;
// out[4] the host's wait from publishing the request to seeing its ack, in ns, summed.
rc_status rc_svc_set_idle_ticks_(uint64_t ticks) {
  g_svc_idle_ticks.store(ticks, std::memory_order_relaxed);
  return RC_OK;
}

rc_status rc_svc_probe_(rc_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return RC_E_ARG;
  auto sv = svc_get(ctx);
  std::lock_guard<std::mutex> lk(sv->mu);
  for (int j = 0; j < 5; ++j) {
    out[j] = sv->probe[j];
    sv->probe[j] = 0;
  }
  return RC_OK;
}

// internal: free the context's staging block (called by rc_ctx_destroy)
void rc_resume_release_(const rc_ctx* ctx) {
  {  // the stream service: stop its wave, free the mailbox
    std::shared_ptr<Svc> sv;
    {
      std::lock_guard<std::mutex> lk(g_svc_mu);
      auto it = g_svcs.find(ctx);
      if (it != g_svcs.end()) {
        sv = std::move(it->second);
        g_svcs.erase(it);
      }
    }
    if (sv) {
      std::lock_guard<std::mutex> lk(sv->mu);
      svc_teardown(sv.get());
      __atomic_store_n(&sv->dead, true, __ATOMIC_RELEASE);  // (svc_get's fast path reads it)
    }
  }
  std::shared_ptr<Stage> st;
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    auto it = g_stages.find(ctx);
    if (it == g_stages.end()) return;
    st = std::move(it->second);
    g_stages.erase(it);
  }
  std::lock_guard<std::mutex> lk(st->mu);  // a call still inside the block finishes first
  if (st->host) (void)hipHostFree(st->host);
  if (st->dev) (void)hipFree(st->dev);
  st->host = st->dev = nullptr;
  st->cap = 0;
  st->dead = true;
}

}  // extern "C"
