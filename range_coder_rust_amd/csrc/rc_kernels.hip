// rc_kernels.hip — host side of the static-model coder (contexts, models, launches) and the
// synthetic workload generator.  The kernels: rc_encode.hip, rc_decode.inc (rc_static.h).
#include "rc_static.h"

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
#include <cmath>
#include <vector>

struct rc_ctx {
  int device;
  hipStream_t own;
  hipStream_t cur;
  uint8_t* inv;  // 64 KiB device scratch for rc_synth_fill's inverse CDF
  RcKnobs knobs;  // read from the environment once, here (rc_common.h)
};

// The only place the library reads its environment (tests/test_abi.py checks that no other
// source calls getenv): once per context, in rc_ctx_create.
RcKnobs rc_knobs_from_env() {
  auto str = [](const char* name) -> const char* {
    const char* e = getenv(name);
    return e && *e ? e : nullptr;
  };
  RcKnobs k;
  const char* e;
  k.prio = !((e = str("RC_PRIO")) && !strcmp(e, "off"));
  k.dec_pair = 0;
  if ((e = str("RC_DEC_PAIR"))) {
    const long x = strtol(e, nullptr, 10);
    k.dec_pair = x == 512 || x == 1024 ? (u32)x : 0u;
  }
  k.stream_service = !((e = str("RC_STREAM_SERVICE")) && e[0] == '0');
  k.stream_dma = (e = str("RC_STREAM_DMA")) && e[0] != '0';
  k.stream_direct = !((e = str("RC_STREAM_DIRECT")) && e[0] == '0');
  k.stream_batch_bytes = (e = str("RC_STREAM_BATCH_BYTES")) ? strtoull(e, nullptr, 0) : 0ull;
  k.hist_hot = !((e = str("RC_HIST_HOT")) && e[0] == '0');
  return k;
}

const RcKnobs& rc_ctx_knobs_(const rc_ctx* ctx) { return ctx->knobs; }

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

struct PinnedScratch {
  void* p = nullptr;
  size_t cap = 0;
  ~PinnedScratch() {
    if (p) (void)hipHostFree(p);
  }
};
thread_local PinnedScratch t_pinned;

}  // namespace

void* rc_pinned_scratch_(size_t bytes) {
  if (bytes > (1u << 20)) return nullptr;
  if (t_pinned.cap < bytes) {
    if (t_pinned.p) (void)hipHostFree(t_pinned.p);
    t_pinned.p = nullptr;
    t_pinned.cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1u << 16);
    if (hipHostMalloc(&t_pinned.p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    t_pinned.cap = cap;
  }
  return t_pinned.p;
}

// range_par_total's constants for `total` (DIV_POW2's shift, DIV_MAGIC's reciprocal and the
// small models' f64 1/total rounded up)
static void div_constants(ModelArgs& a, u32 total) {
  const bool pow2 = (total & (total - 1)) == 0;
  a.total = total;
  a.lg = pow2 ? (u32)__builtin_ctz(total) : 0u;
  a.magic = ~0ull / (u64)total;
  a.inv_up = 1.0 / (double)total;  // rounded up: inv_up * total >= 1 exactly
  if (std::fma(a.inv_up, (double)total, -1.0) < 0.0) a.inv_up = std::nextafter(a.inv_up, 2.0);
}

// range / total through the static coders' three range_par_total forms (rc_static.h), under
// the decoders' rounding mode (f32 toward zero, rc_decode.inc): out[3i] the small-model f64
// form, out[3i + 1] the 64 x 64 magic product, out[3i + 2] the power-of-two shift.  For
// rc_test_range_par_total_ (tests/test_gpu_div.py).
__global__ __launch_bounds__(64) void k_test_range_par_total(const u64* __restrict__ ranges,
                                                             const ModelArgs* __restrict__ ms,
                                                             u32 n, u64* __restrict__ out) {
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 2), 3");
  const u32 i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const ModelArgs m = ms[i];
  const u64 r = ranges[i];
  out[3 * i] = range_par_total<DIV_MAGIC, 1>(r, m);
  out[3 * i + 1] = range_par_total<DIV_MAGIC, 0>(r, m);
  out[3 * i + 2] = range_par_total<DIV_POW2, 0>(r, m);
}

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
  c->knobs = rc_knobs_from_env();
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
void rc_resume_release_(const rc_ctx* ctx);  // rc_resume.hip: the stream API's staging

rc_status rc_ctx_destroy(rc_ctx* ctx) {
  if (!ctx) return RC_E_ARG;
  DeviceGuard g(ctx->device);
  rc_stream_release_(ctx);
  rc_resume_release_(ctx);
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
  div_constants(a, total_freq);
  const bool pow2 = (total_freq & (total_freq - 1)) == 0;
  // bucket table of 2^bits buckets: s0 = symbol containing the bucket's first frequency, s1 =
  // the next symbol with c > 0 starting inside the bucket, split = its offset (0xFFFF: none);
  // padded to a power of two (the kernel masks the bucket index) with the last bucket, so
  // exactly 2^bits entries whenever total > 2048
  const u32 bl = bitlen(total_freq - 1);
  auto bucket_lut = [&](u32 bits, u32* shift_out) {
    const u32 shift = bl > bits ? bl - bits : 0u;
    const u32 nb = ((total_freq - 1) >> shift) + 1;
    std::vector<u32> lt(nb);
    u32 s = 0;
    for (u32 b = 0; b < nb; ++b) {
      const u64 f0 = (u64)b << shift;
      const u64 f1 = std::min<u64>((u64)(b + 1) << shift, total_freq);
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
      lt[b] = s | (s1 << 8) | (split << 16);
    }
    while (lt.size() & (lt.size() - 1)) lt.push_back(lt.back());
    *shift_out = shift;
    return lt;
  };
  a.lut_bits = total_freq <= 65536 ? SM_LUT_BITS : LUT_BITS;
  std::vector<u32> lut = bucket_lut(a.lut_bits, &a.lut_shift);
  a.lut_max = (u32)lut.size() - 1;
  if (total_freq > 2048 && lut.size() != (1u << a.lut_bits)) return RC_E_BAD_MODEL;  // unreachable

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
    // the flat model (raw bytes: configs[1]): cum[s] = s and c = 1 for every symbol
    bool flat = n_symbols == 256 && total_freq == 256;
    for (u32 i = 0; flat && i < 256; ++i) flat = c_freq[i] == 1;
    a.flat = flat ? 1u : 0u;
  }
  // pair buckets (k_decode_static LUT 3, rc_static.h): 2^15 < total <= 2^16, so buckets of 16
  // frequencies, and every c < 2^16 (16-bit fields).  Per bucket both candidates of its bucket
  // entry: s0 (holding the bucket's first frequency) and s1 (the next symbol with c > 0 that
  // starts inside the bucket; none: s1 = s0, so the choice between them does not matter).
  std::vector<u32> pair;
  u32 cmax = 0;
  for (u32 i = 0; i < n_symbols; ++i) cmax = std::max(cmax, c_freq[i]);
  if (!a.direct && total_freq > 32768 && total_freq <= 65536 && cmax < 65536) {
    pair.assign(PAIR_WORDS, 0);
    uint16_t* sp = (uint16_t*)pair.data();
    u32* ent = pair.data() + PAIR_S_WORDS;
    auto tcb = [&](u32 sym) {
      const float tcf = c_freq[sym] ? (float)total_freq / (float)c_freq[sym] : 0.0f;
      u32 b;
      memcpy(&b, &tcf, 4);
      return b;
    };
    u32 pshift = 0;
    const std::vector<u32> plut = bucket_lut(LUT_BITS, &pshift);  // 2^12 buckets of 16
    if (pshift != 4 || plut.size() != PAIR_BUCKETS) return RC_E_BAD_MODEL;  // unreachable
    for (u32 b = 0; b < PAIR_BUCKETS; ++b) {
      const u32 e = plut[b];  // (padded buckets repeat the last)
      const u32 s0 = e & 255u, s1 = (e >> 8) & 255u;  // (s1 = s0 where there is no split)
      sp[b] = (uint16_t)(s0 | s1 << 8);
      ent[4 * b + 0] = cum_freq[s0] | c_freq[s0] << 16;
      ent[4 * b + 1] = cum_freq[s1] | c_freq[s1] << 16;
      ent[4 * b + 2] = tcb(s0);
      ent[4 * b + 3] = tcb(s1);
    }
  }
  // small bucket models (the decoder's LUT 4, rc_static.h): 8-B buckets {16 s0 | 16 s1 << 16,
  // 0x4B400000 + cum[s1]} (s1's absolute cum; 0 without a split, where s1 = s0), at most
  // 2^SMB_LUT_BITS of them and at least 8 frequencies each, so the bucket's byte address is
  // (q >> la_shift) & la_mask with la_shift = lut_shift - 3 >= 0
  if (!a.direct && total_freq <= 65536) {
    const u32 bits = std::min<u32>(SMB_LUT_BITS, bl - 3);  // (total > 2048: bl >= 12)
    u32 shift = 0;
    const std::vector<u32> lt = bucket_lut(bits, &shift);
    if (shift < 3 || lt.size() != (1u << bits)) return RC_E_BAD_MODEL;  // unreachable
    std::vector<u32> l8(2 * lt.size());
    for (size_t b = 0; b < lt.size(); ++b) {
      const u32 e = lt[b], s0 = e & 255u, s1 = (e >> 8) & 255u, split = e >> 16;
      // (padded buckets repeat the last real one, (total - 1) >> shift)
      const u32 br = (u32)std::min<size_t>(b, (total_freq - 1) >> shift);
      // (as hint_floor's bits, 0x4B400000 + cum[s1]: the decoder compares the hint's raw bits)
      const u32 cum1 = 0x4B400000u + (split == 0xFFFFu ? 0u : (br << shift) + split);
      l8[2 * b] = 16 * s0 | (16 * s1) << 16;
      l8[2 * b + 1] = cum1;
    }
    a.lut_bits = bits;
    a.lut_shift = shift;
    a.la_shift = shift - 3;
    a.la_mask = ((u32)lt.size() - 1) << 3;
    a.la_magic = ldexpf(1.5f, 23 + (int)a.la_shift);
    a.lut_max = (u32)lt.size() - 1;
    lut.swap(l8);
  }
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const size_t tab_bytes = 256 * sizeof(uint2);
  const size_t lut_bytes = lut.size() * sizeof(u32);
  const size_t pair_bytes = pair.size() * sizeof(u32);
  void* d = nullptr;
  if (hipMalloc(&d, tab_bytes + lut_bytes + pair_bytes) != hipSuccess) return RC_E_DEVICE;
  if (hipMemcpy(d, tab.data(), tab_bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((char*)d + tab_bytes, lut.data(), lut_bytes, hipMemcpyHostToDevice) !=
          hipSuccess ||
      (pair_bytes && hipMemcpy((char*)d + tab_bytes + lut_bytes, pair.data(), pair_bytes,
                               hipMemcpyHostToDevice) != hipSuccess)) {
    (void)hipFree(d);
    return RC_E_DEVICE;
  }
  a.tab = (const uint2*)d;
  a.lut = (const u32*)((char*)d + tab_bytes);
  a.pair = pair_bytes ? (const u32*)((char*)d + tab_bytes + lut_bytes) : nullptr;
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
  // range_par_total (range_coder.rs:38-40) divides by a total that changes every symbol: the
  // kernels multiply by floor((2^64 - 1) / total) from this table (exact after one correction)
  std::vector<u64> magic(65536, 0);
  for (u32 t = 1; t < 65536; ++t) magic[t] = ~0ull / t;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  void* d = nullptr;
  if (hipMalloc(&d, magic.size() * sizeof(u64)) != hipSuccess) return RC_E_DEVICE;
  if (hipMemcpy(d, magic.data(), magic.size() * sizeof(u64), hipMemcpyHostToDevice) !=
      hipSuccess) {
    (void)hipFree(d);
    return RC_E_DEVICE;
  }
  rc_model* mm = new rc_model;
  memset(mm, 0, sizeof *mm);
  mm->kind = 1;
  mm->device = ctx->device;
  mm->dmem = d;
  mm->ap = AdaptParams{n_symbols, increment, limit, period - 1, (const u64*)d};
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
  rc_svc_yield_all_();
  if (m->kind == 1) {
    const hipError_t e = rc_adaptive_encode_launch(ctx->cur, m->ap, syms, sym_off, n_chunks,
                                                   out, out_off, out_len, flags);
    return e == hipSuccess ? RC_OK : device_error(e, "adaptive encode launch");
  }
  const bool sm = m->args.total >= 256 && m->args.total <= 65536;
  const int smv = sm ? (m->complete ? 2 : 1) : 0;
  const hipError_t e = rc_static_encode_launch(ctx->cur, ctx->knobs, m->args, m->div, smv, syms,
                                               sym_off, n_chunks, out, out_off, out_len, flags);
  return e == hipSuccess ? RC_OK : device_error(e, "encode launch");
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
  rc_svc_yield_all_();
  if (m->kind == 1) {
    const hipError_t e = rc_adaptive_decode_launch(ctx->cur, m->ap, code, code_off, code_len,
                                                   syms_out, sym_off, n_chunks, flags);
    return e == hipSuccess ? RC_OK : device_error(e, "adaptive decode launch");
  }
  const bool sm = m->args.total >= 256 && m->args.total <= 65536;
  const hipError_t e =
      m->div == DIV_POW2
          ? rc_static_decode_launch_pow2(ctx->cur, ctx->knobs, m->args, sm, code, code_off, code_len,
                                         syms_out, sym_off, n_chunks, flags)
          : rc_static_decode_launch_magic(ctx->cur, ctx->knobs, m->args, sm, code, code_off, code_len,
                                          syms_out, sym_off, n_chunks, flags);
  return e == hipSuccess ? RC_OK : device_error(e, "decode launch");
}

// rc_encode_host / rc_decode_host: the pipelined host path lives in rc_stream.hip

rc_status rc_synth_fill(rc_ctx* ctx, uint64_t seed, const uint8_t* inv_cdf_host,
                        uint8_t* syms_dev, uint64_t chunk_len, uint32_t n_chunks) {
  if (!ctx || !inv_cdf_host || !syms_dev) return RC_E_ARG;
  if (n_chunks == 0 || chunk_len == 0) return RC_OK;
  DeviceGuard g(ctx->device);
  if (!g.ok) return RC_E_DEVICE;
  const uint8_t* dinv = ctx->inv;
  void* pin = rc_pinned_scratch_(65536);
  if (!pin) return RC_E_DEVICE;
  memcpy(pin, inv_cdf_host, 65536);
  hipError_t e = hipMemcpyAsync(ctx->inv, pin, 65536, hipMemcpyHostToDevice, ctx->cur);
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
  // the pinned staging is reused by this thread's next call: wait for the copy
  if (st == RC_OK && (e = hipStreamSynchronize(ctx->cur)) != hipSuccess)
    return device_error(e, "rc_synth_fill sync");
  return st;
}

// Internal test hook (not in include/range_coder.h): range / total for n (range, total) pairs
// through k_test_range_par_total; out: 3 n results (host memory).  Synchronous.
rc_status rc_test_range_par_total_(rc_ctx* ctx, const uint64_t* ranges, const uint32_t* totals,
                                   uint32_t n, uint64_t* out) {
  if (!ctx || !ranges || !totals || !out || n == 0 || n > (1u << 20)) return RC_E_ARG;
  std::vector<ModelArgs> ms(n);
  for (u32 i = 0; i < n; ++i) {
    if (totals[i] == 0) return RC_E_BAD_MODEL;
    memset(&ms[i], 0, sizeof(ModelArgs));
    div_constants(ms[i], totals[i]);
  }
  DeviceGuard g(ctx->device);
  char* d = nullptr;
  const size_t b_r = 8ull * n, b_m = sizeof(ModelArgs) * n, b_o = 24ull * n;
  if (hipMalloc((void**)&d, b_r + b_m + b_o) != hipSuccess) return RC_E_DEVICE;
  rc_status st = RC_OK;
  if (hipMemcpy(d, ranges, b_r, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + b_r, ms.data(), b_m, hipMemcpyHostToDevice) != hipSuccess) {
    st = RC_E_DEVICE;
  } else {
    hipLaunchKernelGGL(k_test_range_par_total, dim3((n + 63) / 64), dim3(64), 0, ctx->cur,
                       (const u64*)d, (const ModelArgs*)(d + b_r), n, (u64*)(d + b_r + b_m));
    st = launch_status();
    if (st == RC_OK && (hipStreamSynchronize(ctx->cur) != hipSuccess ||
                        hipMemcpy(out, d + b_r + b_m, b_o, hipMemcpyDeviceToHost) != hipSuccess))
      st = RC_E_DEVICE;
  }
  (void)hipFree(d);
  return st;
}

}  // extern "C"
