// rc_model_build.hip — the step before encode: building the frequency table from the data, on
// the GPU.
//
// The reference builds its model on the CPU, one symbol at a time: FreqTable::new, then
// add_alphabet_freq per symbol (examples/sample_impl.rs:49-60), then calc_cum's exclusive scan
// (:61-69).  Here:
//   * k_histogram counts symbols of many chunks at once (per-chunk and/or batch histograms):
//     16-B loads, eight u16 LDS sub-histograms per wave;
//   * rc_quantize_counts turns counts into a (c, cum, total) table: exactly calc_cum's table
//     when no target is given, or a table scaled to a target total (e.g. 2^16, so the coder
//     takes its fast power-of-two path), deterministic and restated by the oracle;
//   * k_ideal_bits is the batched PModel::ideal_code_length (pmodel.rs:14-40): per chunk,
//     sum over its histogram of count * log2(total / c), in f64.
#include "rc_common.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define HWG 256  // k_ideal_bits

// k_histogram: chunk-stride workgroups of 4 waves; 16-B loads; LDS sub-histograms counted with
// ds_add_u32.  Measured (profiles/r03/ab/hist/): the LDS atomics' latency per
// wave binds, so the rate follows the resident waves per CU, and lanes of one instruction that
// hit one address serialise (a skewed model's hot symbols).  Hence small sub-histograms (4 KiB
// per wave: 32 waves per CU) with many copies: u16 counters, eight copies.
typedef __attribute__((address_space(3))) u32 hl_u32;

static __device__ __forceinline__ void hl_add(hl_u32* p, u32 v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Eight u16 sub-histograms per wave in the LDS of four u32 ones (4 KiB per wave, so 32 waves
// per CU as with four): lane L counts into copy L & 7; dword 8 (b & 127) + copy holds bins b
// (low half) and b + 128 (high half), so the hot low symbols of a skewed model never share a
// dword.  A u16 takes at most 8 lanes x HSEG_LANE symbols before the segment's readout.
#define HSEG_LANE 8176u  // symbols per lane per segment (16 x 511): 8 x (8176 + 2) < 2^16

// blocks [i0, i1) of the chunk (stride 256 from this thread's first) into the sub-histograms.
// HOT: symbol H (wave-uniform) is not added to LDS but counted by ballot into hc (an SGPR):
// the lanes of a skewed model's hottest symbol no longer serialise on its counters.
template <bool HOT>
static __device__ __forceinline__ void h8_blocks(const u32x4* v, u64 i0, u64 i1, u32 colb, u32 one,
                                                 u32 H, u32& hc) {
#pragma unroll 4
  for (u64 i = i0; i < i1; i += 256) {
    const u32x4 w = gload16(v + i);
    const u32 ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // per symbol: the dword's address as one bfe + one v_lshl_add_u32, the increment as
      // one SDWA shift reading byte j of x = 16 (b_j >> 7) per byte (asm: from C the
      // compiler re-derived each shift from the word with a shift, an and and an add)
      const u32 x = (ws[q] >> 3) & 0x10101010u;
      u32 a[4], y[4];
#define H8_SYM(j)                                                                               \
  asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(a[j]) : "v"(__builtin_amdgcn_ubfe(ws[q], 8 * j, 7)), \
      "v"(colb));                                                                               \
  asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #j    \
      " src1_sel:DWORD"                                                                         \
      : "=v"(y[j]) : "v"(x), "v"(one));                                                        \
  if (HOT) {                                                                                    \
    const bool h = __builtin_amdgcn_ubfe(ws[q], 8 * j, 8) == H;                                 \
    hc += (u32)__builtin_popcountll(__builtin_amdgcn_ballot_w64(h));                            \
    if (!h) hl_add((hl_u32*)(uintptr_t)a[j], y[j]);                                             \
  } else {                                                                                      \
    hl_add((hl_u32*)(uintptr_t)a[j], y[j]);                                                     \
  }
      H8_SYM(0) H8_SYM(1) H8_SYM(2) H8_SYM(3)
#undef H8_SYM
    }
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_histogram(
    const uint8_t* __restrict__ syms, const u64* __restrict__ sym_off, u32 n_chunks,
    u32* __restrict__ chunk_hist, u64* __restrict__ hist, u32 hot_ok) {
  __shared__ u32 sh[4 * 1024];
  __shared__ u32 s_hot[4];  // per wave: the segment's ballot count of the hot symbol
  __shared__ u32 s_key[4];  // per wave: max of (count << 8 | bin) of the last chunk
  const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LDS byte address of this lane's copy; a VGPR holding 1 (the SDWA shift's operand)
  const u32 colb = (u32)(uintptr_t)(hl_u32*)(sh + wave * 1024 + (lane & 7));
  u32 one = 1;
  asm volatile("" : "+v"(one));
  RC_VGPR_FLOOR_64();
  u64 acc = 0;  // bin tid over this WG's chunks
  for (u32 j = tid; j < 4 * 1024; j += 256) sh[j] = 0;
  bool have_key = false;
  for (u32 k = blockIdx.x; k < n_chunks; k += gridDim.x) {
    const u64 s0 = sym_off[k], n = sym_off[k + 1] - s0;
    const uint8_t* p = syms + s0;
    u64 head = (16 - ((uintptr_t)p & 15)) & 15;
    if (head > n) head = n;
    const u64 nv = (n - head) >> 4;
    const u32x4* v = reinterpret_cast<const u32x4*>(p + head);
    u32 cnt = 0;
    // segments of 256 * HSEG_LANE / 16 blocks: every lane adds <= HSEG_LANE symbols per segment
    const u64 seg = 256ull * HSEG_LANE / 16;
    u32 H = 256, key = 0;
    for (u64 b0 = 0; b0 == 0 || b0 < nv; b0 += seg) {
      __syncthreads();
      if (b0 == 0) {
        // the hot symbol: the previous chunk's most frequent one, if it held >= 1/8 of it
        if (have_key && hot_ok) {
          key = max(max(s_key[0], s_key[1]), max(s_key[2], s_key[3]));
          key = __builtin_amdgcn_readfirstlane(key);
        }
        H = key >> 8 ? (key & 255u) : 256u;
        if (tid < head) {
          const u32 b = p[tid];
          atomicAdd(&sh[wave * 1024 + (b & 127) * 8 + (lane & 7)], 1u << (16 * (b >> 7)));
        }
        const u64 t0 = head + (nv << 4);
        if (t0 + tid < n) {  // < 16 tail symbols
          const u32 b = p[t0 + tid];
          atomicAdd(&sh[wave * 1024 + (b & 127) * 8 + (lane & 7)], 1u << (16 * (b >> 7)));
        }
      }
      const u64 b1 = b0 + seg < nv ? b0 + seg : nv;
      u32 hc = 0;
      if (H < 256) h8_blocks<true>(v, b0 + tid, b1, colb, one, H, hc);
      else h8_blocks<false>(v, b0 + tid, b1, colb, one, H, hc);
      if (lane == 0) s_hot[wave] = hc;
      __syncthreads();
      // bin tid: the half (tid >> 7) of dwords 8 (tid & 127) + c of the four waves
#pragma unroll
      for (u32 w = 0; w < 4; ++w) {
        u32x4* r = reinterpret_cast<u32x4*>(sh + w * 1024 + (tid & 127) * 8);
#pragma unroll
        for (u32 h = 0; h < 2; ++h) {
          const u32x4 x = r[h];
          const u32 sft = 16 * (tid >> 7);
          cnt += ((x.x >> sft) & 0xFFFFu) + ((x.y >> sft) & 0xFFFFu) + ((x.z >> sft) & 0xFFFFu) +
                 ((x.w >> sft) & 0xFFFFu);
        }
      }
      if (tid == H) cnt += s_hot[0] + s_hot[1] + s_hot[2] + s_hot[3];
      __syncthreads();
      for (u32 j = tid; j < 4 * 1024; j += 256) sh[j] = 0;
    }
    if (chunk_hist) chunk_hist[(u64)k * 256 + tid] = cnt;
    acc += cnt;
    // this chunk's most frequent symbol, for the next one (read after the next barrier); a
    // bin below 1/8 of the chunk gives key 0 (no hot symbol)
    u32 kv = (u64)cnt * 8 >= n && n >= 4096 ? (min(cnt, 0xFFFFFFu) << 8) | tid : 0u;
#pragma unroll
    for (int o = 32; o; o >>= 1) kv = max(kv, (u32)__shfl_xor((int)kv, o));
    if (lane == 0) s_key[wave] = kv;
    have_key = true;
  }
  if (hist && acc) atomicAdd(reinterpret_cast<unsigned long long*>(hist + tid), (unsigned long long)acc);
}

// per chunk: bits = sum_i hist[i] * icl[i] in f64 (icl[i] = +inf for c_i == 0: the reference's
// ideal_code_length returns Err there, pmodel.rs:16-18).  One wave per chunk: lane L reads bins
// 4L .. 4L+3 of the row as one 16-B load (the wave reads the whole 1-KiB row at once) and holds
// their icl in registers for every chunk; the 64 partial sums are added by a butterfly.  Empty
// bins are skipped (0 * inf would be NaN).
__global__ __launch_bounds__(HWG) void k_ideal_bits(const double* __restrict__ icl,
                                                    const u32* __restrict__ chunk_hist,
                                                    u32 n_chunks, double* __restrict__ bits) {
  const u32 lane = threadIdx.x & 63;
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  RC_VGPR_FLOOR_48();
  const double i0 = icl[4 * lane], i1 = icl[4 * lane + 1], i2 = icl[4 * lane + 2],
               i3 = icl[4 * lane + 3];
  const u32 nw = gridDim.x * (HWG / 64);
  for (u32 k = blockIdx.x * (HWG / 64) + wave; k < n_chunks; k += nw) {
    const u32x4 h = gload16(reinterpret_cast<const u32x4*>(chunk_hist + (u64)k * 256) + lane);
    double acc = 0.0;
    if (h.x) acc = fma((double)h.x, i0, acc);
    if (h.y) acc = fma((double)h.y, i1, acc);
    if (h.z) acc = fma((double)h.z, i2, acc);
    if (h.w) acc = fma((double)h.w, i3, acc);
#pragma unroll
    for (int o = 32; o; o >>= 1) {
      const u64 v = (u64)__double_as_longlong(acc);
      const u64 y = ((u64)(u32)__shfl_xor((int)hi32(v), o) << 32) | (u32)__shfl_xor((int)(u32)v, o);
      acc += __longlong_as_double((long long)y);
    }
    if (lane == 0) bits[k] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct rc_ctx;  // rc_kernels.hip
extern "C" {
rc_status rc_ctx_stream_(rc_ctx* ctx, hipStream_t* s, int* device);  // rc_kernels.hip
}

namespace {
struct DevSet {
  int prev = -1;
  explicit DevSet(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevSet() {
    int now = -1;
    if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
  }
};
}  // namespace

extern "C" {

rc_status rc_histogram(rc_ctx* ctx, const uint8_t* syms, const uint64_t* sym_off,
                       uint32_t n_chunks, uint32_t* chunk_hist, uint64_t* hist) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0 || (!chunk_hist && !hist)) return RC_OK;
  if (!syms || !sym_off) return RC_E_ARG;
  DevSet g(dev);
  rc_svc_yield_all_();
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return RC_E_DEVICE;
  // 16 KiB LDS per workgroup: 8 workgroups (32 waves) per CU
  const u32 grid = std::min<u32>(n_chunks, (u32)cus * 8);
  // RC_HIST_HOT=0 (in the environment of rc_ctx_create) turns the ballot-counted hot symbol
  // off (measurements)
  hipLaunchKernelGGL(k_histogram, dim3(grid), dim3(256), 0, s, syms, sym_off, n_chunks,
                     chunk_hist, hist, (u32)rc_ctx_knobs_(ctx).hist_hot);
  return hipGetLastError() == hipSuccess ? RC_OK : RC_E_DEVICE;
}

rc_status rc_quantize_counts(const uint64_t* counts, uint32_t n_symbols, uint64_t target_total,
                             uint32_t qflags, uint32_t* c_out, uint32_t* cum_out,
                             uint32_t* total_out) {
  if (!counts || !c_out || !cum_out || !total_out || n_symbols < 1 || n_symbols > 256)
    return RC_E_ARG;
  const bool all = (qflags & RC_Q_ALL_SYMBOLS) != 0;
  std::vector<u64> c(n_symbols);
  unsigned __int128 N = 0;
  for (u32 i = 0; i < n_symbols; ++i) N += counts[i];
  if (target_total == 0) {  // exact FreqTable: c = counts, total = sum (sample_impl.rs:58-69)
    for (u32 i = 0; i < n_symbols; ++i) c[i] = counts[i] + ((all && counts[i] == 0) ? 1u : 0u);
  } else {
    u32 need = 0;
    for (u32 i = 0; i < n_symbols; ++i) need += (all || counts[i] > 0) ? 1u : 0u;
    if (N == 0) {
      if (!all) return RC_E_BAD_MODEL;  // nothing to model
      need = n_symbols;
    }
    if (target_total < need || target_total > 0xFFFFFFFFull) return RC_E_BAD_MODEL;
    // c_i = max(1, round(counts_i * T / N)) for modelled symbols (half rounds up)
    u64 sum = 0;
    for (u32 i = 0; i < n_symbols; ++i) {
      if (N == 0) {
        c[i] = 1;
      } else if (counts[i] == 0 && !all) {
        c[i] = 0;
      } else {
        const unsigned __int128 q = ((unsigned __int128)counts[i] * target_total + N / 2) / N;
        c[i] = q < 1 ? 1 : (u64)q;
      }
      sum += c[i];
    }
    // fold the difference: a deficit goes to the largest entry (lowest index on ties); an
    // excess is taken from the largest entries first, never below 1
    if (sum < target_total) {
      u32 m = 0;
      for (u32 i = 1; i < n_symbols; ++i)
        if (c[i] > c[m]) m = i;
      c[m] += target_total - sum;
    } else if (sum > target_total) {
      u64 excess = sum - target_total;
      std::vector<u32> order(n_symbols);
      for (u32 i = 0; i < n_symbols; ++i) order[i] = i;
      std::stable_sort(order.begin(), order.end(), [&](u32 a, u32 b) { return c[a] > c[b]; });
      for (u32 j = 0; j < n_symbols && excess; ++j) {
        const u32 i = order[j];
        if (c[i] <= 1) break;
        const u64 take = std::min<u64>(excess, c[i] - 1);
        c[i] -= take;
        excess -= take;
      }
      if (excess) return RC_E_BAD_MODEL;  // unreachable: target >= number of entries
    }
  }
  u64 acc = 0;
  for (u32 i = 0; i < n_symbols; ++i) {
    cum_out[i] = (u32)acc;
    c_out[i] = (u32)c[i];
    acc += c[i];
    if (acc > 0xFFFFFFFFull) return RC_E_BAD_MODEL;  // calc_cum's u32 total would overflow
  }
  if (acc == 0) return RC_E_BAD_MODEL;
  *total_out = (u32)acc;
  return RC_OK;
}

rc_status rc_ideal_bits(rc_ctx* ctx, const uint32_t* c_host, uint32_t n_symbols,
                        uint32_t total_freq, const uint32_t* chunk_hist, uint32_t n_chunks,
                        double* bits) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || !c_host || n_symbols < 1 || n_symbols > 256 ||
      total_freq < 1 || n_chunks > RC_MAX_CHUNKS)
    return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!chunk_hist || !bits) return RC_E_ARG;
  // PModel::ideal_code_length (pmodel.rs:14-40): (ln total - ln c) / ln 2; symbols outside the
  // alphabet or with c == 0 have no code length (+inf here)
  double icl[256];
  const double lt = log((double)total_freq);
  for (u32 i = 0; i < 256; ++i)
    icl[i] = (i < n_symbols && c_host[i] > 0) ? (lt - log((double)c_host[i])) / M_LN2 : INFINITY;
  DevSet g(dev);
  double* d = nullptr;
  if (hipMallocAsync((void**)&d, sizeof icl, s) != hipSuccess) return RC_E_DEVICE;
  void* pin = rc_pinned_scratch_(sizeof icl);
  if (!pin) {
    (void)hipFreeAsync(d, s);
    return RC_E_DEVICE;
  }
  memcpy(pin, icl, sizeof icl);
  if (hipMemcpyAsync(d, pin, sizeof icl, hipMemcpyHostToDevice, s) != hipSuccess) {
    (void)hipFreeAsync(d, s);
    return RC_E_DEVICE;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  // one wave per chunk, waves striding over the chunks: 8 workgroups (32 waves) per CU
  const u32 grid = std::min<u32>((n_chunks + HWG / 64 - 1) / (HWG / 64), (u32)cus * 8);
  hipLaunchKernelGGL(k_ideal_bits, dim3(grid), dim3(HWG), 0, s, d, chunk_hist, n_chunks, bits);
  const bool ok = hipGetLastError() == hipSuccess;
  // the pinned staging is reused by this thread's next call: wait for the copy
  const bool fr = hipFreeAsync(d, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  return ok && fr ? RC_OK : RC_E_DEVICE;
}

}  // extern "C"
