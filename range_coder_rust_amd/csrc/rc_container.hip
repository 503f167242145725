// rc_container.hip — the chunked container ("RCB1"): framing that makes a batch of coded chunks
// a self-describing codec.
//
// The reference's stream carries neither its symbol count nor its model: the decoder gets the
// count out of band (examples/sample_impl.rs:113-120) and the table from the caller
// (decoder.rs:38).  The container stores both, plus a per-chunk index, in front of the
// concatenated chunk streams.  Layout (little-endian, include/range_coder.h):
//   [0, 64)              header (rc_container_header)
//   [64, index_off)      model table: static -> n_symbols x u32 c_freq (cum = calc_cum), padded
//   [index_off, +16n)    per chunk {u64 symbol count, u64 code length}
//   [payload_off, end)   chunk k's code at payload_off + sum_{j<k} pad16(len_j), zero padded
// Every chunk stream starts 16-B aligned, so packing is a 16-B vector copy from the encoder's
// slots and the decoder reads the payload in place.
//
// GPU work: exclusive scans of the padded lengths / symbol counts (k_scan_*), the payload
// gather (k_pack_payload, HBM-bound), index writes and reads.
#include "rc_common.h"

#include <string.h>

#include <algorithm>

#define SWG 256
#define SPER 4                  // items per thread in a scan block
#define SBLK (SWG * SPER)       // items per scan block

static __device__ __forceinline__ u64 pad16(u64 v) { return (v + 15) & ~15ull; }

enum { SCAN_SRC_PLAIN = 0, SCAN_SRC_PAD16 = 1, SCAN_SRC_STRIDE2_PAD16 = 2, SCAN_SRC_STRIDE2 = 3,
       SCAN_SRC_DIFF = 4 };

// item i of the scan input: PLAIN v[i]; PAD16 pad16(v[i]); STRIDE2(_PAD16) (pad16)(v[2i + sel])
// (an index entry field); DIFF v[i+1] - v[i] (chunk sizes from offsets)
static __device__ __forceinline__ u64 scan_item(const u64* v, u32 i, int src, u32 sel) {
  switch (src) {
    case SCAN_SRC_PAD16: return pad16(v[i]);
    case SCAN_SRC_STRIDE2_PAD16: return pad16(v[2 * (u64)i + sel]);
    case SCAN_SRC_STRIDE2: return v[2 * (u64)i + sel];
    case SCAN_SRC_DIFF: return v[i + 1] - v[i];
    default: return v[i];
  }
}

// exclusive scan of one SBLK block; out[i] = base + prefix within the block, block total to
// sums[blockIdx] (pass 1) or, with add != nullptr, add[blockIdx] folded in (pass 3)
__global__ __launch_bounds__(SWG) void k_scan_block(const u64* __restrict__ v, u32 n, int src,
                                                    u32 sel, u64 base, u64* __restrict__ out,
                                                    u64* __restrict__ sums,
                                                    const u64* __restrict__ add) {
  __shared__ u64 s_w[SWG / 64];
  const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u32 i0 = blockIdx.x * SBLK + tid * SPER;
  RC_VGPR_FLOOR_48();
  u64 x[SPER], t = 0;
#pragma unroll
  for (int j = 0; j < SPER; ++j) {
    x[j] = (i0 + j < n) ? scan_item(v, i0 + j, src, sel) : 0ull;
    t += x[j];
  }
  // inclusive wave scan of the thread totals
  u64 inc = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y = ((u64)(u32)__shfl_up((int)hi32(inc), o) << 32) | (u32)__shfl_up((int)(u32)inc, o);
    if (lane >= (u32)o) inc += y;
  }
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  u64 wbase = 0;
  for (u32 w = 0; w < wave; ++w) wbase += s_w[w];
  if (sums) {  // pass 1: block totals only
    if (tid == SWG - 1) sums[blockIdx.x] = wbase + inc;
    return;
  }
  // single block, or pass 3 with the block's exclusive offset in add[]
  u64 run = base + (add ? add[blockIdx.x] : 0ull) + wbase + inc - t;
#pragma unroll
  for (int j = 0; j < SPER; ++j) {
    if (i0 + j < n) out[i0 + j] = run;
    run += x[j];
  }
  if (i0 < n && n <= i0 + SPER) out[n] = run;  // the total, by the thread of the last item
}

// the block sums of pass 1 -> their exclusive prefix (one WG, sequential over tiles)
__global__ __launch_bounds__(SWG) void k_scan_sums(u64* __restrict__ sums, u32 nb) {
  __shared__ u64 s[SWG];
  __shared__ u64 carry;
  const u32 tid = threadIdx.x;
  RC_VGPR_FLOOR_32();
  if (tid == 0) carry = 0;
  for (u32 b0 = 0; b0 < nb; b0 += SWG) {
    __syncthreads();
    const u64 v = (b0 + tid < nb) ? sums[b0 + tid] : 0ull;
    s[tid] = v;
    __syncthreads();
    for (u32 o = 1; o < SWG; o <<= 1) {  // Hillis-Steele inclusive scan in LDS
      const u64 y = tid >= o ? s[tid - o] : 0ull;
      __syncthreads();
      s[tid] += y;
      __syncthreads();
    }
    const u64 c = carry;
    if (b0 + tid < nb) sums[b0 + tid] = c + s[tid] - v;
    __syncthreads();
    if (tid == SWG - 1) carry = c + s[tid];
  }
}

// Exclusive scan (n items -> out[0..n], out[n] = base + total), stream-ordered.  tmp: >=
// ceil(n / SBLK) u64 of scratch.
static hipError_t device_scan(hipStream_t s, const u64* v, u32 n, int src, u32 sel, u64 base,
                              u64* out, u64* tmp) {
  const u32 nb = (n + SBLK - 1) / SBLK;
  if (nb <= 1) {
    hipLaunchKernelGGL(k_scan_block, dim3(1), dim3(SWG), 0, s, v, n, src, sel, base, out,
                       (u64*)nullptr, (const u64*)nullptr);
    if (n == 0) {
      u64 z = base;  // empty: out[0] = base
      return hipMemcpyAsync(out, &z, 8, hipMemcpyHostToDevice, s) == hipSuccess &&
                     hipStreamSynchronize(s) == hipSuccess
                 ? hipSuccess
                 : hipErrorUnknown;
    }
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_scan_block, dim3(nb), dim3(SWG), 0, s, v, n, src, sel, base, out, tmp,
                     (const u64*)nullptr);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SWG), 0, s, tmp, nb);
  hipLaunchKernelGGL(k_scan_block, dim3(nb), dim3(SWG), 0, s, v, n, src, sel, base, out,
                     (u64*)nullptr, (const u64*)tmp);
  return hipGetLastError();
}

// payload gather: chunk k's code (len[k] bytes of its encoder slot) -> dst + doff[k], zero
// padded to 16 B; index entry k = {symbol count, code length}.  One wave per chunk (SWG / 64
// chunks per workgroup), grid-stride over the chunks.
__global__ __launch_bounds__(SWG) void k_pack_payload(const uint8_t* __restrict__ slots,
                                                      const u64* __restrict__ slot_off,
                                                      const u64* __restrict__ len,
                                                      const u64* __restrict__ sym_off,
                                                      u32 n_chunks, uint8_t* __restrict__ dst,
                                                      const u64* __restrict__ doff,
                                                      u64* __restrict__ index) {
  // one wave per chunk (four chunks per workgroup in flight, no barriers): a chunk's last
  // partial round of 16-B granules idles fewer lanes, and one chunk's offset loads overlap the
  // other waves' copies
  const u32 tid = threadIdx.x & 63;
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  RC_VGPR_FLOOR_32();
  for (u32 k = blockIdx.x * (SWG / 64) + wave; k < n_chunks; k += gridDim.x * (SWG / 64)) {
    const u64 l = len[k];
    const uint8_t* sp = slots + slot_off[k];
    uint8_t* dp = dst + doff[k];  // 16-B aligned
    if (tid == 0) {
      index[2 * (u64)k] = sym_off[k + 1] - sym_off[k];
      index[2 * (u64)k + 1] = l;
    }
    const u64 ng = pad16(l) >> 4;
    if (((uintptr_t)sp & 15) == 0) {
      const u64 full = l >> 4;  // whole granules inside the stream
      const u32x4* src = reinterpret_cast<const u32x4*>(sp);
      u64 g = tid;
      for (; g + 192 < full; g += 256) {  // four granules per lane in flight
        const u32x4 a = gload16(src + g), b = gload16(src + g + 64), c = gload16(src + g + 128),
                    d = gload16(src + g + 192);
        gstore128(dp + 16 * g, a);
        gstore128(dp + 16 * (g + 64), b);
        gstore128(dp + 16 * (g + 128), c);
        gstore128(dp + 16 * (g + 192), d);
      }
      for (; g < full; g += 64) gstore128(dp + 16 * g, gload16(src + g));
      if (tid == 0 && full < ng) {  // last partial granule: stream bytes, then zeros
        u32 w[4] = {0, 0, 0, 0};
        for (u32 j = 0; j < (u32)(l & 15); ++j) w[j >> 2] |= (u32)sp[16 * full + j] << (8 * (j & 3));
        u32x4 v;
        v.x = w[0];
        v.y = w[1];
        v.z = w[2];
        v.w = w[3];
        gstore128(dp + 16 * full, v);
      }
    } else {  // misaligned slot: dword-assembled granules
      for (u64 g = tid; g < ng; g += 64) {
        u32 w[4] = {0, 0, 0, 0};
        for (u32 j = 0; j < 16; ++j) {
          const u64 p = 16 * g + j;
          if (p < l) w[j >> 2] |= (u32)sp[p] << (8 * (j & 3));
        }
        u32x4 v;
        v.x = w[0];
        v.y = w[1];
        v.z = w[2];
        v.w = w[3];
        gstore128(dp + 16 * g, v);
      }
    }
  }
}

// index -> decode arguments: code_len[k] = index[2k+1]; entries with absurd sizes raise *bad
__global__ __launch_bounds__(SWG) void k_unpack_index(const u64* __restrict__ index, u32 n,
                                                      u64* __restrict__ code_len,
                                                      u32* __restrict__ bad) {
  const u32 k = blockIdx.x * SWG + threadIdx.x;
  RC_VGPR_FLOOR_32();
  if (k >= n) return;
  const u64 sc = index[2 * (u64)k], l = index[2 * (u64)k + 1];
  code_len[k] = l;
  if (sc > (1ull << 48) || l > (1ull << 48)) atomicOr(bad, 1u);
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct rc_ctx;
struct rc_model;
extern "C" {
rc_status rc_ctx_stream_(rc_ctx* ctx, hipStream_t* s, int* device);
rc_status rc_model_describe_(const rc_model* m, int* kind, int* device, uint32_t* n_symbols,
                             uint32_t* total, const uint32_t** c_host, uint32_t* increment,
                             uint32_t* limit, uint32_t* period);
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

u64 hpad16(u64 v) { return (v + 15) & ~15ull; }

struct Scratch {
  void* p = nullptr;
  hipStream_t s;
  explicit Scratch(hipStream_t st) : s(st) {}
  bool alloc(size_t n) { return hipMallocAsync(&p, n ? n : 16, s) == hipSuccess; }
  ~Scratch() {
    if (p) (void)hipFreeAsync(p, s);
  }
};

void put32(uint8_t* p, u32 v) { memcpy(p, &v, 4); }
void put64(uint8_t* p, u64 v) { memcpy(p, &v, 8); }
u32 get32(const uint8_t* p) {
  u32 v;
  memcpy(&v, p, 4);
  return v;
}
u64 get64(const uint8_t* p) {
  u64 v;
  memcpy(&v, p, 8);
  return v;
}
}  // namespace

extern "C" {

rc_status rc_container_info_parse(const uint8_t* head, uint64_t head_len, rc_container_info* info) {
  if (!head || !info) return RC_E_ARG;
  if (head_len < RC_CONTAINER_HEADER_BYTES) return RC_E_BAD_CONTAINER;
  if (memcmp(head, "RCB1", 4) != 0) return RC_E_BAD_CONTAINER;
  rc_container_info in;
  memset(&in, 0, sizeof in);
  const u32 vh = get32(head + 4);
  in.version = vh & 0xFFFF;
  if (in.version != 1 || (vh >> 16) != RC_CONTAINER_HEADER_BYTES) return RC_E_BAD_CONTAINER;
  in.kind = get32(head + 8);
  in.n_symbols = get32(head + 12);
  in.total_freq = get32(head + 16);
  in.increment = get32(head + 20);
  in.limit = get32(head + 24);
  in.period = get32(head + 28);
  in.n_chunks = get64(head + 32);
  in.n_syms = get64(head + 40);
  in.payload_bytes = get64(head + 48);
  if (in.kind > 1 || in.n_symbols < 1 || in.n_symbols > 256 || in.n_chunks > RC_MAX_CHUNKS)
    return RC_E_BAD_CONTAINER;
  in.table_off = RC_CONTAINER_HEADER_BYTES;
  in.index_off = in.table_off + (in.kind == 0 ? hpad16(4ull * in.n_symbols) : 0);
  in.payload_off = in.index_off + 16 * in.n_chunks;
  in.container_bytes = in.payload_off + in.payload_bytes;
  if (in.payload_bytes & 15 || in.payload_bytes > (1ull << 56)) return RC_E_BAD_CONTAINER;
  *info = in;
  return RC_OK;
}

rc_status rc_container_pack(rc_ctx* ctx, const rc_model* m, const uint8_t* slots_dev,
                            const uint64_t* slot_off_dev, const uint64_t* code_len_dev,
                            const uint64_t* sym_off_dev, uint32_t n_chunks, uint8_t* dst_dev,
                            uint64_t dst_cap, uint64_t* dst_len_host) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || !m || !dst_len_host || n_chunks > RC_MAX_CHUNKS)
    return RC_E_ARG;
  if (n_chunks && (!slots_dev || !slot_off_dev || !code_len_dev || !sym_off_dev)) return RC_E_ARG;
  int kind, mdev;
  u32 nsym, total, inc, lim, per;
  const u32* c_host;
  if (rc_model_describe_(m, &kind, &mdev, &nsym, &total, &c_host, &inc, &lim, &per) != RC_OK ||
      mdev != dev)
    return RC_E_ARG;
  DevSet g(dev);
  rc_svc_yield_all_();
  const u64 index_off = RC_CONTAINER_HEADER_BYTES + (kind == 0 ? hpad16(4ull * nsym) : 0);
  const u64 payload_off = index_off + 16ull * n_chunks;
  // scans: dst offsets of the padded streams, and the symbol total
  const u32 nb = (n_chunks + SBLK - 1) / SBLK;
  Scratch sc(s);
  if (!sc.alloc(8ull * (n_chunks + 1) * 2 + 8ull * (nb + 1))) return RC_E_DEVICE;
  u64* doff = (u64*)sc.p;
  u64* soff = doff + (n_chunks + 1);
  u64* tmp = soff + (n_chunks + 1);
  hipError_t e = device_scan(s, code_len_dev, n_chunks, SCAN_SRC_PAD16, 0, payload_off, doff, tmp);
  if (e == hipSuccess) e = device_scan(s, sym_off_dev, n_chunks, SCAN_SRC_DIFF, 0, 0, soff, tmp);
  // small read-backs and the header go through pinned memory: [0, 16) ends, [64, ...) header
  char* pin = (char*)rc_pinned_scratch_(64 + RC_CONTAINER_HEADER_BYTES + 1024 + 16);
  if (!pin) return RC_E_DEVICE;
  u64* ends = (u64*)pin;
  ends[0] = payload_off;
  ends[1] = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&ends[0], doff + n_chunks, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&ends[1], soff + n_chunks, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return RC_E_DEVICE;
  const u64 total_bytes = ends[0];
  *dst_len_host = total_bytes;
  if (!dst_dev || total_bytes > dst_cap) return RC_E_CAPACITY;
  // header + table (host-built, one copy)
  uint8_t head[RC_CONTAINER_HEADER_BYTES + 1024 + 16];
  memset(head, 0, sizeof head);
  memcpy(head, "RCB1", 4);
  put32(head + 4, 1u | ((u32)RC_CONTAINER_HEADER_BYTES << 16));
  put32(head + 8, (u32)kind);
  put32(head + 12, nsym);
  put32(head + 16, kind == 0 ? total : 0u);
  put32(head + 20, kind == 1 ? inc : 0u);
  put32(head + 24, kind == 1 ? lim : 0u);
  put32(head + 28, kind == 1 ? per : 0u);
  put64(head + 32, n_chunks);
  put64(head + 40, ends[1]);
  put64(head + 48, total_bytes - payload_off);
  if (kind == 0)
    for (u32 i = 0; i < nsym; ++i) put32(head + RC_CONTAINER_HEADER_BYTES + 4 * i, c_host[i]);
  memcpy(pin + 64, head, index_off);
  if (hipMemcpyAsync(dst_dev, pin + 64, index_off, hipMemcpyHostToDevice, s) != hipSuccess)
    return RC_E_DEVICE;
  if (n_chunks) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const u32 grid = std::min<u32>((n_chunks + SWG / 64 - 1) / (SWG / 64), (u32)std::max(cus, 1) * 16);
    hipLaunchKernelGGL(k_pack_payload, dim3(grid), dim3(SWG), 0, s, slots_dev, slot_off_dev,
                       code_len_dev, sym_off_dev, n_chunks, dst_dev, doff,
                       reinterpret_cast<u64*>(dst_dev + index_off));
    if (hipGetLastError() != hipSuccess) return RC_E_DEVICE;
  }
  // the pinned staging is reused by this thread's next call: wait for its copy (and free the
  // scratch in order)
  return hipStreamSynchronize(s) == hipSuccess ? RC_OK : RC_E_DEVICE;
}

rc_status rc_container_offsets(rc_ctx* ctx, const uint8_t* container_dev,
                               const rc_container_info* info, uint64_t* code_off_dev,
                               uint64_t* code_len_dev, uint64_t* sym_off_dev) {
  hipStream_t s;
  int dev;
  if (rc_ctx_stream_(ctx, &s, &dev) != RC_OK || !container_dev || !info) return RC_E_ARG;
  const u32 n = (u32)info->n_chunks;
  if (info->n_chunks > RC_MAX_CHUNKS) return RC_E_BAD_CONTAINER;
  if (n && (!code_off_dev || !code_len_dev || !sym_off_dev)) return RC_E_ARG;
  DevSet g(dev);
  const u64* index = reinterpret_cast<const u64*>(container_dev + info->index_off);
  const u32 nb = (n + SBLK - 1) / SBLK;
  // code_off needs n + 1 slots for the scan total: scratch, then copy the first n
  Scratch sc(s);
  if (!sc.alloc(8ull * (n + 1) + 8ull * (nb + 1) + 16)) return RC_E_DEVICE;
  u64* coff = (u64*)sc.p;
  u64* tmp = coff + (n + 1);
  u32* bad = reinterpret_cast<u32*>(tmp + nb + 1);
  hipError_t e = hipMemsetAsync(bad, 0, 4, s);
  if (e == hipSuccess && n) {
    hipLaunchKernelGGL(k_unpack_index, dim3((n + SWG - 1) / SWG), dim3(SWG), 0, s, index, n,
                       code_len_dev, bad);
    e = hipGetLastError();
  }
  if (e == hipSuccess)
    e = device_scan(s, index, n, SCAN_SRC_STRIDE2_PAD16, 1, info->payload_off, coff, tmp);
  if (e == hipSuccess) e = device_scan(s, index, n, SCAN_SRC_STRIDE2, 0, 0, sym_off_dev, tmp);
  if (e == hipSuccess && n)
    e = hipMemcpyAsync(code_off_dev, coff, 8ull * n, hipMemcpyDeviceToDevice, s);
  u64* ends = (u64*)rc_pinned_scratch_(24);  // small read-backs through pinned memory
  if (!ends) return RC_E_DEVICE;
  ends[0] = ends[1] = ends[2] = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&ends[0], coff + n, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(&ends[1], sym_off_dev + n, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&ends[2], bad, 4, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return RC_E_DEVICE;
  const u32 hbad = (u32)ends[2];
  // the index must describe exactly the payload the header announces
  if (hbad || ends[0] != info->payload_off + info->payload_bytes || ends[1] != info->n_syms)
    return RC_E_BAD_CONTAINER;
  return RC_OK;
}

}  // extern "C"
