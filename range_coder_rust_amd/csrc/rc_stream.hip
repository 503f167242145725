// rc_stream.hip — host-resident data through the GPU coder: a pipelined H2D / kernel / D2H
// stream over batches of chunks.
//
// rc_encode_host / rc_decode_host replace n_chunks x {Encoder::new; encode...; finish}
// (src/encoder.rs:14-46) / {Decoder::new; decode...} (src/decoder.rs:14-54) for data that lives
// in host memory.  The chunks are cut into batches of ~RC_STREAM_BATCH_BYTES; batch b uses slot
// b % RC_STREAM_SLOTS's device buffers.  Two streams:
//  * the in stream moves batch inputs host -> HBM with the DMA engines (hipMemcpyAsync), running
//    up to RC_STREAM_SLOTS batches ahead;
//  * the coder stream codes batch b with its output pointed straight at the mapped host buffer
//    (the kernel's stores cross PCIe), then copies the per-chunk lengths and flags back with
//    k_pcie_copy.  RC_STREAM_DIRECT=0 stages the output in HBM and moves it with k_pcie_copy
//    instead (8 GiB Zipf: encode 35.9 -> 42.4 GB/s, decode 32.1 -> 35.1 direct).
// The caller's big buffers are page-locked in place for the call (hipHostRegister; already
// pinned memory is used as it is) and mapped into the device's address space.  PCIe, not HBM,
// bounds this path.
//
// Why this split (tools/pcie_duplex.py, tools/pcie_kernel_probe.hip on the MI355X boxes):
//  * the DMA engines move 57 GB/s one way, but only 28.7 GB/s each way when H2D and D2H run at
//    once, which is a pipeline's steady state;
//  * copy kernels keep 45-47 GB/s each way at once, but while they touch host memory every other
//    kernel's HBM loads stall (a latency-bound probe kernel: 2.4 ms alone, 30-47 ms beside copy
//    kernels of 16-256 workgroups, on disjoint CUs too; a decode batch: 9.7 -> 36 ms);
//  * DMA H2D (31.6 GB/s) beside a D2H copy kernel (50.6 GB/s) is 82 GB/s together, and DMA
//    traffic leaves the coder alone (probe kernel 2.85 ms).
// So the coder never runs beside a copy kernel, and the DMA engines refill the input slots the
// whole time.  Each batch is staged in HBM at its host ranges' addresses mod 64, so the copy
// kernel moves 16-B vectors on both sides whatever the caller's alignment.  RC_STREAM_DMA=1 (or
// memory that cannot be mapped) moves outputs with hipMemcpyAsync too.
#include "rc_common.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#define RC_STREAM_SLOTS 3
// A chunk is one lane's serial stream: a batch kernel takes ~7-15 ms whatever its size (up to
// ~20 GiB of 64 KiB chunks, when every SIMD holds its 5 waves), and the coder stream pays it
// once per batch beside ~20 ms of output copy per GiB, so batches are large: 2 GiB, with the
// first two at 1/4 and 1/2 of that so the first input copy is short.
#define RC_STREAM_BATCH_BYTES (2ull << 30)
#define RC_STEP_COPIES 4  // copies per launch of k_pcie_copy (a batch's output: data, lengths,
                          // flags)
#ifndef RC_COPY_WGS
#define RC_COPY_WGS 256   // workgroups per bulk copy (tools/pcie_kernel_probe.hip: 256 keeps
                          // 46.7 GB/s each way with both directions at once; 2048 drops to 33)
#endif

struct rc_ctx;
struct rc_model;
extern "C" {
rc_status rc_ctx_stream_(rc_ctx* ctx, hipStream_t* s, int* device);
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

// set on the worker threads of rc_*_multi, which page-locked the caller's whole buffers once:
// a worker registering a sub-range again would, on unregistering it, unpin the whole range
thread_local bool t_pinned_by_caller = false;

// page-lock a caller buffer for the duration of the call (no-op if it is already pinned)
struct Pin {
  void* p = nullptr;
  bool mine = false;
  Pin(const void* ptr, size_t n, unsigned flags = hipHostRegisterMapped) {
    if (!ptr || !n || t_pinned_by_caller) return;
    p = const_cast<void*>(ptr);
    mine = hipHostRegister(p, n, flags) == hipSuccess;
    if (!mine) (void)hipGetLastError();  // already registered / pinned: fine either way
  }
  ~Pin() {
    if (mine && hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
  }
};

// device address of a pinned host byte (nullptr: not mapped, use the DMA engines)
const uint8_t* mapped(const void* host) {
  void* d = nullptr;
  if (!host || hipHostGetDevicePointer(&d, const_cast<void*>(host), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return (const uint8_t*)d;
}

struct CopyArgs {
  const uint8_t* src[RC_STEP_COPIES];
  uint8_t* dst[RC_STEP_COPIES];
  u64 n[RC_STEP_COPIES];
};

// copy blockIdx.y of a step: n bytes, one side mapped host memory.  When (src & 15) == (dst & 15)
// (bulk data: staging follows the host address) the body moves 16-B vectors, 4 per lane in
// flight, and the first wave copies the unaligned head and tail; otherwise (offset and result
// arrays, a few KiB) it copies bytes.
__global__ __launch_bounds__(256) void k_pcie_copy(CopyArgs a) {
  RC_VGPR_FLOOR_32();  // (build() requires allocations in 16-register steps)
  const uint8_t* __restrict__ src = a.src[blockIdx.y];
  uint8_t* __restrict__ dst = a.dst[blockIdx.y];
  const u64 n = a.n[blockIdx.y];
  if (((uintptr_t)src ^ (uintptr_t)dst) & 15) {
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256)
      dst[i] = src[i];
    return;
  }
  const u64 head = min(n, (u64)((16u - ((u32)(uintptr_t)dst & 15u)) & 15u));
  const u64 n16 = (n - head) >> 4, tail = (n - head) & 15;
  const uint4* s4 = (const uint4*)(src + head);
  uint4* d4 = (uint4*)(dst + head);
  const u64 stride = (u64)gridDim.x * 1024;
  for (u64 i = (u64)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) v[u] = s4[i + 256 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) d4[i + 256 * u] = v[u];
  }
  if (blockIdx.x == 0 && threadIdx.x < 32) {
    const u32 t = threadIdx.x;
    if (t < head) dst[t] = src[t];
    if (t >= 16 && t - 16 < tail) {
      const u64 o = head + 16 * n16 + (t - 16);
      dst[o] = src[o];
    }
  }
}

// one copy of a step; the host side's device address hdev is nullptr when it is not mapped
struct Copy {
  uint8_t* dst;
  const uint8_t* src;
  u64 n;
  bool h2d;
  const uint8_t* hdev;
};

// issue a step's copies on s: one k_pcie_copy launch for all mapped ones, hipMemcpyAsync for
// the rest
bool copy_step(const std::vector<Copy>& cs, hipStream_t s) {
  CopyArgs a{};
  u32 k = 0;
  u64 nmax = 0;
  for (const Copy& c : cs) {
    if (c.n == 0) continue;
    if (!c.hdev) {
      if (hipMemcpyAsync(c.dst, c.src, c.n,
                         c.h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, s) != hipSuccess)
        return false;
      continue;
    }
    a.src[k] = c.h2d ? c.hdev : c.src;
    a.dst[k] = c.h2d ? c.dst : const_cast<uint8_t*>(c.hdev);
    a.n[k] = c.n;
    nmax = std::max(nmax, c.n);
    ++k;
  }
  if (k == 0) return true;
  const unsigned gx = (unsigned)std::min<u64>(RC_COPY_WGS, (nmax + 16383) / 16384);
  hipLaunchKernelGGL(k_pcie_copy, dim3(gx, k), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess;
}

struct Batch {
  u32 k0, k1;       // chunks [k0, k1)
  u64 in0, in1;     // input byte range (host)
  u64 out0, out1;   // output byte range (host)
  u64 mi, mo;       // staging displacement: the host ranges' addresses mod 64
  u64* ho;          // its offsets in the pinned offset array
};

// Resources of the pipeline: RC_STREAM_SLOTS sets of device buffers, the copy and coder
// streams, per-slot events, and one pinned array for every batch's relative offsets and
// per-chunk results.
struct Pipe {
  hipStream_t copy = nullptr, code = nullptr;  // in stream (DMA), coder + out stream
  hipEvent_t copied[RC_STREAM_SLOTS] = {};  // batch t's input is in HBM (slot t % SLOTS)
  hipEvent_t coded[RC_STREAM_SLOTS] = {};   // batch t is coded and out (slot t % SLOTS)
  uint8_t* din[RC_STREAM_SLOTS] = {};
  uint8_t* dout[RC_STREAM_SLOTS] = {};
  u64* doff[RC_STREAM_SLOTS] = {};  // [2 * (kmax + 1)] offsets + [kmax] lengths
  u32* dfl[RC_STREAM_SLOTS] = {};
  u64* hoff = nullptr;              // pinned: per batch 2 * (chunks + 1) relative offsets
  u64* hlen = nullptr;              // pinned: n_chunks lengths (encode) / unused
  u32* hfl = nullptr;               // pinned: n_chunks flags
  bool ok = true;
  int device = -1;
  size_t c_in = 0, c_out = 0, c_off = 0;  // capacities this pipe was built for
  u32 c_k = 0, c_n = 0;

  bool fits(int dev, size_t in_max, size_t out_max, u32 kmax, u32 n_chunks, size_t n_off) const {
    return ok && dev == device && in_max <= c_in && out_max <= c_out && kmax <= c_k &&
           n_chunks <= c_n && n_off <= c_off;
  }
  bool init(size_t in_max, size_t out_max, u32 kmax, u32 n_chunks, size_t n_off) {
    (void)hipGetDevice(&device);
    c_in = in_max, c_out = out_max, c_k = kmax, c_n = n_chunks, c_off = n_off;
    ok = ok && make_streams();
    for (int i = 0; i < RC_STREAM_SLOTS; ++i) {
      ok = ok && hipEventCreateWithFlags(&copied[i], hipEventDisableTiming) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&coded[i], hipEventDisableTiming) == hipSuccess;
      ok = ok && hipMalloc((void**)&din[i], in_max + 64) == hipSuccess;
      ok = ok && hipMalloc((void**)&dout[i], out_max + 64) == hipSuccess;
      ok = ok && hipMalloc((void**)&doff[i], 8ull * (3ull * kmax + 2)) == hipSuccess;
      ok = ok && hipMalloc((void**)&dfl[i], 4ull * kmax + 4) == hipSuccess;
    }
    ok = ok && hipHostMalloc((void**)&hoff, 8ull * n_off + 8, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&hlen, 8ull * n_chunks + 8, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&hfl, 4ull * n_chunks + 4, hipHostMallocDefault) == hipSuccess;
    return ok;
  }
  bool make_streams() {
    return hipStreamCreateWithFlags(&copy, hipStreamNonBlocking) == hipSuccess &&
           hipStreamCreateWithFlags(&code, hipStreamNonBlocking) == hipSuccess;
  }
  bool drain() {
    bool r = true;
    if (copy) r = hipStreamSynchronize(copy) == hipSuccess && r;
    if (code) r = hipStreamSynchronize(code) == hipSuccess && r;
    return r;
  }
  ~Pipe() {
    drain();
    for (int i = 0; i < RC_STREAM_SLOTS; ++i) {
      if (din[i]) (void)hipFree(din[i]);
      if (dout[i]) (void)hipFree(dout[i]);
      if (doff[i]) (void)hipFree(doff[i]);
      if (dfl[i]) (void)hipFree(dfl[i]);
      if (copied[i]) (void)hipEventDestroy(copied[i]);
      if (coded[i]) (void)hipEventDestroy(coded[i]);
    }
    if (copy) (void)hipStreamDestroy(copy);
    if (code) (void)hipStreamDestroy(code);
    if (hoff) (void)hipHostFree(hoff);
    if (hlen) (void)hipHostFree(hlen);
    if (hfl) (void)hipHostFree(hfl);
  }
};

// One pipeline per context, kept between calls: its ~8 GiB of device buffers and pinned arrays
// cost far more to allocate than a batch takes to move (with most of HBM already allocated,
// per-call hipMalloc / hipFree cut the encode path from 29 to 12 GB/s).  A call takes the
// context's pipe out of the cache (so concurrent calls never share one), grows it if this
// call needs more, and puts it back; rc_ctx_destroy frees it.
std::mutex g_pipe_mu;
std::unordered_map<const rc_ctx*, Pipe*> g_pipes;

Pipe* pipe_acquire(const rc_ctx* ctx, int dev, size_t in_max, size_t out_max, u32 kmax,
                   u32 n_chunks, size_t n_off) {
  Pipe* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    auto it = g_pipes.find(ctx);
    if (it != g_pipes.end()) {
      p = it->second;
      g_pipes.erase(it);
    }
  }
  if (p && p->fits(dev, in_max, out_max, kmax, n_chunks, n_off)) return p;
  size_t a = in_max, b = out_max, e = n_off;
  u32 c = kmax, d = n_chunks;
  if (p && p->ok && p->device == dev) {  // grow to cover both the old and the new shape
    a = std::max(a, p->c_in), b = std::max(b, p->c_out), e = std::max(e, p->c_off);
    c = std::max(c, p->c_k), d = std::max(d, p->c_n);
  }
  delete p;
  p = new Pipe;
  if (!p->init(a, b, c, d, e)) {
    delete p;
    return nullptr;
  }
  return p;
}

void pipe_release(const rc_ctx* ctx, Pipe* p) {
  if (!p) return;
  if (!p->ok) {
    delete p;
    return;
  }
  Pipe* old = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    Pipe*& slot = g_pipes[ctx];
    old = slot;
    slot = p;
  }
  delete old;  // a concurrent call on the same context returned one first
}

// the pipe goes back to the cache on every return path
struct PipeLease {
  const rc_ctx* ctx;
  Pipe* p;
  ~PipeLease() {
    if (p && !p->drain()) p->ok = false;
    pipe_release(ctx, p);
  }
};

// cut [0, n) into batches of about `bytes` of input (>= 1 chunk each; the first two of 1/4
// and 1/2 of that).  A chunk for which alone(k) holds (one the kernel flags
// RC_F_TOO_LONG without reading or writing it) is a batch of its own, so no batch's input or
// output range spans its bytes.
template <class InRange, class OutRange, class Alone>
std::vector<Batch> plan(u64 bytes, u32 n, InRange in_range, OutRange out_range, Alone alone) {
  std::vector<Batch> b;
  u32 k = 0;
  while (k < n) {
    const u64 cap = bytes >> (b.size() < 2 ? 2 - b.size() : 0);
    Batch x{};
    x.k0 = k;
    u64 lo, hi, olo, ohi;
    in_range(k, lo, hi);
    out_range(k, olo, ohi);
    x.in0 = lo, x.in1 = hi, x.out0 = olo, x.out1 = ohi;
    ++k;
    while (k < n && !alone(k - 1) && !alone(k)) {
      u64 a, c, oa, oc;
      in_range(k, a, c);
      out_range(k, oa, oc);
      const u64 nin0 = std::min(x.in0, a), nin1 = std::max(x.in1, c);
      if (nin1 - nin0 > cap) break;
      x.in0 = nin0, x.in1 = nin1;
      x.out0 = std::min(x.out0, oa), x.out1 = std::max(x.out1, oc);
      ++k;
    }
    x.k1 = k;
    b.push_back(x);
  }
  return b;
}

rc_status any_flag(const uint32_t* flags, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (flags[i]) return RC_E_CHUNK;
  return RC_OK;
}

// Run the pipeline over B batches: batch t's input moves in on p.copy once batch t - SLOTS is
// out (its slot free), then p.code codes it and moves its output out.
template <class In, class Code, class Out>
rc_status run_pipeline(Pipe& p, size_t B, In in, Code code, Out out) {
  std::vector<Copy> cs;
  for (size_t t = 0; t < B; ++t) {
    const int i = (int)(t % RC_STREAM_SLOTS);
    cs.clear();
    if (t >= RC_STREAM_SLOTS && hipStreamWaitEvent(p.copy, p.coded[i], 0) != hipSuccess)
      return RC_E_DEVICE;
    in(t, i, cs);
    if (!copy_step(cs, p.copy) || hipEventRecord(p.copied[i], p.copy) != hipSuccess ||
        hipStreamWaitEvent(p.code, p.copied[i], 0) != hipSuccess)
      return RC_E_DEVICE;
    const rc_status st = code(t, i);
    if (st != RC_OK) return st;
    cs.clear();
    out(t, i, cs);
    if (!copy_step(cs, p.code) || hipEventRecord(p.coded[i], p.code) != hipSuccess)
      return RC_E_DEVICE;
  }
  return p.drain() ? RC_OK : RC_E_DEVICE;
}

}  // namespace

extern "C" {

rc_status rc_encode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* syms,
                         const uint64_t* sym_off, uint32_t n_chunks, uint8_t* out,
                         const uint64_t* out_off, uint64_t* out_len, uint32_t* flags) {
  hipStream_t s0;
  int dev;
  if (rc_ctx_stream_(ctx, &s0, &dev) != RC_OK || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!syms || !sym_off || !out || !out_off || !out_len || !flags) return RC_E_ARG;
  for (u32 k = 0; k < n_chunks; ++k)
    if (sym_off[k + 1] < sym_off[k] || out_off[k + 1] < out_off[k]) return RC_E_ARG;
  DevSet g(dev);
  // a chunk the kernel flags RC_F_TOO_LONG (never read nor written) is staged as empty
  auto too_long = [&](u32 k) { return sym_off[k + 1] - sym_off[k] > RC_MAX_CHUNK_SYMBOLS; };
  const RcKnobs& kn = rc_ctx_knobs_(ctx);
  std::vector<Batch> bs = plan(
      kn.stream_batch_bytes ? kn.stream_batch_bytes : (u64)RC_STREAM_BATCH_BYTES,
      n_chunks,
      [&](u32 k, u64& a, u64& b) { a = sym_off[k], b = too_long(k) ? a : sym_off[k + 1]; },
      [&](u32 k, u64& a, u64& b) { a = out_off[k], b = too_long(k) ? a : out_off[k + 1]; },
      too_long);
  size_t in_max = 0, out_max = 0, n_off = 0;
  u32 kmax = 0;
  for (const Batch& b : bs) {
    in_max = std::max<size_t>(in_max, b.in1 - b.in0);
    out_max = std::max<size_t>(out_max, b.out1 - b.out0);
    kmax = std::max(kmax, b.k1 - b.k0);
    n_off += 3ull * (b.k1 - b.k0 + 1);
  }
  // (the pins outlive the lease, whose destructor drains the streams on every return path)
  Pin pin_in(syms + sym_off[0], sym_off[n_chunks] - sym_off[0]);
  Pin pin_out(out + out_off[0], out_off[n_chunks] - out_off[0]);
  const bool dma = kn.stream_dma;
  const uint8_t* const m_out = dma ? nullptr : mapped(out + out_off[0]);
  PipeLease lease{ctx, pipe_acquire(ctx, dev, in_max, out_max, kmax, n_chunks, n_off)};
  if (!lease.p) return RC_E_DEVICE;
  Pipe& p = *lease.p;
  const uint8_t* const m_len = m_out ? mapped(p.hlen) : nullptr;
  const bool direct = m_out && kn.stream_direct;
  const uint8_t* const m_fl = m_out ? mapped(p.hfl) : nullptr;
  // the caller's stream must not run ahead into our buffers, nor we into its pending work
  (void)hipStreamSynchronize(s0);
  size_t o = 0;
  auto in = [&](size_t t, int i, std::vector<Copy>& cs) {
    Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    b.mi = (uintptr_t)(syms + b.in0) & 63, b.mo = (uintptr_t)(out + b.out0) & 63;
    u64* ho = b.ho = p.hoff + o;  // [sym_off rel (nk+1)] [out_off rel (nk+1)]
    for (u32 j = 0; j <= nk; ++j) {
      ho[j] = sym_off[b.k0 + j] - b.in0 + b.mi;
      ho[nk + 1 + j] = out_off[b.k0 + j] - b.out0 + b.mo;
    }
    o += 2ull * (nk + 1);
    cs.push_back({p.din[i] + b.mi, syms + b.in0, b.in1 - b.in0, true, nullptr});
    cs.push_back({(uint8_t*)p.doff[i], (const uint8_t*)ho, 16ull * (nk + 1), true, nullptr});
  };
  auto code = [&](size_t t, int i) {
    const Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    if (rc_ctx_set_stream(ctx, p.code) != RC_OK) return RC_E_DEVICE;
    // direct: the encoder writes the code straight into the mapped host buffer
    uint8_t* const ob = direct ? (uint8_t*)m_out + (b.out0 - out_off[0]) - b.mo : p.dout[i];
    const rc_status st = rc_encode_batch(ctx, m, p.din[i], p.doff[i], nk, ob,
                                         p.doff[i] + (nk + 1), p.doff[i] + 2 * (nk + 1), p.dfl[i]);
    (void)rc_ctx_set_stream(ctx, s0);
    return st;
  };
  auto outc = [&](size_t t, int i, std::vector<Copy>& cs) {
    const Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    if (!direct)
      cs.push_back({out + b.out0, p.dout[i] + b.mo, b.out1 - b.out0, false,
                    m_out ? m_out + (b.out0 - out_off[0]) : nullptr});
    cs.push_back({(uint8_t*)(p.hlen + b.k0), (const uint8_t*)(p.doff[i] + 2 * (nk + 1)), 8ull * nk,
                  false, m_len ? m_len + 8ull * b.k0 : nullptr});
    cs.push_back({(uint8_t*)(p.hfl + b.k0), (const uint8_t*)p.dfl[i], 4ull * nk, false,
                  m_fl ? m_fl + 4ull * b.k0 : nullptr});
  };
  const rc_status st = run_pipeline(p, bs.size(), in, code, outc);
  if (st != RC_OK) return st;
  memcpy(out_len, p.hlen, 8ull * n_chunks);
  memcpy(flags, p.hfl, 4ull * n_chunks);
  return any_flag(flags, n_chunks);
}

rc_status rc_decode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                         const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                         const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags) {
  hipStream_t s0;
  int dev;
  if (rc_ctx_stream_(ctx, &s0, &dev) != RC_OK || !m || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!code || !code_off || !code_len || !syms_out || !sym_off || !flags) return RC_E_ARG;
  for (u32 k = 0; k < n_chunks; ++k)
    if (sym_off[k + 1] < sym_off[k]) return RC_E_ARG;
  DevSet g(dev);
  auto too_long = [&](u32 k) { return sym_off[k + 1] - sym_off[k] > RC_MAX_CHUNK_SYMBOLS; };
  const RcKnobs& kn = rc_ctx_knobs_(ctx);
  std::vector<Batch> bs = plan(
      kn.stream_batch_bytes ? kn.stream_batch_bytes : (u64)RC_STREAM_BATCH_BYTES,
      n_chunks,
      [&](u32 k, u64& a, u64& b) { a = code_off[k], b = too_long(k) ? a : a + code_len[k]; },
      [&](u32 k, u64& a, u64& b) { a = sym_off[k], b = too_long(k) ? a : sym_off[k + 1]; },
      too_long);
  size_t in_max = 0, out_max = 0, n_off = 0;
  u32 kmax = 0;
  u64 cmin = ~0ull, cmax = 0;
  for (const Batch& b : bs) {
    in_max = std::max<size_t>(in_max, b.in1 - b.in0);
    out_max = std::max<size_t>(out_max, b.out1 - b.out0);
    kmax = std::max(kmax, b.k1 - b.k0);
    n_off += 3ull * (b.k1 - b.k0 + 1);
    cmin = std::min(cmin, b.in0);
    cmax = std::max(cmax, b.in1);
  }
  Pin pin_in(code + cmin, cmax - cmin);
  Pin pin_out(syms_out + sym_off[0], sym_off[n_chunks] - sym_off[0]);
  const bool dma = kn.stream_dma;
  const uint8_t* const m_out = dma ? nullptr : mapped(syms_out + sym_off[0]);
  PipeLease lease{ctx, pipe_acquire(ctx, dev, in_max, out_max, kmax, n_chunks, n_off)};
  if (!lease.p) return RC_E_DEVICE;
  Pipe& p = *lease.p;
  const uint8_t* const m_fl = m_out ? mapped(p.hfl) : nullptr;
  const bool direct = m_out && kn.stream_direct;
  (void)hipStreamSynchronize(s0);
  size_t o = 0;
  auto in = [&](size_t t, int i, std::vector<Copy>& cs) {
    Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    b.mi = (uintptr_t)(code + b.in0) & 63, b.mo = (uintptr_t)(syms_out + b.out0) & 63;
    u64* ho = b.ho = p.hoff + o;  // [code_off rel (nk) | code_len (nk)] [sym_off rel (nk+1)]
    for (u32 j = 0; j < nk; ++j) {
      ho[j] = code_off[b.k0 + j] - b.in0 + b.mi;
      ho[nk + j] = code_len[b.k0 + j];
    }
    for (u32 j = 0; j <= nk; ++j) ho[2 * nk + j] = sym_off[b.k0 + j] - b.out0 + b.mo;
    o += 3ull * nk + 1;
    cs.push_back({p.din[i] + b.mi, code + b.in0, b.in1 - b.in0, true, nullptr});
    cs.push_back({(uint8_t*)p.doff[i], (const uint8_t*)ho, 8ull * (3ull * nk + 1), true, nullptr});
  };
  auto coder = [&](size_t t, int i) {
    const Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    if (rc_ctx_set_stream(ctx, p.code) != RC_OK) return RC_E_DEVICE;
    // direct: the decoder writes the symbols straight into the mapped host buffer
    uint8_t* const ob = direct ? (uint8_t*)m_out + (b.out0 - sym_off[0]) - b.mo : p.dout[i];
    const rc_status st = rc_decode_batch(ctx, m, p.din[i], p.doff[i], p.doff[i] + nk, ob,
                                         p.doff[i] + 2 * nk, nk, p.dfl[i]);
    (void)rc_ctx_set_stream(ctx, s0);
    return st;
  };
  auto outc = [&](size_t t, int i, std::vector<Copy>& cs) {
    const Batch& b = bs[t];
    const u32 nk = b.k1 - b.k0;
    if (!direct)
      cs.push_back({syms_out + b.out0, p.dout[i] + b.mo, b.out1 - b.out0, false,
                    m_out ? m_out + (b.out0 - sym_off[0]) : nullptr});
    cs.push_back({(uint8_t*)(p.hfl + b.k0), (const uint8_t*)p.dfl[i], 4ull * nk, false,
                  m_fl ? m_fl + 4ull * b.k0 : nullptr});
  };
  const rc_status st = run_pipeline(p, bs.size(), in, coder, outc);
  if (st != RC_OK) return st;
  memcpy(flags, p.hfl, 4ull * n_chunks);
  return any_flag(flags, n_chunks);
}

}  // extern "C"

// ---- several devices from one host thread (rc_*_multi) ----
namespace {

// contiguous chunk ranges of about equal input bytes, one per context
std::vector<u32> split_by_bytes(u32 n, u32 parts, const std::function<u64(u32)>& bytes_of) {
  std::vector<u64> pre(n + 1, 0);
  for (u32 k = 0; k < n; ++k) pre[k + 1] = pre[k] + bytes_of(k);
  std::vector<u32> cut(parts + 1, n);
  cut[0] = 0;
  for (u32 i = 1; i < parts; ++i) {
    const u64 target = pre[n] / parts * i + std::min<u64>(pre[n] % parts, i);
    cut[i] = (u32)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
    cut[i] = std::max(cut[i], cut[i - 1]);
  }
  return cut;
}

template <class F>
rc_status run_parts(u32 n_ctx, const std::vector<u32>& cut, F f) {
  std::vector<rc_status> st(n_ctx, RC_OK);
  std::vector<std::thread> th;
  for (u32 i = 0; i < n_ctx; ++i)
    if (cut[i + 1] > cut[i])
      th.emplace_back([&, i] {
        t_pinned_by_caller = true;  // the multi call holds the pins
        st[i] = f(i, cut[i], cut[i + 1] - cut[i]);
      });
  for (auto& t : th) t.join();
  rc_status res = RC_OK;
  for (rc_status x : st)
    if (x != RC_OK && (res == RC_OK || res == RC_E_CHUNK)) res = x;
  return res;
}

}  // namespace

extern "C" {

rc_status rc_encode_host_multi(rc_ctx* const* ctxs, const rc_model* const* models, uint32_t n_ctx,
                               const uint8_t* syms, const uint64_t* sym_off, uint32_t n_chunks,
                               uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                               uint32_t* flags) {
  if (!ctxs || !models || n_ctx == 0 || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!syms || !sym_off || !out || !out_off || !out_len || !flags) return RC_E_ARG;
  for (u32 i = 0; i < n_ctx; ++i)
    if (!ctxs[i] || !models[i]) return RC_E_ARG;
  for (u32 k = 0; k < n_chunks; ++k)
    if (sym_off[k + 1] < sym_off[k] || out_off[k + 1] < out_off[k]) return RC_E_ARG;
  // pinned once for every device (each device's call then finds its range already pinned)
  const unsigned pf = hipHostRegisterPortable | hipHostRegisterMapped;
  Pin pin_in(syms + sym_off[0], sym_off[n_chunks] - sym_off[0], pf);
  Pin pin_out(out + out_off[0], out_off[n_chunks] - out_off[0], pf);
  const std::vector<u32> cut =
      split_by_bytes(n_chunks, n_ctx, [&](u32 k) { return sym_off[k + 1] - sym_off[k]; });
  return run_parts(n_ctx, cut, [&](u32 i, u32 k0, u32 nk) {
    return rc_encode_host(ctxs[i], models[i], syms, sym_off + k0, nk, out, out_off + k0,
                          out_len + k0, flags + k0);
  });
}

rc_status rc_decode_host_multi(rc_ctx* const* ctxs, const rc_model* const* models, uint32_t n_ctx,
                               const uint8_t* code, const uint64_t* code_off,
                               const uint64_t* code_len, uint8_t* syms_out,
                               const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags) {
  if (!ctxs || !models || n_ctx == 0 || n_chunks > RC_MAX_CHUNKS) return RC_E_ARG;
  if (n_chunks == 0) return RC_OK;
  if (!code || !code_off || !code_len || !syms_out || !sym_off || !flags) return RC_E_ARG;
  for (u32 i = 0; i < n_ctx; ++i)
    if (!ctxs[i] || !models[i]) return RC_E_ARG;
  for (u32 k = 0; k < n_chunks; ++k)
    if (sym_off[k + 1] < sym_off[k]) return RC_E_ARG;
  u64 cmin = ~0ull, cmax = 0;
  for (u32 k = 0; k < n_chunks; ++k) {
    cmin = std::min(cmin, code_off[k]);
    cmax = std::max(cmax, code_off[k] + code_len[k]);
  }
  const unsigned pf = hipHostRegisterPortable | hipHostRegisterMapped;
  Pin pin_in(code + cmin, cmax - cmin, pf);
  Pin pin_out(syms_out + sym_off[0], sym_off[n_chunks] - sym_off[0], pf);
  const std::vector<u32> cut = split_by_bytes(n_chunks, n_ctx, [&](u32 k) { return code_len[k]; });
  return run_parts(n_ctx, cut, [&](u32 i, u32 k0, u32 nk) {
    return rc_decode_host(ctxs[i], models[i], code, code_off + k0, code_len + k0, syms_out,
                          sym_off + k0, nk, flags + k0);
  });
}

// internal: free the context's cached pipeline (called by rc_ctx_destroy)
void rc_stream_release_(const rc_ctx* ctx) {
  Pipe* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    auto it = g_pipes.find(ctx);
    if (it != g_pipes.end()) {
      p = it->second;
      g_pipes.erase(it);
    }
  }
  delete p;
}

}  // extern "C"
