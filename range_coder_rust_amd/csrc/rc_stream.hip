// rc_stream.hip — host-resident data through the GPU coder: a pipelined H2D / kernel / D2H
// stream over batches of chunks.
//
// rc_encode_host / rc_decode_host replace n_chunks x {Encoder::new; encode...; finish}
// (src/encoder.rs:14-46) / {Decoder::new; decode...} (src/decoder.rs:14-54) for data that lives
// in host memory.  The chunks are cut into batches of ~RC_STREAM_BATCH_BYTES; batch b runs on
// stream b % RC_STREAM_SLOTS with that slot's device buffers, so the copy engines move batch
// b+1 in and batch b-1 out while batch b is coded.  The caller's big buffers are page-locked in
// place for the call (hipHostRegister; already pinned memory is used as it is), so every copy
// is a direct DMA.  PCIe, not HBM, bounds this path: ~50 GB/s each way on Gen5 x16.
#include "rc_common.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#define RC_STREAM_SLOTS 4
// A chunk is one lane's serial stream: a batch kernel takes ~10-20 ms whatever its size, so a
// batch must carry ~1 GiB for the coder to outrun PCIe (~50 GB/s x 20 ms).
#define RC_STREAM_BATCH_BYTES (1ull << 30)

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
  Pin(const void* ptr, size_t n, unsigned flags = hipHostRegisterDefault) {
    if (!ptr || !n || t_pinned_by_caller) return;
    p = const_cast<void*>(ptr);
    mine = hipHostRegister(p, n, flags) == hipSuccess;
    if (!mine) (void)hipGetLastError();  // already registered / pinned: fine either way
  }
  ~Pin() {
    if (mine && hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
  }
};

struct Batch {
  u32 k0, k1;       // chunks [k0, k1)
  u64 in0, in1;     // input byte range (host)
  u64 out0, out1;   // output byte range (host)
};

// Resources of the pipeline: RC_STREAM_SLOTS streams, each with its own device buffers, and
// one pinned array for every batch's relative offsets and per-chunk results.
struct Pipe {
  hipStream_t st[RC_STREAM_SLOTS] = {};
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
    for (int i = 0; i < RC_STREAM_SLOTS; ++i) {
      ok = ok && hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) == hipSuccess;
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
  bool drain() {
    bool r = true;
    for (int i = 0; i < RC_STREAM_SLOTS; ++i)
      if (st[i]) r = hipStreamSynchronize(st[i]) == hipSuccess && r;
    return r;
  }
  ~Pipe() {
    drain();
    for (int i = 0; i < RC_STREAM_SLOTS; ++i) {
      if (din[i]) (void)hipFree(din[i]);
      if (dout[i]) (void)hipFree(dout[i]);
      if (doff[i]) (void)hipFree(doff[i]);
      if (dfl[i]) (void)hipFree(dfl[i]);
      if (st[i]) (void)hipStreamDestroy(st[i]);
    }
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

// batch size: RC_STREAM_BATCH_BYTES, or the environment variable of that name (tests use small
// batches to run many of them)
u64 batch_bytes() {
  const char* e = getenv("RC_STREAM_BATCH_BYTES");
  const u64 v = e ? strtoull(e, nullptr, 0) : 0;
  return v ? v : RC_STREAM_BATCH_BYTES;
}

// cut [0, n) into batches of about batch_bytes() of input (>= 1 chunk each)
template <class InRange, class OutRange>
std::vector<Batch> plan(u32 n, InRange in_range, OutRange out_range) {
  const u64 cap = batch_bytes();
  std::vector<Batch> b;
  u32 k = 0;
  while (k < n) {
    Batch x;
    x.k0 = k;
    u64 lo, hi, olo, ohi;
    in_range(k, lo, hi);
    out_range(k, olo, ohi);
    x.in0 = lo, x.in1 = hi, x.out0 = olo, x.out1 = ohi;
    ++k;
    while (k < n) {
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
  const std::vector<Batch> bs = plan(
      n_chunks,
      [&](u32 k, u64& a, u64& b) { a = sym_off[k], b = too_long(k) ? a : sym_off[k + 1]; },
      [&](u32 k, u64& a, u64& b) { a = out_off[k], b = too_long(k) ? a : out_off[k + 1]; });
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
  PipeLease lease{ctx, pipe_acquire(ctx, dev, in_max, out_max, kmax, n_chunks, n_off)};
  if (!lease.p) return RC_E_DEVICE;
  Pipe& p = *lease.p;
  // the caller's stream must not run ahead into our buffers, nor we into its pending work
  (void)hipStreamSynchronize(s0);
  size_t o = 0;
  for (size_t bi = 0; bi < bs.size(); ++bi) {
    const Batch& b = bs[bi];
    const int i = (int)(bi % RC_STREAM_SLOTS);
    hipStream_t s = p.st[i];
    const u32 nk = b.k1 - b.k0;
    u64* ho = p.hoff + o;  // [sym_off rel (nk+1)] [out_off rel (nk+1)]
    for (u32 j = 0; j <= nk; ++j) {
      ho[j] = sym_off[b.k0 + j] - b.in0;
      ho[nk + 1 + j] = out_off[b.k0 + j] - b.out0;
    }
    o += 2ull * (nk + 1);
    bool ok = hipMemcpyAsync(p.din[i], syms + b.in0, b.in1 - b.in0, hipMemcpyHostToDevice, s) ==
                  hipSuccess &&
              hipMemcpyAsync(p.doff[i], ho, 16ull * (nk + 1), hipMemcpyHostToDevice, s) == hipSuccess;
    if (!ok) return RC_E_DEVICE;
    u64* d_soff = p.doff[i];
    u64* d_ooff = p.doff[i] + (nk + 1);
    u64* d_len = p.doff[i] + 2 * (nk + 1);
    if (rc_ctx_set_stream(ctx, s) != RC_OK) return RC_E_DEVICE;
    const rc_status st = rc_encode_batch(ctx, m, p.din[i], d_soff, nk, p.dout[i], d_ooff, d_len,
                                         p.dfl[i]);
    (void)rc_ctx_set_stream(ctx, s0);
    if (st != RC_OK) return st;
    ok = hipMemcpyAsync(out + b.out0, p.dout[i], b.out1 - b.out0, hipMemcpyDeviceToHost, s) ==
             hipSuccess &&
         hipMemcpyAsync(p.hlen + b.k0, d_len, 8ull * nk, hipMemcpyDeviceToHost, s) == hipSuccess &&
         hipMemcpyAsync(p.hfl + b.k0, p.dfl[i], 4ull * nk, hipMemcpyDeviceToHost, s) == hipSuccess;
    if (!ok) return RC_E_DEVICE;
  }
  if (!p.drain()) return RC_E_DEVICE;
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
  const std::vector<Batch> bs = plan(
      n_chunks,
      [&](u32 k, u64& a, u64& b) { a = code_off[k], b = too_long(k) ? a : a + code_len[k]; },
      [&](u32 k, u64& a, u64& b) { a = sym_off[k], b = too_long(k) ? a : sym_off[k + 1]; });
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
  PipeLease lease{ctx, pipe_acquire(ctx, dev, in_max, out_max, kmax, n_chunks, n_off)};
  if (!lease.p) return RC_E_DEVICE;
  Pipe& p = *lease.p;
  (void)hipStreamSynchronize(s0);
  size_t o = 0;
  for (size_t bi = 0; bi < bs.size(); ++bi) {
    const Batch& b = bs[bi];
    const int i = (int)(bi % RC_STREAM_SLOTS);
    hipStream_t s = p.st[i];
    const u32 nk = b.k1 - b.k0;
    u64* ho = p.hoff + o;  // [code_off rel (nk) | code_len (nk)] [sym_off rel (nk+1)]
    for (u32 j = 0; j < nk; ++j) {
      ho[j] = code_off[b.k0 + j] - b.in0;
      ho[nk + j] = code_len[b.k0 + j];
    }
    for (u32 j = 0; j <= nk; ++j) ho[2 * nk + j] = sym_off[b.k0 + j] - b.out0;
    o += 3ull * nk + 1;
    bool ok = hipMemcpyAsync(p.din[i], code + b.in0, b.in1 - b.in0, hipMemcpyHostToDevice, s) ==
                  hipSuccess &&
              hipMemcpyAsync(p.doff[i], ho, 8ull * (3ull * nk + 1), hipMemcpyHostToDevice, s) ==
                  hipSuccess;
    if (!ok) return RC_E_DEVICE;
    if (rc_ctx_set_stream(ctx, s) != RC_OK) return RC_E_DEVICE;
    const rc_status st = rc_decode_batch(ctx, m, p.din[i], p.doff[i], p.doff[i] + nk, p.dout[i],
                                         p.doff[i] + 2 * nk, nk, p.dfl[i]);
    (void)rc_ctx_set_stream(ctx, s0);
    if (st != RC_OK) return st;
    ok = hipMemcpyAsync(syms_out + b.out0, p.dout[i], b.out1 - b.out0, hipMemcpyDeviceToHost,
                        s) == hipSuccess &&
         hipMemcpyAsync(p.hfl + b.k0, p.dfl[i], 4ull * nk, hipMemcpyDeviceToHost, s) == hipSuccess;
    if (!ok) return RC_E_DEVICE;
  }
  if (!p.drain()) return RC_E_DEVICE;
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
  Pin pin_in(syms + sym_off[0], sym_off[n_chunks] - sym_off[0], hipHostRegisterPortable);
  Pin pin_out(out + out_off[0], out_off[n_chunks] - out_off[0], hipHostRegisterPortable);
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
  Pin pin_in(code + cmin, cmax - cmin, hipHostRegisterPortable);
  Pin pin_out(syms_out + sym_off[0], sym_off[n_chunks] - sym_off[0], hipHostRegisterPortable);
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
