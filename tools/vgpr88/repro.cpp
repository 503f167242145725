// tools/vgpr88/repro.cpp — the 88-VGPR question: run the round-1 coder kernels
// (rc_kernels_r1.hip) built at their natural 88-VGPR allocation and, from the same source with
// one clobbered register, at 96, on a co-resident workload (2^17 chunks = 512 workgroups of 256
// lanes), and compare every chunk with the C oracle.  Host buffers are pinned and every copy is
// synchronous, so nothing but the kernels can differ between the two builds.
// Usage: repro <n_chunks> <chunk_symbols>   (prints mismatch counts per model; always exits 0)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "range_coder_r1.h"
#include "../../oracle/rc_oracle.h"

#ifdef RC_PROBE
extern "C" int rc_probe_read(void* probe, size_t probe_bytes, void* canary, size_t canary_bytes);
#endif

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(0);                                                           \
    }                                                                    \
  } while (0)

static void run(rc_ctx* ctx, const char* name, const std::vector<uint32_t>& c, uint32_t n,
                uint64_t L) {
  const uint32_t na = (uint32_t)c.size();
  std::vector<uint32_t> cum(na);
  uint32_t total = 0;
  for (uint32_t i = 0; i < na; ++i) cum[i] = total, total += c[i];
  std::vector<uint8_t> inv(total);  // inverse CDF for sampling
  for (uint32_t s = 0; s < na; ++s)
    for (uint32_t j = 0; j < c[s]; ++j) inv[cum[s] + j] = (uint8_t)s;
  rc_model* m = nullptr;
  if (rc_model_create_static(ctx, na, c.data(), cum.data(), total, &m) != RC_OK) {
    printf("%s: model rejected\n", name);
    return;
  }
  const uint64_t cap = (2 * L + 64 + 15) & ~15ull, nsym = (uint64_t)n * L;
  uint8_t *hs, *hout, *hdec;
  uint64_t *hsoff, *hooff, *hlen;
  uint32_t *hfl, *hfd;
  CK(hipHostMalloc((void**)&hs, nsym));
  CK(hipHostMalloc((void**)&hdec, nsym));
  CK(hipHostMalloc((void**)&hout, n * cap));
  CK(hipHostMalloc((void**)&hsoff, 8ull * (n + 1)));
  CK(hipHostMalloc((void**)&hooff, 8ull * (n + 1)));
  CK(hipHostMalloc((void**)&hlen, 8ull * n));
  CK(hipHostMalloc((void**)&hfl, 4ull * n));
  CK(hipHostMalloc((void**)&hfd, 4ull * n));
  for (uint64_t i = 0; i < nsym; ++i) hs[i] = inv[mix64(0x5EED ^ i) % total];
  for (uint32_t k = 0; k <= n; ++k) hsoff[k] = k * L, hooff[k] = k * cap;
  uint8_t *ds, *dout, *ddec;
  uint64_t *dsoff, *dooff, *dlen;
  uint32_t *dfl, *dfd;
  CK(hipMalloc((void**)&ds, nsym));
  CK(hipMalloc((void**)&ddec, nsym));
  CK(hipMalloc((void**)&dout, n * cap));
  CK(hipMalloc((void**)&dsoff, 8ull * (n + 1)));
  CK(hipMalloc((void**)&dooff, 8ull * (n + 1)));
  CK(hipMalloc((void**)&dlen, 8ull * n));
  CK(hipMalloc((void**)&dfl, 4ull * n));
  CK(hipMalloc((void**)&dfd, 4ull * n));
  CK(hipMemcpy(ds, hs, nsym, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsoff, hsoff, 8ull * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dooff, hooff, 8ull * (n + 1), hipMemcpyHostToDevice));
  rc_status st = rc_encode_batch(ctx, m, ds, dsoff, n, dout, dooff, dlen, dfl);
  if (st == RC_OK) st = rc_ctx_synchronize(ctx);
  if (st != RC_OK) printf("%s: encode status %d\n", name, st);
  CK(hipMemcpy(hout, dout, n * cap, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hlen, dlen, 8ull * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hfl, dfl, 4ull * n, hipMemcpyDeviceToHost));
#ifdef RC_PROBE
  const uint32_t n_waves = (n + 63) / 64;
  std::vector<uint32_t> probe((size_t)n_waves * 8), canary(2ull * n);
  if (rc_probe_read(probe.data(), 4 * probe.size(), canary.data(), 4 * canary.size()))
    printf("%s: probe read failed\n", name);
#endif
  // decode the GPU's own code
  st = rc_decode_batch(ctx, m, dout, dooff, dlen, ddec, dsoff, n, dfd);
  if (st == RC_OK) st = rc_ctx_synchronize(ctx);
  if (st != RC_OK) printf("%s: decode status %d\n", name, st);
  CK(hipMemcpy(hdec, ddec, nsym, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hfd, dfd, 4ull * n, hipMemcpyDeviceToHost));
  // oracle, chunk by chunk
  std::vector<uint8_t> ob(cap);
  uint32_t bad_enc = 0, bad_dec = 0, first_enc = ~0u, first_dec = ~0u;
  std::vector<int64_t> first_byte(n, -1);  // first wrong byte of each chunk's stream
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t ol = 0;
    const uint32_t f = orc_encode(c.data(), cum.data(), na, total, hs + hsoff[k], L, ob.data(),
                                  cap, &ol);
    if (f != hfl[k] || ol != hlen[k] || memcmp(ob.data(), hout + hooff[k], ol)) {
      if (!bad_enc++) first_enc = k;
      uint64_t j = 0;
      while (j < ol && ob[j] == hout[hooff[k] + j]) ++j;
      first_byte[k] = (int64_t)j;
      // dump: this chunk's GPU and oracle bytes, and the chunk 65536 before it (the same lane
      // of the workgroup that shares its CU at two workgroups per CU), GPU and oracle
      static FILE* dump = nullptr;
      static uint32_t dumped = 0;
      const char* dp = getenv("RC_DUMP");
      if (dp && !dump) dump = fopen(dp, "ab");
      if (dump && dumped < 32 && k >= 65536) {
        ++dumped;
        std::vector<uint8_t> pb(cap);
        uint64_t pl = 0;
        orc_encode(c.data(), cum.data(), na, total, hs + hsoff[k - 65536], L, pb.data(), cap, &pl);
        uint32_t hdr[4] = {k, (uint32_t)ol, (uint32_t)pl, (uint32_t)hlen[k - 65536]};
        fwrite(hdr, 4, 4, dump);
        uint8_t b[4][256];
        memset(b, 0, sizeof b);
        memcpy(b[0], hout + hooff[k], std::min<uint64_t>(256, ol));
        memcpy(b[1], ob.data(), std::min<uint64_t>(256, ol));
        memcpy(b[2], hout + hooff[k - 65536], std::min<uint64_t>(256, pl));
        memcpy(b[3], pb.data(), std::min<uint64_t>(256, pl));
        fwrite(b, 1, sizeof b, dump);
        fflush(dump);
      }
      if (bad_enc <= 4)
        printf("%s: chunk %u: len gpu %llu oracle %llu flag %u/%u, first wrong byte %llu "
               "(gpu %02x oracle %02x)\n", name, k, (unsigned long long)hlen[k],
               (unsigned long long)ol, hfl[k], f, (unsigned long long)j,
               j < ol ? hout[hooff[k] + j] : 0, j < ol ? ob[j] : 0);
    }
    if (hfd[k] || memcmp(hdec + hsoff[k], hs + hsoff[k], L)) {
      if (!bad_dec++) first_dec = k;
    }
  }
#ifdef RC_PROBE
  {
    const char* dir = getenv("RC_PROBE_DIR");
    char path[512];
    snprintf(path, sizeof path, "%s/probe_%s.csv", dir ? dir : ".", name);
    FILE* fp = fopen(path, "w");
    if (fp) {
      fprintf(fp, "wave,wg,hw_id,gpr_alloc,lds_alloc,xcc_id,t0,t1,bad_chunks,min_first_byte,"
                  "canary_mask,canary_first\n");
      for (uint32_t w = 0; w < n_waves; ++w) {
        const uint32_t* pp = &probe[8ull * w];
        uint32_t nb = 0, cm = 0, cf = 0;
        int64_t mfb = -1;
        for (uint32_t k = 64 * w; k < 64 * w + 64 && k < n; ++k) {
          if (first_byte[k] >= 0) {
            ++nb;
            if (mfb < 0 || first_byte[k] < mfb) mfb = first_byte[k];
          }
          if (canary[2 * k] && !cm) cf = canary[2 * k + 1];
          cm |= canary[2 * k];
        }
        fprintf(fp, "%u,%u,%u,%u,%u,%u,%llu,%llu,%u,%lld,%u,%u\n", w, w / 4, pp[0], pp[1], pp[2],
                pp[3], (unsigned long long)pp[4] | ((unsigned long long)pp[5] << 32),
                (unsigned long long)pp[6] | ((unsigned long long)pp[7] << 32), nb,
                (long long)mfb, cm, cf);
      }
      fclose(fp);
    }
  }
#endif
  printf("%s: %u chunks x %llu symbols: encode mismatches %u (first %d), decode mismatches %u "
         "(first %d)\n", name, n, (unsigned long long)L, bad_enc, (int)first_enc, bad_dec,
         (int)first_dec);
  hipFree(ds), hipFree(ddec), hipFree(dout), hipFree(dsoff), hipFree(dooff), hipFree(dlen);
  hipFree(dfl), hipFree(dfd);
  hipHostFree(hs), hipHostFree(hdec), hipHostFree(hout), hipHostFree(hsoff), hipHostFree(hooff);
  hipHostFree(hlen), hipHostFree(hfl), hipHostFree(hfd);
  rc_model_destroy(m);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 0) : (1u << 17);
  const uint64_t L = argc > 2 ? strtoull(argv[2], nullptr, 0) : 4096;
  rc_ctx* ctx = nullptr;
  if (rc_ctx_create(0, &ctx) != RC_OK) {
    printf("no device\n");
    return 0;
  }
  std::vector<uint32_t> uni(256, 1), zipf(256);
  double w[256], sw = 0;
  for (int i = 0; i < 256; ++i) sw += (w[i] = 1.0 / __builtin_pow(i + 1.0, 1.2));
  uint32_t t = 0;
  for (int i = 0; i < 256; ++i) {
    zipf[i] = (uint32_t)__builtin_fmax(1.0, __builtin_rint(65536.0 * w[i] / sw));
    t += zipf[i];
  }
  zipf[0] += 65536 - t;
  run(ctx, "uniform", uni, n, L);
  run(ctx, "zipf", zipf, n, L);
  rc_ctx_destroy(ctx);
  return 0;
}
