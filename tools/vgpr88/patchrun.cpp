// tools/vgpr88/patchrun.cpp — the same machine code at different VGPR allocations.
//
// Loads a round-1 code object (out/co_*.elf, built by build.sh), rewrites the VGPR granule field
// of k_encode_static<DIV_POW2>'s kernel descriptor (compute_pgm_rsrc1[5:0]) to the requested
// allocation, loads the patched image with hipModuleLoadData and encodes n chunks of L symbols
// (uniform 256-symbol model) with it.  Every chunk is compared with the C oracle.  With the probe
// build (co_p88.elf) each wave's HW_REG_GPR_ALLOC is read back, and mismatches are reported per
// VGPR base.  Only the allocation changes between runs: the instructions are byte-identical.
// Usage: patchrun <co.elf> <alloc VGPRs> <n_chunks> <L>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <elf.h>
#include <map>
#include <string>
#include <vector>

#include "../../oracle/rc_oracle.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static const char* kKernel = "_Z15k_encode_staticILi0EEv9ModelArgsPKhPKmjPhS4_PmPj";

// file offset of symbol `name` (an object in a section with file contents)
static long sym_offset(const std::vector<char>& img, const std::string& name) {
  const Elf64_Ehdr* eh = (const Elf64_Ehdr*)img.data();
  const Elf64_Shdr* sh = (const Elf64_Shdr*)(img.data() + eh->e_shoff);
  for (int i = 0; i < eh->e_shnum; ++i) {
    if (sh[i].sh_type != SHT_SYMTAB && sh[i].sh_type != SHT_DYNSYM) continue;
    const Elf64_Sym* sy = (const Elf64_Sym*)(img.data() + sh[i].sh_offset);
    const char* str = img.data() + sh[sh[i].sh_link].sh_offset;
    for (size_t j = 0; j < sh[i].sh_size / sizeof(Elf64_Sym); ++j)
      if (name == str + sy[j].st_name) {
        const Elf64_Shdr& s = sh[sy[j].st_shndx];
        return (long)(s.sh_offset + (sy[j].st_value - s.sh_addr));
      }
  }
  return -1;
}

struct ModelArgs {  // rc_kernels_r1.hip
  const void* tab;
  const void* lut;
  uint64_t magic;
  uint32_t n, total, lg, lut_shift, lut_max;
  float ftotal;
};

int main(int argc, char** argv) {
  if (argc < 5) {
    printf("usage: patchrun <co.elf> <alloc> <n_chunks> <L>\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<char> img;
  char buf[65536];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) img.insert(img.end(), buf, buf + r);
  fclose(f);
  const uint32_t alloc = (uint32_t)strtoul(argv[2], nullptr, 0);
  const uint32_t n = (uint32_t)strtoul(argv[3], nullptr, 0);
  const uint64_t L = strtoull(argv[4], nullptr, 0);
  const long kd = sym_offset(img, std::string(kKernel) + ".kd");
  if (kd < 0 || alloc % 8 || alloc < 8 || alloc > 512) {
    printf("bad descriptor or allocation\n");
    return 2;
  }
  uint32_t rsrc1;
  memcpy(&rsrc1, img.data() + kd + 48, 4);
  const uint32_t old = ((rsrc1 & 63) + 1) * 8;
  rsrc1 = (rsrc1 & ~63u) | (alloc / 8 - 1);
  memcpy(img.data() + kd + 48, &rsrc1, 4);

  hipModule_t mod;
  CK(hipModuleLoadData(&mod, img.data()));
  hipFunction_t fn;
  CK(hipModuleGetFunction(&fn, mod, kKernel));
  hipDeviceptr_t probe = nullptr;
  size_t probe_bytes = 0;
  const bool has_probe = hipModuleGetGlobal(&probe, &probe_bytes, mod, "g_probe") == hipSuccess;

  // uniform 256-symbol model: (cum, c) = (i, 1), total 256
  std::vector<uint32_t> c(256, 1), cum(256);
  for (int i = 0; i < 256; ++i) cum[i] = i;
  std::vector<uint32_t> tab(512);
  for (int i = 0; i < 256; ++i) tab[2 * i] = cum[i], tab[2 * i + 1] = 1;
  const uint64_t cap = (2 * L + 64 + 15) & ~15ull, nsym = (uint64_t)n * L;
  std::vector<uint8_t> hs(nsym), hout(n * cap);
  std::vector<uint64_t> soff(n + 1), ooff(n + 1), hlen(n);
  std::vector<uint32_t> hfl(n);
  for (uint64_t i = 0; i < nsym; ++i) hs[i] = (uint8_t)(mix64(0x5EED ^ i) & 255);
  for (uint32_t k = 0; k <= n; ++k) soff[k] = k * L, ooff[k] = k * cap;
  void *dtab, *ds, *dout, *dsoff, *dooff, *dlen, *dfl;
  CK(hipMalloc(&dtab, 2048));
  CK(hipMalloc(&ds, nsym));
  CK(hipMalloc(&dout, n * cap));
  CK(hipMalloc(&dsoff, 8ull * (n + 1)));
  CK(hipMalloc(&dooff, 8ull * (n + 1)));
  CK(hipMalloc(&dlen, 8ull * n));
  CK(hipMalloc(&dfl, 4ull * n));
  CK(hipMemcpy(dtab, tab.data(), 2048, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), nsym, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsoff, soff.data(), 8ull * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dooff, ooff.data(), 8ull * (n + 1), hipMemcpyHostToDevice));

  struct {
    ModelArgs m;
    const void* syms;
    const void* sym_off;
    uint32_t n_chunks, pad;
    void* out;
    const void* out_off;
    void* out_len;
    void* flags;
  } args;
  static_assert(sizeof(args) == 104, "kernarg layout");
  memset(&args, 0, sizeof args);
  args.m.tab = dtab;
  args.m.magic = ~0ull / 256;
  args.m.n = 256;
  args.m.total = 256;
  args.m.lg = 8;
  args.m.ftotal = 256.f;
  args.syms = ds, args.sym_off = dsoff, args.n_chunks = n, args.out = dout, args.out_off = dooff;
  args.out_len = dlen, args.flags = dfl;
  size_t asz = sizeof args;
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz,
                 HIP_LAUNCH_PARAM_END};
  CK(hipModuleLaunchKernel(fn, (n + 255) / 256, 1, 1, 256, 1, 1, 0, nullptr, nullptr, cfg));
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hout.data(), dout, n * cap, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hlen.data(), dlen, 8ull * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hfl.data(), dfl, 4ull * n, hipMemcpyDeviceToHost));
  std::vector<uint32_t> pr;
  if (has_probe) {
    pr.resize(probe_bytes / 4);
    CK(hipMemcpy(pr.data(), probe, probe_bytes, hipMemcpyDeviceToHost));
  }
  std::vector<uint8_t> ob(cap);
  uint32_t bad = 0;
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> by_base;  // vbase -> (waves, bad waves)
  for (uint32_t w = 0; w < (n + 63) / 64; ++w) {
    uint32_t wb = 0;
    for (uint32_t k = 64 * w; k < 64 * w + 64 && k < n; ++k) {
      uint64_t ol = 0;
      const uint32_t fl = orc_encode(c.data(), cum.data(), 256, 256, hs.data() + soff[k], L,
                                     ob.data(), cap, &ol);
      if (fl != hfl[k] || ol != hlen[k] || memcmp(ob.data(), hout.data() + ooff[k], ol)) ++wb;
    }
    bad += wb;
    const uint32_t base = has_probe && 8 * w + 1 < pr.size() ? (pr[8 * w + 1] & 63) * 8 : 0;
    auto& e = by_base[has_probe ? base : 9999];
    e.first += 1;
    e.second += wb != 0;
  }
  printf("alloc %u (built %u), %u chunks x %llu: mismatching chunks %u\n", alloc, old, n,
         (unsigned long long)L, bad);
  for (auto& kv : by_base)
    printf("   vgpr base %4u: waves %6u  bad waves %6u\n", kv.first, kv.second.first,
           kv.second.second);
  return 0;
}
