"""Scratch timing of the adaptive (C4) kernels: 2^18 x 16 KiB Zipf chunks, encode + decode."""
import sys, time
sys.path.insert(0, "/root/repo")
import torch
import range_coder_rust_amd as rc
from range_coder_rust_amd import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
L = 16384
ctx = rc.default_context(0)
c, _, _ = synth.zipf_table()
inv = synth.inverse_cdf(c)
syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
synth.fill(ctx, 0x5EED0004, inv, syms, L, n)
m = rc.AdaptiveModel(256, 32, 57343, 256, ctx=ctx)
cap = rc.slot_capacity(L, 16)
so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
dec = torch.empty_like(syms)
torch.cuda.synchronize()
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    t0 = time.perf_counter()
    ol, fl = rc.encode_batch(m, syms, so, out, oo)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    N = n * L
    print(f"enc {1e3*(t1-t0):.1f} ms {N/(t1-t0)/1e9:.1f} Gsym/s  dec {1e3*(t2-t1):.1f} ms "
          f"{N/(t2-t1)/1e9:.1f} Gsym/s  B/sym {float(ol.sum())/N:.4f} "
          f"flags {int(fl.abs().sum())} {int(fd.abs().sum())} eq {torch.equal(dec, syms)}",
          flush=True)
