"""Adaptive (C4) encode/decode time per symbol and lane at 1, 4 and 16 workgroups per CU
(2^14, 2^16, 2^18 x 16 KiB chunks): python tools/adapt_occupancy.py [n1,n2,...]
NODEC=1 skips the decode."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import range_coder_rust_amd as rc
from range_coder_rust_amd import synth
L = 16384
ctx = rc.default_context(0)
c, _, _ = synth.zipf_table()
m = rc.AdaptiveModel(256, 32, 57343, 256, ctx=ctx)
cap = rc.slot_capacity(L, 16)
for n in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["16384","65536","262144"])]:
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0004, synth.inverse_cdf(c), syms, L, n)
    so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    dec = torch.empty_like(syms)
    best, bestd = 1e9, 1e9
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ol, fl = rc.encode_batch(m, syms, so, out, oo)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if not os.environ.get("NODEC"): fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        best, bestd = min(best, t1 - t0), min(bestd, t2 - t1)
    print(f"n={n:7d} ({n // 64 // 256} enc WG/CU): encode {best * 1e3:7.2f} ms = {best / L * 1e9:6.1f} ns/symbol/lane, "
          f"{n * L / best / 1e9:6.1f} Gsym/s; decode {bestd * 1e3:7.2f} ms {n * L / bestd / 1e9:6.1f} Gsym/s", flush=True)
    del syms, out, dec
