"""Second-workgroup-per-CU check: uniform static model at 2^17 x 1 KiB chunks
(512 workgroups, two per CU), decoded twice; prints the chunks that do not round-trip, their
workgroups and first wrong symbol, then decodes slices of the grid on their own.
    gpurun -- 'python tools/coresident_debug.py'   (RC_LIB_PATH selects a library variant)"""
import sys
sys.path.insert(0, "/root/repo")
import numpy as np, torch
import range_coder_rust_amd as rc
from range_coder_rust_amd import synth
ctx = rc.default_context(0)
c, cum, total = synth.uniform_table()
m = rc.StaticModel(c, cum, total)
inv = synth.inverse_cdf(c)
n, L = 1 << 17, 1024
syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
synth.fill(ctx, 0x5EED0002, inv, syms, L, n)
so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
cap = rc.slot_capacity(L, 8.0, slack=1.05)
oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
ol, fl = rc.encode_batch(m, syms, so, out, oo)
torch.cuda.synchronize()
for rep in range(2):
    dec = torch.empty_like(syms)
    fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
    torch.cuda.synchronize()
    S = syms.view(n, L).cpu().numpy(); D = dec.view(n, L).cpu().numpy(); F = fd.cpu().numpy()
    bad = np.nonzero((S != D).any(1))[0]
    print("rep", rep, "bad", len(bad), "flagged", int((F != 0).sum()), "first", bad[:12].tolist(),
          "wg", sorted(set((bad // 256).tolist()))[:12])
    if len(bad):
        pos = [int(np.argmax(S[k] != D[k])) for k in bad[:12]]
        print("  first mismatch positions", pos)
for lo, hi in [(0, 256), (256, 512), (0, 512), (0, 4096)]:
    idx = torch.arange(lo, hi, device="cuda")
    so2 = torch.arange(len(idx) + 1, dtype=torch.int64, device="cuda") * L
    dec2 = torch.empty(len(idx) * L, dtype=torch.uint8, device="cuda")
    fd2 = rc.decode_batch(m, out, oo[idx].contiguous(), ol[idx].contiguous(), dec2, so2)
    torch.cuda.synchronize()
    D2 = dec2.view(-1, L).cpu().numpy()
    print("chunks", lo, hi, "bad", int((S[lo:hi] != D2).any(1).sum()))
