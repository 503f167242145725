"""A/B of the histogram kernels (RC_HIST_MODE, in the build that had them: wg4 | h8 | wg8 | pd2;
now RC_HIST_HOT: modes nohot | hot) on one box: per-chunk rows and
the batch histogram of 2^18 x 64 KiB chunks, uniform and Zipf(1.2); exactness vs torch.bincount."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402

ctx = rc.default_context(0)
n, L = 1 << 18, 65536
syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
res = {}
for data in ("uniform", "zipf"):
    if data == "zipf":
        c, _, _ = synth.zipf_table()
        synth.fill(ctx, 11, synth.inverse_cdf(c), syms, L, n)
    else:
        synth.fill(ctx, 11, synth.inverse_cdf([1] * 256), syms, L, n)
    want = torch.bincount(syms, minlength=256).to(torch.int64)
    for mode in sys.argv[1:] or ["nohot", "hot"]:
        os.environ["RC_HIST_MODE"] = mode
        os.environ["RC_HIST_HOT"] = "0" if mode == "nohot" else "1"
        hist, ch = rc.histogram(syms, off, per_chunk=True)
        ok = torch.equal(hist, want) and torch.equal(ch.sum(0, dtype=torch.int64), want)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = []
        for _ in range(5):
            ev[0].record()
            rc.histogram(syms, off, per_chunk=True)
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        ms = min(ts)
        res[f"{data}/{mode}"] = dict(ms=round(ms, 3), gbps=round(n * L / ms / 1e6, 1), exact=ok)
        print(data, mode, res[f"{data}/{mode}"], flush=True)
print(json.dumps(res))
