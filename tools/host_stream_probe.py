"""Where does rc_encode_host's time go?  Times encode_host / decode_host on pinned host buffers
(131072 x 64 KiB Zipf chunks, 8 GiB), per call, so it can run under
`rocprofv3 --kernel-trace --memory-copy-trace --stats` to split kernels from PCIe copies.
    python tools/host_stream_probe.py [n_chunks] [zipf|uniform]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    cfg = sys.argv[2] if len(sys.argv) > 2 else "zipf"
    L = 65536
    ctx = rc.default_context(0)
    c, cum, total = synth.zipf_table() if cfg == "zipf" else synth.uniform_table()
    m = rc.StaticModel(c, cum, total, ctx=ctx)
    cap = rc.slot_capacity(L, 8.0, slack=1.02)
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 7, synth.inverse_cdf(c), d, L, n)
    hs = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    hs.copy_(d)
    torch.cuda.synchronize()
    syms = hs.numpy()
    out = torch.empty(n * cap, dtype=torch.uint8, pin_memory=True).numpy()
    dec = torch.empty(n * L, dtype=torch.uint8, pin_memory=True).numpy()
    soff = np.arange(n + 1, dtype=np.uint64) * L
    ooff = np.arange(n + 1, dtype=np.uint64) * cap
    for rep in range(3):
        t0 = time.perf_counter()
        out, ol, fl = rc.encode_host(m, syms, soff, ooff, out=out)
        t1 = time.perf_counter()
        dec, fd = rc.decode_host(m, out, ooff[:-1], ol, soff, out=dec)
        t2 = time.perf_counter()
        print(f"rep {rep}: encode {t1 - t0:.3f} s ({n * L / (t1 - t0) / 1e9:.1f} GB/s), "
              f"decode {t2 - t1:.3f} s ({n * L / (t2 - t1) / 1e9:.1f} GB/s), "
              f"ok={bool((fl == 0).all() and (fd == 0).all())}", flush=True)
        if rep == 0:
            print("round trip exact:", bool(np.array_equal(dec, syms)), flush=True)


if __name__ == "__main__":
    main()
