#!/usr/bin/env python3
"""One configuration of the hot path, no extras: encode then decode `--steps` times over
synthetic chunks in HBM, per-kernel HIP-event times, the round trip checked.  For counter
passes (tools/pmc_bound.sh, tools/profile.sh) and same-box A/B runs; bench.py is the headline.

  python3 tools/kbench.py --config zipf --chunks 1048576 --steps 3 --warmup 1

--config: uniform (c = 1, total 256), zipf (Zipf(1.2), total 2^16), adaptive (C4 over Zipf(1.2)
data), adaptive128 (C4 with a 128-symbol alphabet over Zipf(1.2) data on 128 symbols).
Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="zipf",
                   choices=["uniform", "zipf", "adaptive", "adaptive128"])
    p.add_argument("--chunks", type=int, default=1 << 20)
    p.add_argument("--chunk-bytes", type=int, default=65536)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--zipf-s", type=float, default=1.2, help="zipf: the exponent")
    p.add_argument("--zipf-total", type=int, default=1 << 16, help="zipf: the table's total")
    p.add_argument("--first-chunk", type=int, default=0,
                   help="global index of this run's first chunk (a shard of the bench stream)")
    a = p.parse_args()
    import torch
    import range_coder_rust_amd as rc
    from range_coder_rust_amd import shard, synth
    ctx = rc.default_context(0)
    n, L = a.chunks, a.chunk_bytes
    if a.config == "uniform":
        c, cum, total = synth.uniform_table()
    elif a.config == "adaptive128":
        c, cum, total = synth.zipf_table(n=128, total=1 << 16)
    else:
        c, cum, total = synth.zipf_table(s=a.zipf_s, total=a.zipf_total)
    if a.config.startswith("adaptive"):
        m = rc.AdaptiveModel(len(c), **rc.ADAPTIVE_DEFAULTS, ctx=ctx)
        bits = 6.0 if a.config == "adaptive" else 5.5
    else:
        m = rc.StaticModel(c, cum, total, ctx=ctx)
        bits = 8.0
    cap = rc.slot_capacity(L, bits, slack=1.02)
    dev = torch.device("cuda", 0)
    syms = torch.empty(n * L, dtype=torch.uint8, device=dev)
    synth.fill(ctx, shard.synth_seed(0x5EED0001, a.first_chunk), synth.inverse_cdf(c), syms, L, n)
    out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    dec = torch.empty(n * L, dtype=torch.uint8, device=dev)
    so = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
    oo = torch.arange(n + 1, dtype=torch.int64, device=dev) * cap
    co = oo[:-1].contiguous()
    ol = torch.zeros(n, dtype=torch.int64, device=dev)
    fe = torch.zeros(n, dtype=torch.int32, device=dev)
    fd = torch.zeros(n, dtype=torch.int32, device=dev)
    for _ in range(a.warmup):
        rc.encode_batch(m, syms, so, out, oo, ol, fe)
        rc.decode_batch(m, out, co, ol, dec, so, fd)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    torch.cuda.synchronize()
    for e0, e1, e2 in ev:
        e0.record()
        rc.encode_batch(m, syms, so, out, oo, ol, fe)
        e1.record()
        rc.decode_batch(m, out, co, ol, dec, so, fd)
        e2.record()
    torch.cuda.synchronize()
    enc = float(np.mean([x.elapsed_time(y) for x, y, _ in ev])) if ev else 0.0
    dcd = float(np.mean([y.elapsed_time(z) for _, y, z in ev])) if ev else 0.0
    ok = int(fe.abs().sum()) == 0 and int(fd.abs().sum()) == 0
    for i in range(0, n * L, 1 << 30):
        ok = ok and torch.equal(dec[i:i + (1 << 30)], syms[i:i + (1 << 30)])
    code = int(ol.sum())
    res = dict(config=a.config, chunks=n, table_total=int(total), chunk_bytes=L, steps=a.steps,
               encode_ms=round(enc, 3), decode_ms=round(dcd, 3),
               encode_gsym_s=round(n * L / enc / 1e6, 3) if enc else None,
               decode_gsym_s=round(n * L / dcd / 1e6, 3) if dcd else None,
               round_trip_gsym_s=round(n * L / (enc + dcd) / 1e6, 3) if enc else None,
               bytes_per_symbol=round(code / (n * L), 5), alg_bytes=n * L + code,
               decode_frac=round((n * L + code) / dcd / 1e6 / 8000.0, 4) if dcd else None,
               bit_exact_round_trip=bool(ok))
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
