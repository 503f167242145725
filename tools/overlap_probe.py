"""Does the encoder of one batch overlap the decoder of the previous one? (scratch measurement)

At 2^17 chunks per GPU (the configs[4] N = 8 shard) each coder has 2 waves per SIMD and is bound
by its per-symbol dependency chain, not by issue.  This probe times, on one GPU
and the same buffers, K steps of
  seq:  encode(batch) then decode(batch), one stream (bench.py's schedule);
  pipe: encode(batch k + 1) on one HIP stream while decode(batch k) runs on another (two code
        buffers; each step waits for both halves of the previous one).
Both do the same K encodes and K decodes of 64 KiB Zipf(1.2) chunks and check decode == input.

  python3 tools/overlap_probe.py --chunks 131072 [--steps 5] [--config zipf]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chunks", type=int, default=1 << 17)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--config", default="zipf")
    a = p.parse_args()
    import torch
    import bench
    import range_coder_rust_amd as rc
    from range_coder_rust_amd import synth
    ctx = rc.default_context(0)
    dev = torch.device("cuda", 0)
    n, L = a.chunks, 65536
    bufs = bench.Leg.alloc(torch, dev, n, L)
    legA = bench.Leg(torch, rc, synth, ctx, a.config, n, L, 0, bufs=bufs)
    out2 = torch.empty_like(bufs["out"])
    legB = bench.Leg(torch, rc, synth, ctx, a.config, n, L, 0,
                     bufs=dict(syms=bufs["syms"], out=out2, dec=bufs["dec"]))
    legs = (legA, legB)
    N = n * L * a.steps
    res = {"chunks": n, "config": a.config, "steps": a.steps}

    # sequential (bench.py's schedule)
    legA.encode(); legA.decode()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        legA.encode()
        legA.decode()
    torch.cuda.synchronize()
    ts = time.perf_counter() - t0
    ok = int(legA.fdec.abs().sum()) == 0 and bench.equal_chunked(torch, legA.dec, legA.syms)
    res["seq"] = dict(gsym_s=N / ts / 1e9, ms_per_step=ts / a.steps * 1e3, ok=ok)

    # pipelined: step k encodes into legs[(k + 1) % 2] while decoding legs[k % 2]
    se, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    legA.encode()
    torch.cuda.synchronize()
    enc_done = torch.cuda.Event()
    dec_done = torch.cuda.Event()
    enc_done.record(torch.cuda.current_stream(dev))
    dec_done.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    for k in range(a.steps):
        e_prev, d_prev = enc_done, dec_done
        enc_done, dec_done = torch.cuda.Event(), torch.cuda.Event()
        with torch.cuda.stream(se):
            se.wait_event(d_prev)  # the buffer this encode overwrites was read by decode k-1
            legs[(k + 1) % 2].encode()
            enc_done.record(se)
        with torch.cuda.stream(sd):
            sd.wait_event(e_prev)  # encode of batch k finished
            legs[k % 2].decode()
            dec_done.record(sd)
    torch.cuda.synchronize()
    tp = time.perf_counter() - t0
    okp = (int(legA.fdec.abs().sum()) == 0 and int(legB.fdec.abs().sum()) == 0
           and int(legA.fenc.abs().sum()) == 0 and int(legB.fenc.abs().sum()) == 0
           and bench.equal_chunked(torch, bufs["dec"], bufs["syms"]))
    res["pipe"] = dict(gsym_s=N / tp / 1e9, ms_per_step=tp / a.steps * 1e3, ok=okp)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
