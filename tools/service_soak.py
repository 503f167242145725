"""Stream-service soak (GPU box): many short per-call sessions through the Python mirror with a
caller-adaptive model, with pauses around the service wave's idle exit (0.25 ms) and lifetime
(1 ms), batch round trips on the same context between and inside sessions (a batch launch makes
the wave yield), and contexts destroyed and recreated, for a time budget.  Every session encodes a random symbol string with
rc.Encoder (reading encode()'s byte count at random calls, so some flushes are one symbol), checks
the bytes against the C oracle's resumable encoder over the same (c, cum, total) triples, then
decodes them with rc.Decoder under the same adaptive model and checks the symbols.  Prints a
progress line every few seconds and one JSON summary line; exits 1 at the first mismatch.

Usage (GPU box): python3 tools/service_soak.py [seconds] [seed]
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import percall_bench as pb  # noqa: E402
import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import cpu  # noqa: E402


def batch_check(rng, ctx):
    """A small batch round trip on ctx (rc_encode_batch / rc_decode_batch): its launches make a
    live service wave of the context yield.  Returns an error string or None."""
    import torch
    n, L = rng.randint(1, 96), rng.choice([0, 1, 100, 1024, 4096])
    c, cum, total = synth.zipf_table(s=rng.uniform(0.5, 1.5), total=1 << 12)
    m = rc.StaticModel(c, cum, total, ctx=ctx)
    dev = torch.device("cuda", 0)
    syms = torch.randint(0, 256, (max(n * L, 1),), dtype=torch.uint8, device=dev)
    cap = rc.slot_capacity(L, 16.0)  # (uniform data, total 2^12: at most 12 bits a symbol)
    so = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
    oo = torch.arange(n + 1, dtype=torch.int64, device=dev) * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    ol = torch.zeros(n, dtype=torch.int64, device=dev)
    fe = torch.zeros(n, dtype=torch.int32, device=dev)
    dec = torch.empty_like(syms)
    fd = torch.zeros(n, dtype=torch.int32, device=dev)
    rc.encode_batch(m, syms, so, out, oo, ol, fe)
    rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so, fd)
    torch.cuda.synchronize()
    if int(fe.abs().sum()) or int(fd.abs().sum()) or not torch.equal(dec[:n * L], syms[:n * L]):
        return "batch round trip between per-call sessions"
    return None


def session(rng, ctx):
    n = rng.choice([1, 2, 5, 40, rng.randint(1, 400)])
    mid = rng.randint(0, n - 1) if rng.random() < 0.1 else -1  # a batch inside the session
    syms = [min(255, int(rng.paretovariate(1.1)) - 1) for _ in range(n)]
    m = pb.Adaptive()
    enc = rc.Encoder(ctx)
    trip = []
    for i, s in enumerate(syms):
        trip.append((m.c_freq(s), m.cum_freq(s), m.total_freq()))
        b = enc.encode(m, s)
        if rng.random() < 0.2:
            int(b)  # encode()'s return value now: a flush of the staged symbols
        if i == mid and batch_check(rng, ctx):
            return n, "batch round trip inside a session"
        m.update(s, i)
    code = enc.finish()
    st = cpu.Stream.fresh()
    f, want, _ = cpu.stream_encode(st, np.array(trip, np.uint32), finish=True)
    if f != 0 or bytes(want) != code:
        return n, "encode bytes differ from the oracle"
    m = pb.Adaptive()
    dec = rc.Decoder(code, ctx=ctx)
    for i in range(n):
        s = dec.decode(m)
        if s != syms[i]:
            return n, f"decode symbol {i}"
        if i == mid and batch_check(rng, ctx):
            return n, "batch round trip inside a decode session"
        m.update(s, i)
    return n, None


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    rng = random.Random(seed)
    t_end = time.time() + budget
    ctx = rc.Context(0)
    sessions = symbols = pauses = recreated = batches = 0
    t_print = time.time()
    while time.time() < t_end:
        n, bad = session(rng, ctx)
        sessions += 1
        symbols += n
        if bad:
            print(json.dumps({"mismatch": bad, "session": sessions, "seed": seed}))
            return 1
        r = rng.random()
        if r < 0.3:  # around the wave's 0.25-ms idle exit and 1-ms lifetime
            time.sleep(rng.uniform(0.0001, 0.002))
            pauses += 1
        elif r < 0.4:  # a batch round trip: the live wave yields to its launches
            bad = batch_check(rng, ctx)
            if bad:
                print(json.dumps({"mismatch": bad, "session": sessions, "seed": seed}))
                return 1
            batches += 1
        elif r < 0.45:  # destroy the context (stops its wave) and start over
            ctx.close()
            ctx = rc.Context(0)
            recreated += 1
        if time.time() - t_print > 5:
            print(f"{sessions} sessions, {symbols} symbols, {pauses} idle pauses, "
                  f"{batches} batches, {recreated} contexts recreated", flush=True)
            t_print = time.time()
    print(json.dumps({"seed": seed, "seconds": budget, "sessions": sessions, "symbols": symbols,
                      "idle_pauses": pauses, "batches_between": batches,
                      "contexts_recreated": recreated, "mismatches": 0}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
