"""Stream-service soak (GPU box): many short per-call sessions through the Python mirror with a
caller-adaptive model, with pauses that cross the service wave's idle exit (5 ms) and contexts
destroyed and recreated, for a time budget.  Every session encodes a random symbol string with
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
from oracle import cpu  # noqa: E402


def session(rng, ctx):
    n = rng.choice([1, 2, 5, 40, rng.randint(1, 400)])
    syms = [min(255, int(rng.paretovariate(1.1)) - 1) for _ in range(n)]
    m = pb.Adaptive()
    enc = rc.Encoder(ctx)
    trip = []
    for i, s in enumerate(syms):
        trip.append((m.c_freq(s), m.cum_freq(s), m.total_freq()))
        b = enc.encode(m, s)
        if rng.random() < 0.2:
            int(b)  # encode()'s return value now: a flush of the staged symbols
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
        m.update(s, i)
    return n, None


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    rng = random.Random(seed)
    t_end = time.time() + budget
    ctx = rc.Context(0)
    sessions = symbols = pauses = recreated = 0
    t_print = time.time()
    while time.time() < t_end:
        n, bad = session(rng, ctx)
        sessions += 1
        symbols += n
        if bad:
            print(json.dumps({"mismatch": bad, "session": sessions, "seed": seed}))
            return 1
        r = rng.random()
        if r < 0.3:  # past the wave's 5-ms idle exit: the next call starts a new wave
            time.sleep(rng.uniform(0.004, 0.012))
            pauses += 1
        elif r < 0.35:  # destroy the context (stops its wave) and start over
            ctx.close()
            ctx = rc.Context(0)
            recreated += 1
        if time.time() - t_print > 5:
            print(f"{sessions} sessions, {symbols} symbols, {pauses} idle pauses, "
                  f"{recreated} contexts recreated", flush=True)
            t_print = time.time()
    print(json.dumps({"seed": seed, "seconds": budget, "sessions": sessions, "symbols": symbols,
                      "idle_pauses": pauses, "contexts_recreated": recreated, "mismatches": 0}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
