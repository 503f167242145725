"""cProfile of the Python mirror's caller-adaptive Decoder.decode loop (tools/percall_bench.py's
Adaptive model), to see where a call's host time goes beside the GPU round trip (GPU box)."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import percall_bench as pb  # noqa: E402
import range_coder_rust_amd as rc  # noqa: E402


def main():
    rng = np.random.default_rng(3)
    syms = [int(x) for x in rng.integers(0, 256, 3000)]
    m = pb.Adaptive()
    enc = rc.Encoder()
    for i, s in enumerate(syms):
        enc.encode(m, s)
        m.update(s, i)
    code = enc.finish()
    for rep in range(2):
        m = pb.Adaptive()
        dec = rc.Decoder(code)
        pr = cProfile.Profile() if rep else None
        if pr:
            pr.enable()
        for i in range(len(syms)):
            s = dec.decode(m)
            m.update(s, i)
        if pr:
            pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(15)
    print(out.getvalue())


if __name__ == "__main__":
    main()
