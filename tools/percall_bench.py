"""Per-call cost of the host mirrors (rc.Encoder / rc.Decoder), in microseconds per symbol.

The reference's surface is one Encoder::encode / Decoder::decode call per symbol
(encoder.rs:24-37, decoder.rs:38-54), at CPU speed.  The mirrors keep that surface over the
resumable stream kernels (rc_resume.hip), so their cost per symbol depends on how often a call
needs the GPU:
  static table        encode stages triples (one launch per 2^20 symbols or per result that is
                      asked for); decode runs ahead in doubling blocks: launches are amortised
  caller-adaptive     encode as above (the model is read at the call, staged as a triple);
                      decode: the table changes at every symbol, so every symbol is one launch
                      of one lane plus two pinned PCIe round trips and a 2 x 256-entry table read
  own find_index      decode: one launch per symbol (decoder.rs:40 semantics)
Beside them: the C oracle (oracle/rc_oracle.c, a u64 restatement of the reference) coding the
same static stream on one core, as the stand-in for the reference's own CPU cost per symbol
(Rust is not available here), and the model update each caller-adaptive loop pays in Python.

Usage (GPU box): python3 tools/percall_bench.py [n_static] [n_adaptive]  -> one JSON line
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import range_coder_rust_amd as rc  # noqa: E402
from oracle import cpu  # noqa: E402


class Adaptive(rc.FreqTable):
    """The caller-side adaptive model of tests/test_gpu_stream.py (updated after every symbol)."""

    def __init__(self, n=256, inc=32, limit=57343, period=256):
        super().__init__(n)
        self.c = [1] * n
        self.calc_cum()
        self.inc, self.limit, self.period = inc, limit, period

    def update(self, s, i):
        self.c[s] += self.inc
        if (i + 1) % self.period == 0 and sum(self.c) > self.limit:
            self.c = [(x + 1) >> 1 for x in self.c]
        self.calc_cum()


class OwnFindIndex(rc.FreqTable):
    """find_index overridden (a linear scan: the canonical inverse, found another way)."""

    def find_index(self, decoder):
        r = decoder.range_coder()
        rf = ((decoder.data() - r.lower_bound()) & ((1 << 64) - 1)) // (r.range() // self.total)
        i = 0
        while i + 1 < len(self.c) and self.cum[i + 1] <= rf:
            i += 1
        return i


def us_per(fn, n):
    t0 = time.perf_counter()
    fn()
    return (time.perf_counter() - t0) * 1e6 / n


def main():
    n_static = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    n_adapt = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rng = random.Random(7)
    syms = [min(255, int(rng.paretovariate(1.15)) - 1) for _ in range(n_static)]
    counts = np.bincount(syms, minlength=256) + 1
    table = rc.FreqTable.from_counts([int(x) for x in counts])
    rc.default_context(0)
    res = {"n_static": n_static, "n_adaptive": n_adapt}

    # warm-up (context, staging blocks, first launches)
    e = rc.Encoder()
    for s in syms[:1000]:
        e.encode(table, s)
    d = rc.Decoder(e.finish())
    for _ in range(1000):
        d.decode(table)

    enc = rc.Encoder()

    def run_enc():
        for s in syms:
            enc.encode(table, s)
        res["_code"] = enc.finish()
    res["static_encode_us"] = us_per(run_enc, n_static)
    code = res.pop("_code")
    dec = rc.Decoder(code)
    out = []
    res["static_decode_us"] = us_per(lambda: out.extend(dec.decode(table) for _ in syms),
                                     n_static)
    assert out == syms

    # caller-adaptive (the model update is timed on its own and subtracted)
    asy = syms[:n_adapt]
    m = Adaptive()
    res["adaptive_update_us"] = us_per(lambda: [m.update(s, i) for i, s in enumerate(asy)],
                                       n_adapt)
    m = Adaptive()
    enc = rc.Encoder()

    def run_aenc():
        for i, s in enumerate(asy):
            enc.encode(m, s)
            m.update(s, i)
        res["_code"] = enc.finish()
    res["adaptive_encode_us"] = us_per(run_aenc, n_adapt) - res["adaptive_update_us"]
    acode = res.pop("_code")

    # encode() with its return value read at every call (encoder.rs:34-36): a flush per symbol
    m = Adaptive()
    enc = rc.Encoder()
    cnt = []

    def run_aenc_count():
        for i, s in enumerate(asy):
            cnt.append(int(enc.encode(m, s)))
            m.update(s, i)
        res["_code"] = enc.finish()
    res["adaptive_encode_count_us"] = (us_per(run_aenc_count, n_adapt)
                                       - res["adaptive_update_us"])
    assert res.pop("_code") == acode and sum(cnt) + 8 == len(acode)
    m = Adaptive()
    dec = rc.Decoder(acode)
    got = []

    def run_adec():
        for i in range(n_adapt):
            s = dec.decode(m)
            m.update(s, i)
            got.append(s)
    res["adaptive_decode_us"] = us_per(run_adec, n_adapt) - res["adaptive_update_us"]
    assert got == asy

    own = OwnFindIndex(256)
    own.c = list(table.c)
    own.calc_cum()
    dec = rc.Decoder(code)
    got = []
    res["own_find_index_decode_us"] = us_per(
        lambda: got.extend(dec.decode(own) for _ in range(n_adapt)), n_adapt)
    assert got == syms[:n_adapt]

    # the C oracle, one stream on one core
    c = np.asarray(table.c, np.uint32)
    cum = np.asarray(table.cum, np.uint32)
    a = np.asarray(syms, np.uint8)
    t0 = time.perf_counter()
    f, b, lb = cpu.encode(c, cum, table.total, a)
    t1 = time.perf_counter()
    fl, back = cpu.decode(c, cum, table.total, b, len(a))
    t2 = time.perf_counter()
    assert f == 0 and bytes(b) == bytes(code) and np.array_equal(back, a)
    res["cpu_oracle_encode_us"] = (t1 - t0) * 1e6 / n_static
    res["cpu_oracle_decode_us"] = (t2 - t1) * 1e6 / n_static
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
