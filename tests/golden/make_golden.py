"""Generates tests/golden/*.json (committed).  Run from the repo root:

    python tests/golden/make_golden.py

kat.json        K1-K3 known-answer vectors of SURVEY.md §8c.  Their expected bytes were derived
                in the survey by two independent scratch restatements (not by running the Rust
                reference, which cannot be built here).  This script asserts that the C oracle
                and the literal Python restatement both reproduce them before writing them.
fixtures.json   small seeded chunks of the C2 (uniform-256), C3 (Zipf 1.2) and C4 (adaptive)
                configurations with their encodings, produced by the oracle once it matched
                the KATs, and cross-checked against oracle/ref_literal.py.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import cpu, ref_literal as R  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def cum_of(c):
    return [int(x) for x in np.concatenate([[0], np.cumsum(c)[:-1]])]


def kats():
    out = []
    # K1: examples/sample_impl.rs:74-81
    counts = [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    data = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]
    out.append(dict(name="K1", c=counts, symbols=data,
                    expect_hex="64475f8970365a2f83b20246c0", expect_len=13))
    # K2: c[i] = 1, total 256, symbols 0..255
    out.append(dict(name="K2", c=[1] * 256, symbols=list(range(256)), expect_len=263,
                    expect_head="00010203040506070506060606060606",
                    expect_tail="0505040302010100", expect_fnv="4e6af22e141a83a7"))
    # K3: c[i] = i + 1, total 32896, symbols (7i + 3) mod 256, i < 1024
    out.append(dict(name="K3", c=[i + 1 for i in range(256)],
                    symbols=[(7 * i + 3) % 256 for i in range(1024)], expect_len=1086,
                    expect_head="000bf775ee7539d30c5f3ac8bc6a61c4",
                    expect_tail="894261225240d700", expect_fnv="d9f9fbff0aaf5a09"))
    for k in out:
        c = k["c"]
        cum = cum_of(c)
        f, b, L = cpu.encode(c, cum, sum(c), k["symbols"])
        lit = R.encode_stream(R.FreqTable.from_counts(c), k["symbols"])
        assert f == 0 and b == lit, k["name"]
        assert len(b) == k["expect_len"], k["name"]
        if "expect_hex" in k:
            assert b.hex() == k["expect_hex"]
        else:
            assert b[:16].hex() == k["expect_head"] and b[-8:].hex() == k["expect_tail"]
            assert "%016x" % cpu.fnv1a64(b) == k["expect_fnv"]
        k["cum"] = cum
        k["total"] = sum(c)
        k["encoded_hex"] = b.hex()
    return out


def fixtures():
    res = []
    seed = 0x5EED0001
    cu, cumu, tu = synth.uniform_table()
    cz, cumz, tz = synth.zipf_table()
    for name, (c, cum, total) in (("C2_uniform256", (cu, cumu, tu)), ("C3_zipf1.2", (cz, cumz, tz))):
        inv = synth.inverse_cdf(c)
        for k in range(4):
            syms = synth.host_chunk(seed, inv, k, 1024)
            f, b, L = cpu.encode(c, cum, total, syms)
            assert f == 0
            if k == 0:  # literal restatement cross-check (slow pure Python)
                assert R.encode_stream(R.FreqTable.from_counts(list(map(int, c))),
                                       list(map(int, syms))) == b
            res.append(dict(config=name, seed=seed, chunk=k, n=1024, c=[int(x) for x in c],
                            total=int(total), symbols_hex=bytes(syms).hex(), encoded_hex=b.hex()))
    inv = synth.inverse_cdf(cz)
    for k in range(4):  # 4096 symbols: long enough for the count halving to trigger
        syms = synth.host_chunk(seed, inv, k, 4096)
        f, b, L = cpu.encode_adaptive(256, 32, 57343, 256, syms)
        assert f == 0
        assert b == R.encode_adaptive_stream(256, 32, 57343, 256, syms.tolist())
        f2, d = cpu.decode_adaptive(256, 32, 57343, 256, b, len(syms))
        assert f2 == 0 and bytes(d) == bytes(syms)
        res.append(dict(config="C4_adaptive", seed=seed, chunk=k, n=4096, inc=32, limit=57343,
                        period=256, n_alpha=256, symbols_hex=bytes(syms).hex(),
                        encoded_hex=b.hex()))
    return res


if __name__ == "__main__":
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    with open(os.path.join(HERE, "fixtures.json"), "w") as f:
        json.dump(fixtures(), f, indent=1)
    print("wrote kat.json, fixtures.json")
