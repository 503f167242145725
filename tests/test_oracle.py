"""CPU tests of the parity oracle (oracle/rc_oracle.c) — pins it before it is trusted.

The reference's own test is the examples/sample_impl.rs round trip (assert at :123); the
known-answer vectors are SURVEY.md §8c K1-K3; oracle/ref_literal.py is a statement-by-
statement restatement of the Rust used as a second, independent implementation.
"""
import json
import os
import random

import numpy as np
import pytest

from oracle import cpu, ref_literal as R


def cum_of(c):
    return [int(x) for x in np.concatenate([[0], np.cumsum(c)[:-1]])] if len(c) else []


def test_sample_impl_round_trip():
    # examples/sample_impl.rs:72-128: table built by counting the test data (:77-81)
    data = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]
    t = R.FreqTable(10)
    for i in data:
        t.add_alphabet_freq(i)
    t.calc_cum()
    assert t.c == [1, 5, 2, 0, 2, 2, 1, 1, 1, 1] and t.total == 16
    code = R.encode_stream(t, data)
    assert R.decode_stream(t, code, len(data)) == data  # sample_impl.rs:123
    f, b, _ = cpu.encode(t.c, t.cum, t.total, data)
    assert f == 0 and b == code
    f, d = cpu.decode(t.c, t.cum, t.total, b, len(data))
    assert f == 0 and list(d) == data


def test_known_answer_vectors(golden_dir):
    kats = json.load(open(os.path.join(golden_dir, "kat.json")))
    assert [k["name"] for k in kats] == ["K1", "K2", "K3"]
    for k in kats:
        f, b, L = cpu.encode(k["c"], k["cum"], k["total"], k["symbols"])
        assert f == 0
        assert b.hex() == k["encoded_hex"]
        assert L == k["expect_len"]
        if "expect_fnv" in k:
            assert "%016x" % cpu.fnv1a64(b) == k["expect_fnv"]
        f, d = cpu.decode(k["c"], k["cum"], k["total"], b, len(k["symbols"]))
        assert f == 0 and list(d) == k["symbols"]


def test_fixtures(golden_dir):
    fx = json.load(open(os.path.join(golden_dir, "fixtures.json")))
    assert len(fx) == 12
    for e in fx:
        syms = bytes.fromhex(e["symbols_hex"])
        if e["config"] == "C4_adaptive":
            f, b, _ = cpu.encode_adaptive(e["n_alpha"], e["inc"], e["limit"], e["period"], syms)
        else:
            f, b, _ = cpu.encode(e["c"], cum_of(e["c"]), e["total"], syms)
        assert f == 0 and b.hex() == e["encoded_hex"]


def _rand_table(rng, n, total_bits, zero_frac=0.0):
    c = [max(1, int(rng.paretovariate(1.2) * 4)) for _ in range(n)]
    if zero_frac:
        for i in range(n):
            if rng.random() < zero_frac and sum(1 for x in c if x) > 1:
                c[i] = 0
    return c


@pytest.mark.parametrize("seed", range(12))
def test_oracle_matches_literal_restatement(seed):
    rng = random.Random(seed)
    n = rng.choice([1, 2, 3, 10, 17, 64, 255, 256])
    c = _rand_table(rng, n, 16, zero_frac=0.2 if n > 2 else 0.0)
    if rng.random() < 0.3:  # large non-power-of-two totals stress range_par_total
        c = [x * rng.randint(1, 1 << 14) for x in c]
    if sum(c) >= 1 << 32:
        c = [max(1 if x else 0, x >> 8) for x in c]
    nz = [i for i in range(n) if c[i]]
    syms = [rng.choice(nz) for _ in range(rng.randint(0, 600))]
    t = R.FreqTable.from_counts(c)
    lit = R.encode_stream(t, syms)
    f, b, L = cpu.encode(c, t.cum, t.total, syms)
    assert f == 0 and b == lit and L == len(lit)
    assert R.decode_stream(t, lit, len(syms)) == syms
    f, d = cpu.decode(c, t.cum, t.total, b, len(syms))
    assert f == 0 and list(d) == syms


def test_error_flags():
    c = [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    cum = cum_of(c)
    assert cpu.encode(c, cum, 16, [1, 3, 2])[0] == cpu.F_ZERO_FREQ  # reference: infinite loop
    assert cpu.encode(c, cum, 16, [1, 10])[0] == cpu.F_BAD_SYMBOL  # reference: panic
    f, b, L = cpu.encode(c, cum, 16, [1, 2, 4, 5] * 10, cap=5)
    assert f == cpu.F_CAPACITY and len(b) == 5 and L > 5
    f, full, _ = cpu.encode(c, cum, 16, [1, 2, 4, 5] * 10)
    assert full[:5] == b and len(full) == L
    assert cpu.decode(c, cum, 16, full[:7], 1)[0] == cpu.F_TRUNCATED  # Decoder::new panics
    assert cpu.decode(c, cum, 16, full[:-1], 40)[0] == cpu.F_TRUNCATED
    with pytest.raises(R.ReferencePanic):
        R.decode_stream(R.FreqTable.from_counts(c), full[:-1], 40)
    with pytest.raises(R.ReferencePanic):
        R.encode_stream(R.FreqTable.from_counts(c), [3])


def test_empty_stream():
    f, b, L = cpu.encode([1] * 4, [0, 1, 2, 3], 4, [])
    assert f == 0 and b == bytes(8)  # finish() emits the 8 bytes of lower_bound == 0
    assert R.encode_stream(R.FreqTable.from_counts([1] * 4), []) == bytes(8)


def test_batch_threads_match_single():
    rng = np.random.default_rng(1)
    c = np.array([5, 1, 9, 3, 0, 7, 2, 1], dtype=np.uint32)
    cum = np.array(cum_of(c), dtype=np.uint32)
    total = int(c.sum())
    nz = np.nonzero(c)[0]
    lens = rng.integers(0, 300, 37)
    syms = np.concatenate([rng.choice(nz, L).astype(np.uint8) for L in lens])
    so = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    caps = lens * 2 + 16
    oo = np.concatenate([[0], np.cumsum(caps)]).astype(np.uint64)
    out1, ol1, f1 = cpu.encode_batch(c, cum, total, syms, so, oo, threads=1)
    out4, ol4, f4 = cpu.encode_batch(c, cum, total, syms, so, oo, threads=4)
    assert (f1 == 0).all() and (ol1 == ol4).all() and (out1 == out4).all()
    for k in range(len(lens)):
        f, b, _ = cpu.encode(c, cum, total, syms[so[k]:so[k + 1]])
        assert bytes(out1[oo[k]:oo[k] + ol1[k]]) == b
    dec, fd = cpu.decode_batch(c, cum, total, out1, oo[:-1], ol1, so, threads=3)
    assert (fd == 0).all() and (dec == syms).all()


def test_adaptive_round_trip():
    rng = np.random.default_rng(7)
    syms = rng.integers(0, 40, 5000).astype(np.uint8)
    f, b, L = cpu.encode_adaptive(40, 32, 57343, 256, syms)
    assert f == 0
    f, d = cpu.decode_adaptive(40, 32, 57343, 256, b, len(syms))
    assert f == 0 and (d == syms).all()


@pytest.mark.parametrize("n_alpha,inc,limit,period,n", [
    (256, 32, 57343, 256, 3000), (2, 1, 300, 1, 2000), (17, 5, 1000, 4, 2500),
    (1, 7, 600, 8, 300), (256, 255, 255 * 16, 16, 1500)])
def test_adaptive_oracle_matches_literal_restatement(n_alpha, inc, limit, period, n):
    """The C adaptive model against oracle/ref_literal.py's PModel-based restatement."""
    rng = np.random.default_rng(n_alpha * 7 + inc)
    w = 1.0 / np.arange(1, n_alpha + 1) ** 1.1
    syms = rng.choice(n_alpha, size=n, p=w / w.sum()).astype(np.uint8)
    f, b, L = cpu.encode_adaptive(n_alpha, inc, limit, period, syms)
    assert f == 0 and L == len(b)
    assert b == R.encode_adaptive_stream(n_alpha, inc, limit, period, syms.tolist())
    f, d = cpu.decode_adaptive(n_alpha, inc, limit, period, b, n)
    assert f == 0 and (d == syms).all()
    assert R.decode_adaptive_stream(n_alpha, inc, limit, period, b, n) == syms.tolist()
    # a truncated stream is flagged where the literal restatement panics
    f, _ = cpu.decode_adaptive(n_alpha, inc, limit, period, b[:-1], n)
    with pytest.raises(R.ReferencePanic):
        R.decode_adaptive_stream(n_alpha, inc, limit, period, b[:-1], n)
    assert f == 8  # RC_F_TRUNCATED
