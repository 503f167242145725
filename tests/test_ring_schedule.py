"""The static decoder's code-ring schedule on the host (tests/ring_sim.py replays
k_decode_static's refills and checks, rc_decode.inc): the round-4 schedule never reads a code byte
before it is staged nor overwrites one before it is read, on the directed ring fixtures
(tests/golden/ring_fixtures.json, steered to the tightest rings after range_reduction_expansion)
and on random streams; and the byte bound the schedule rests on (over any s
symbols of a model with total <= 2^16, no_carry_expansion settles at most 2 s + 2 bytes)."""
import json
import os

import numpy as np
import pytest

from oracle import cpu
import ring_sim

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ring_fx():
    with open(os.path.join(HERE, "golden", "ring_fixtures.json")) as f:
        return json.load(f)


def test_ring_fixtures_match_oracle(ring_fx):
    c, cum, total = ring_fx["c"], ring_fx["cum"], ring_fx["total"]
    for k, ch in enumerate(ring_fx["chunks"]):
        f, code, _ = cpu.encode(c, cum, total, ch["symbols"])
        assert f == 0 and code.hex() == ch["encoded_hex"], k
        f, d = cpu.decode(c, cum, total, code, len(ch["symbols"]))
        assert f == 0 and list(d) == ch["symbols"], k
        km = ring_sim.settle(c, cum, total, ch["symbols"])
        assert 8 + sum(a + b for a, b in km) == len(code)
        assert [i for i, (_, m) in enumerate(km) if m] == ch["rare_at"]


def test_ring_fixtures_cover_every_span_offset(ring_fx):
    offs = {i % ring_sim.DEC_CHECK_SPAN for ch in ring_fx["chunks"] for i in ch["rare_at"]}
    assert offs == set(range(ring_sim.DEC_CHECK_SPAN))
    assert {ch["align"] for ch in ring_fx["chunks"]} >= {0, 1, 31, 33, 63}


@pytest.mark.parametrize("head", [0, 1, 15, 16, 63])
def test_round4_schedule_on_ring_fixtures(ring_fx, head):
    c, cum, total = ring_fx["c"], ring_fx["cum"], ring_fx["total"]
    for k, ch in enumerate(ring_fx["chunks"]):
        km = ring_sim.settle(c, cum, total, ch["symbols"])
        under, over = ring_sim.replay(km, ch["align"], head)
        assert not under and not over, (k, under, over)
        if head == 0:
            assert under == ch["underruns_r4"]


def _models(rng):
    out = []
    for total in (256, 4096, 32768, 65536):
        c = np.ones(256, np.int64)
        c[0] = total - 255
        out.append(("rare-heavy", c, total))
    for total in (256, 65536):
        out.append(("uniform", np.full(256, total // 256, np.int64), total))
    w = 1.0 / np.arange(1, 257) ** 1.2
    c = np.maximum(1, np.floor(w / w.sum() * 65536)).astype(np.int64)
    c[0] += 65536 - int(c.sum())
    out.append(("zipf", c, 65536))
    return out


@pytest.mark.parametrize("seed", range(3))
def test_round4_schedule_on_random_streams(seed):
    rng = np.random.default_rng(seed)
    for name, c, total in _models(rng):
        cum = np.concatenate([[0], np.cumsum(c)[:-1]])
        for _ in range(6):
            n = int(rng.integers(1, 700))
            if name == "rare-heavy":
                syms = rng.integers(1, 256, n)
                syms[rng.random(n) < 0.1] = 0
            else:
                p = c / c.sum()
                syms = rng.choice(256, n, p=p)
            km = ring_sim.settle(c, cum, total, syms)
            for head in (0, int(rng.integers(1, 64))):
                under, over = ring_sim.replay(km, int(rng.integers(0, 64)), head)
                assert not under and not over, (name, n, head, under, over)


@pytest.mark.parametrize("total", [256, 4096, 65536])
def test_no_carry_bytes_bound(ring_fx, total):
    """Over any window of s symbols, no_carry_expansion settles at most 2 s + 2 bytes when
    total <= 2^16 (the range grows by at most 2^64 / 2^48 across the window and each symbol
    narrows it by at most total / c <= 2^16; a range_reduction_expansion only raises it).  The
    ring checks rest on this: 8-symbol spans stage 24 >= 18 bytes, and the rare path stages its
    m bytes plus 24 >= 16 for the at most 7 symbols left in its span."""
    rng = np.random.default_rng(total)
    streams = []
    c = np.ones(256, np.int64)
    c[0] = total - 255
    cum = np.concatenate([[0], np.cumsum(c)[:-1]])
    for _ in range(8):
        syms = rng.integers(1, 256, 2000)
        syms[rng.random(2000) < 0.05] = 0
        streams.append(ring_sim.settle(c, cum, total, syms))
    if total == ring_fx["total"]:
        streams += [ring_sim.settle(ring_fx["c"], ring_fx["cum"], total, ch["symbols"])
                    for ch in ring_fx["chunks"]]
    worst = 0
    for km in streams:
        k = np.array([a for a, _ in km])
        cs = np.concatenate([[0], np.cumsum(k)])
        for s in range(1, 9):
            w = cs[s:] - cs[:-s]
            assert w.max() <= 2 * s + 2, (s, int(w.max()))
            worst = max(worst, int(w.max()) - 2 * s)
    assert worst <= 2
