"""k_encode_static (rc_encode.hip) against the oracle, one battery per model class: wide, small,
small and complete; power-of-two and magic totals; the headline uniform model and a rare-heavy
one (range_reduction_expansion back to back).  Ragged and misaligned chunks, the reference's
errors (the first one wins), capacity overflow (the exact length, nothing written past the
slot), and the decoder's directed ring fixtures, whose streams the encoder must reproduce.
(Round 4 ran the same battery on a split coder-wave / output-wave encoder before measuring it
slower)"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from oracle import cpu  # noqa: E402
from gpu_helpers import cum_of, run_encode  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


def _models(rng):
    out = []
    # wide (total > 2^16), magic division
    c = rng.integers(1, 1 << 22, 256).astype(np.uint32)
    out.append(("wide", c))
    # small, pow2 total, complete (SM == 2)
    w = 1.0 / np.arange(1, 257) ** 1.2
    c = np.maximum(1, np.floor(w / w.sum() * 65536)).astype(np.int64)
    c[0] += 65536 - int(c.sum())
    out.append(("zipf", c.astype(np.uint32)))
    # small, magic total, with zero frequencies (SM == 1)
    c = rng.integers(1, 300, 200).astype(np.uint32)
    c[rng.random(200) < 0.1] = 0
    c[0] = max(int(c[0]), 1)
    out.append(("small-zeros", c))
    # uniform 256 (the headline model)
    out.append(("uniform", np.ones(256, np.uint32)))
    # rare-heavy: c = 1 symbols of a 2^16 total
    c = np.ones(256, np.uint32)
    c[0] = 65536 - 255
    out.append(("rare-heavy", c))
    return out


@pytest.mark.parametrize("misalign", [False, True])
def test_encoder_vs_oracle(ctx, misalign):
    rng = np.random.default_rng(5 + misalign)
    for name, c in _models(rng):
        cum = cum_of(c)
        total = int(c.astype(np.uint64).sum())
        m = rc.StaticModel(c, cum, total)
        nz = np.nonzero(c)[0]
        lens = [int(x) for x in rng.choice([0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 100, 257,
                                            1000, 4099, 20000], 150)]
        if name == "rare-heavy":
            chunks = []
            for L in lens:
                ch = rng.integers(1, 256, L)
                ch[rng.random(L) < 0.05] = 0
                chunks.append(ch.astype(np.uint8))
        else:
            p = c[nz] / c[nz].sum()
            chunks = [rng.choice(nz, L, p=p).astype(np.uint8) for L in lens]
        caps = [rc.slot_capacity(L, m.max_bits_per_symbol() + 1) for L in lens]
        out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=misalign, seed=len(name))
        for k, ch in enumerate(chunks):
            f, b, L = cpu.encode(c, cum, total, ch)
            assert (fl[k], ol[k]) == (f, L), (name, k, fl[k], f, ol[k], L)
            assert bytes(out[out_off[k]: out_off[k] + ol[k]]) == b, (name, k)


def test_encoder_errors_and_capacity(ctx):
    """Zero-frequency and out-of-alphabet symbols (the first error wins) and slots too small for
    the stream (RC_F_CAPACITY with the exact length, nothing written past the slot)."""
    rng = np.random.default_rng(17)
    for total_kind in ("small", "wide"):
        if total_kind == "small":
            c = rng.integers(1, 400, 200).astype(np.uint32)
        else:
            c = rng.integers(1, 1 << 20, 200).astype(np.uint32)
        c[[5, 77, 150]] = 0
        total = int(c.astype(np.uint64).sum())
        cum = cum_of(c)
        m = rc.StaticModel(c, cum, total)
        good = [i for i in range(200) if c[i]]
        chunks, caps = [], []
        for k in range(96):
            ch = rng.choice(good, size=int(rng.integers(1, 3000))).astype(np.uint8)
            kind = k % 6
            if kind == 1:
                ch[len(ch) // 2] = 77
            elif kind == 2:
                ch[len(ch) // 3] = 230
            chunks.append(ch)
            cap = rc.slot_capacity(len(ch), 24)
            if kind == 3:
                cap = int(rng.integers(0, 40))  # overflow
            caps.append(cap)
        out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=k)
        for k, ch in enumerate(chunks):
            f, want, L = cpu.encode(c, cum, total, ch)
            if f == 0 and L > caps[k]:
                f = rc.api.N.F_CAPACITY
            assert fl[k] == f, (total_kind, k, fl[k], f)
            if f in (0, rc.api.N.F_CAPACITY):  # the exact length either way
                assert ol[k] == L, (total_kind, k)
            if f == 0:
                assert bytes(out[out_off[k]:out_off[k] + L]) == want, (total_kind, k)


def test_encoder_on_ring_fixtures(ctx):
    """The decoder's directed ring fixtures (rare paths at every span offset, 3-byte symbols
    after them) encode to their recorded streams."""
    with open(os.path.join(HERE, "golden", "ring_fixtures.json")) as f:
        fx = json.load(f)
    c = np.array(fx["c"], np.uint32)
    m = rc.StaticModel(c, cum_of(c), fx["total"])
    chunks = [np.array(ch["symbols"], np.uint8) for ch in fx["chunks"]] * 8
    caps = [rc.slot_capacity(len(ch), 24) for ch in chunks]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=9)
    for k in range(len(chunks)):
        want = bytes.fromhex(fx["chunks"][k % len(fx["chunks"])]["encoded_hex"])
        assert fl[k] == 0 and ol[k] == len(want), k
        assert bytes(out[out_off[k]:out_off[k] + ol[k]]) == want, k


@pytest.mark.parametrize("name", ["zipf", "uniform"])
def test_capacity_end_mid_stream_with_busy_flush_rounds(ctx, name):
    """Slots that end deep inside their streams, on 320 ragged chunks (five waves, so each flush
    round ranks many ready chunks, rc_encode.hip enc_round): RC_F_CAPACITY with the exact
    length, and the slot holds the oracle stream's first cap bytes (encoder.rs:24-46).  The
    slots are adjacent and misaligned, so a byte written past a slot's end would show in the
    next slot's bytes."""
    rng = np.random.default_rng(29)
    if name == "zipf":
        w = 1.0 / np.arange(1, 257) ** 1.2
        c = np.maximum(1, np.floor(w / w.sum() * 65536)).astype(np.int64)
        c[0] += 65536 - int(c.sum())
        c = c.astype(np.uint32)
    else:
        c = np.ones(256, np.uint32)
    total = int(c.astype(np.uint64).sum())
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, total)
    p = c / c.sum()
    chunks = [rng.choice(256, size=int(rng.integers(2000, 9000)), p=p).astype(np.uint8)
              for _ in range(320)]
    want = [cpu.encode(c, cum, total, ch) for ch in chunks]
    caps = []
    for k, (f, b, L) in enumerate(want):
        assert f == 0
        caps.append(int(rng.integers(L // 4, L)) if k % 2 else L + int(rng.integers(0, 80)))
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=31)
    for k, (f, b, L) in enumerate(want):
        assert ol[k] == L, (name, k)
        if caps[k] < L:
            assert fl[k] == rc.api.N.F_CAPACITY, (name, k, fl[k])
            assert bytes(out[out_off[k]:out_off[k] + caps[k]]) == b[:caps[k]], (name, k)
        else:
            assert fl[k] == 0, (name, k, fl[k])
            assert bytes(out[out_off[k]:out_off[k] + L]) == b, (name, k)
