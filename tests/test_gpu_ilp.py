"""The two-chunks-per-lane decoder (k_decode_ilp, rc_decode_ilp.inc) against the CPU oracle.

It decodes small bucket models (2048 < total <= 2^16: the Zipf(1.2) model of configs[2] and
configs[4]) by default in launches of at least one full round of its workgroups; RC_DEC_ILP=2
sends every launch through it, so these tests reach it at small sizes.  Bar: the decoded
symbols and the flags of every chunk equal the oracle's (oracle/rc_oracle.c, which restates
decoder.rs:14-54 and sample_impl.rs:27-45), whatever the two chains of a lane hold: ragged and
empty chunks, a chain whose partner is absent (chunk counts that are not a multiple of the
workgroup's 1,536), misaligned outputs, flagged chunks in either chain, garbage streams, and the
ring fixtures' worst-case byte schedules."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import _native as N, synth  # noqa: E402
from oracle import cpu  # noqa: E402
from gpu_helpers import cum_of, dev, knob_context, run_decode  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
WG2 = 2 * 768  # chunks per workgroup of k_decode_ilp


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _zipf_model(ctx):
    c, cum, total = synth.zipf_table()
    return rc.StaticModel(c, cum, total, ctx=ctx), np.asarray(c), np.asarray(cum), total


def _chunks(rng, c, lens):
    p = c / c.sum()
    return [rng.choice(256, int(L), p=p).astype(np.uint8) for L in lens]


@pytest.mark.parametrize("n_chunks", [1, 2, 769, WG2 + 1, 2 * WG2 - 3])
def test_ilp_ragged_vs_oracle(gpu, monkeypatch, n_chunks):
    rng = np.random.default_rng(n_chunks)
    with knob_context(monkeypatch, RC_DEC_ILP=2) as kc:
        m, c, cum, total = _zipf_model(kc)
        lens = rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 127, 200, 1000, 4099], n_chunks)
        chunks = _chunks(rng, c, lens)
        codes = [cpu.encode(c, cum, total, ch)[1] for ch in chunks]
        dec, fd = run_decode(m, codes, lens, misalign=True, seed=n_chunks)
        for k, ch in enumerate(chunks):
            assert fd[k] == 0 and (dec[k] == ch).all(), k


def test_ilp_equal_lengths_lock_step(gpu, monkeypatch):
    """Equal 4 KiB chunks (the lock-step loop covers everything) and one odd chunk per workgroup
    (its partner finishes alone), outputs 64-B aligned."""
    rng = np.random.default_rng(5)
    with knob_context(monkeypatch, RC_DEC_ILP=2) as kc:
        m, c, cum, total = _zipf_model(kc)
        n = WG2 + 64
        lens = np.full(n, 4096)
        lens[::97] = 4096 + 64 * 3 + 5
        chunks = _chunks(rng, c, lens)
        codes = [cpu.encode(c, cum, total, ch)[1] for ch in chunks]
        dec, fd = run_decode(m, codes, lens)
        assert (fd == 0).all()
        for k, ch in enumerate(chunks):
            assert (dec[k] == ch).all(), k


def test_ilp_flags_and_garbage_vs_oracle(gpu, monkeypatch):
    """Garbage streams decode to the oracle's symbols and flags (corrupt / truncated) in both
    chain positions; streams shorter than 8 bytes are flagged truncated without being read."""
    rng = np.random.default_rng(9)
    with knob_context(monkeypatch, RC_DEC_ILP=2) as kc:
        m, c, cum, total = _zipf_model(kc)
        n = 900  # chains 0 and 1 of the first 132 lanes
        garbage = [rng.integers(0, 256, int(rng.integers(0, 300))).astype(np.uint8).tobytes()
                   for _ in range(n)]
        counts = [int(rng.integers(0, 400)) for _ in garbage]
        dec, fd = run_decode(m, garbage, counts, misalign=True, seed=3)
        for k in range(n):
            f, d = cpu.decode(c, cum, total, garbage[k], counts[k])
            assert fd[k] == f, (k, fd[k], f)
            if f == 0:
                assert (dec[k] == d).all(), k
        assert (fd == N.F_TRUNCATED).any()


def test_ilp_ring_fixtures(gpu, monkeypatch):
    """The directed ring fixtures (range_reduction_expansion at every ring-check offset, code
    at the steered alignments) in both chains of many lanes."""
    with open(os.path.join(HERE, "golden", "ring_fixtures.json")) as f:
        fx = json.load(f)
    with knob_context(monkeypatch, RC_DEC_ILP=2) as kc:
        c = np.array(fx["c"], np.uint32)
        cum = np.array(fx["cum"], np.uint32)
        m = rc.StaticModel(c, cum, fx["total"], ctx=kc)
        chunks = fx["chunks"] * 80
        codes = [bytes.fromhex(ch["encoded_hex"]) for ch in chunks]
        aligns = [ch["align"] for ch in chunks]
        counts = [len(ch["symbols"]) for ch in chunks]
        slot = 64 * ((max(len(x) for x in codes) + 64 + 63) // 64)
        blob = np.zeros(slot * len(codes) + 64, np.uint8)
        coff = np.zeros(len(codes), np.int64)
        for k, (cd, a) in enumerate(zip(codes, aligns)):
            coff[k] = slot * k + a
            blob[coff[k]:coff[k] + len(cd)] = np.frombuffer(cd, np.uint8)
        clen = np.array([len(x) for x in codes], np.int64)
        sym_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        syms = torch.full((int(sym_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        flags = rc.decode_batch(m, dev(blob), dev(coff), dev(clen), syms, dev(sym_off))
        torch.cuda.synchronize()
        s = syms.cpu().numpy()
        assert (flags.cpu().numpy() == 0).all()
        for k, ch in enumerate(chunks):
            assert (s[sym_off[k]:sym_off[k + 1]] == np.array(ch["symbols"], np.uint8)).all(), k


def test_ilp_equals_single_chain_decoder(gpu, monkeypatch):
    """Seeded synthetic 64 KiB Zipf chunks (the bench's generator) encoded on the GPU, decoded
    through both decoders: identical symbols, no flags; the first chunks against the oracle."""
    n, L = 3 * WG2 + 17, 1 << 14
    c, cum, total = synth.zipf_table()
    inv = synth.inverse_cdf(c)
    outs = {}
    for mode in ("2", "0"):
        with knob_context(monkeypatch, RC_DEC_ILP=mode) as kc:
            m = rc.StaticModel(c, cum, total, ctx=kc)
            syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
            synth.fill(kc, 0x5EED0001, inv, syms, L, n)
            cap = rc.slot_capacity(L, 8.0)
            so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
            oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
            out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
            ol, fe = rc.encode_batch(m, syms, so, out, oo)
            dec = torch.empty_like(syms)
            fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
            torch.cuda.synchronize()
            assert int(fe.abs().sum()) == 0 and int(fd.abs().sum()) == 0
            assert torch.equal(dec, syms)
            outs[mode] = dec.cpu().numpy()
            if mode == "2":
                h = out.cpu().numpy()
                lens = ol.cpu().numpy()
                for k in (0, 1, WG2 - 1, WG2, n - 1):
                    f, d = cpu.decode(c, cum, total, bytes(h[k * cap:k * cap + int(lens[k])]), L)
                    assert f == 0 and (d == syms[k * L:(k + 1) * L].cpu().numpy()).all(), k
    assert np.array_equal(outs["2"], outs["0"])
