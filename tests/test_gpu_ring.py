"""The static decoder's code ring on the GPU: the directed ring fixtures
(tests/golden/ring_fixtures.json, made by tests/golden/make_ring_fixtures.py) put a
range_reduction_expansion at every offset of the 8-symbol ring-check span, each followed by the
symbols that settle the most bytes, with the code streams at the alignments the fixtures were
steered for (the decoder's 64-B load bursts start on 64-B boundaries).  Every decoder variant of
the model (pair buckets at both workgroup sizes, and the bucket decoder) must return the
fixture's symbols with no flag, also with the output misaligned (a head of single symbols).

Run against a scratch `-DRC_RING_GUARD` library (RC_LIB_PATH, tools/ring_guard.py), the same
assertions show that no symbol read a code byte its ring had not staged: the guard flag would
make the chunk's flags non-zero."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from oracle import cpu  # noqa: E402
from gpu_helpers import dev  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


@pytest.fixture(scope="module")
def ring_fx():
    with open(os.path.join(HERE, "golden", "ring_fixtures.json")) as f:
        return json.load(f)


def _decode_at(m, chunks, head, reps=1):
    """Code stream k at its fixture alignment mod 64 inside 64-B slots; decoded output at
    `head` bytes past a 64-B boundary (plus 64-B aligned chunk strides)."""
    codes = [bytes.fromhex(ch["encoded_hex"]) for ch in chunks] * reps
    aligns = [ch["align"] for ch in chunks] * reps
    counts = [len(ch["symbols"]) for ch in chunks] * reps
    slot = 64 * ((max(len(c) for c in codes) + 64 + 63) // 64)
    blob = np.zeros(slot * len(codes) + 64, np.uint8)
    coff = np.zeros(len(codes), np.int64)
    for k, (c, a) in enumerate(zip(codes, aligns)):
        coff[k] = slot * k + a
        blob[coff[k]:coff[k] + len(c)] = np.frombuffer(c, np.uint8)
    clen = np.array([len(c) for c in codes], np.int64)
    # every fixture holds the same count (a multiple of 64): contiguous outputs keep every
    # chunk's output at `head` past a 64-B boundary
    assert len(set(counts)) == 1 and counts[0] % 64 == 0
    sym_off = np.arange(len(codes) + 1, dtype=np.int64) * counts[0] + head
    syms = torch.full((int(sym_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    flags = rc.decode_batch(m, dev(blob), dev(coff), dev(clen), syms, dev(sym_off))
    torch.cuda.synchronize()
    s = syms.cpu().numpy()
    return s, sym_off, flags.cpu().numpy()


@pytest.mark.parametrize("pair", ["512", "1024", "0"])
@pytest.mark.parametrize("head", [0, 5, 48])
def test_ring_fixtures_decode(ctx, ring_fx, knob_ctx, pair, head):
    c = np.array(ring_fx["c"], np.uint32)
    cum = np.array(ring_fx["cum"], np.uint32)
    chunks = ring_fx["chunks"]
    m = rc.StaticModel(c, cum, ring_fx["total"], ctx=knob_ctx(RC_DEC_PAIR=pair))
    s, sym_off, flags = _decode_at(m, chunks, head)
    assert (flags == 0).all(), flags
    assert (s[:head] == 0xEE).all() and (s[sym_off[-1]:] == 0xEE).all()
    for k, ch in enumerate(chunks):
        got = s[sym_off[k]:sym_off[k + 1]]
        assert (got == np.array(ch["symbols"], np.uint8)).all(), (pair, head, k)


def test_ring_fixtures_full_waves(ctx, ring_fx, knob_ctx):
    """Every fixture in many lanes at once (whole workgroups of the bucket decoder, LUT 4: the
    fixtures' model, total 2^16, has 2^12 buckets and so runs 512-lane workgroups, the variant
    2^20-chunk launches of this model take), against the oracle's decode."""
    c = np.array(ring_fx["c"], np.uint32)
    cum = np.array(ring_fx["cum"], np.uint32)
    total = ring_fx["total"]
    chunks = ring_fx["chunks"]
    m = rc.StaticModel(c, cum, total, ctx=knob_ctx(RC_DEC_PAIR="0"))
    s, sym_off, flags = _decode_at(m, chunks, 0, reps=64)
    assert (flags == 0).all()
    for k in range(len(flags)):
        ch = chunks[k % len(chunks)]
        f, d = cpu.decode(c, cum, total, bytes.fromhex(ch["encoded_hex"]), len(ch["symbols"]))
        assert f == 0
        assert (s[sym_off[k]:sym_off[k + 1]] == d).all(), k
