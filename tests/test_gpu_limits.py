"""Chunk-length limits of the batch kernels (include/range_coder.h RC_MAX_CHUNK_SYMBOLS = 2^25).

The batch kernels keep 32-bit in-chunk stream positions.  A chunk longer than the limit is
flagged RC_F_TOO_LONG before anything of it is read or written: here its symbol range points far
past a small buffer (a fake huge sym_off range), so any read of it would fault and any write
would hit the sentinels.  A chunk of exactly 2^25 symbols is coded, bit-exact vs the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import _native as N, synth  # noqa: E402
from oracle import cpu  # noqa: E402
from gpu_helpers import dev  # noqa: E402

MAX = 1 << 25


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


def _models(ctx):
    uc, ucum, ut = synth.uniform_table()
    zc, zcum, zt = synth.zipf_table()
    wc = np.arange(1, 201, dtype=np.uint32) * 1000  # wide (total > 2^16), magic division
    wcum = np.concatenate([[0], np.cumsum(wc.astype(np.uint64))[:-1]]).astype(np.uint32)
    return {"uniform": rc.StaticModel(uc, ucum, ut), "zipf": rc.StaticModel(zc, zcum, zt),
            "wide": rc.StaticModel(wc, wcum, int(wc.astype(np.uint64).sum())),
            "adaptive": rc.AdaptiveModel(256, **rc.ADAPTIVE_DEFAULTS)}


@pytest.mark.parametrize("kind", ["uniform", "zipf", "wide", "adaptive"])
def test_too_long_chunk_is_flagged_untouched(ctx, kind):
    m = _models(ctx)[kind]
    rng = np.random.default_rng(7)
    alpha = 200 if kind == "wide" else 256
    syms = rng.integers(0, alpha, 300).astype(np.uint8)
    # chunk 2 claims MAX + 1 symbols starting inside a 300-byte buffer
    sym_off = np.array([0, 100, 200, 200 + MAX + 1], np.int64)
    cap = 2048
    out_off = np.arange(4, dtype=np.int64) * cap
    out = torch.full((3 * cap + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    out_len, flags = rc.encode_batch(m, dev(syms), dev(sym_off), out, dev(out_off))
    torch.cuda.synchronize()
    fl, ol, h = flags.cpu().numpy(), out_len.cpu().numpy(), out.cpu().numpy()
    assert fl.tolist() == [0, 0, N.F_TOO_LONG] and ol[2] == 0
    assert (h[2 * cap:] == 0xEE).all()  # the flagged slot and everything after it untouched
    if kind != "adaptive":
        for k in range(2):
            f, b, lb = cpu.encode(m.c, m.cum, m.total, syms[sym_off[k]:sym_off[k + 1]])
            assert f == 0 and lb == ol[k] and bytes(h[out_off[k]:out_off[k] + lb]) == b
    # decode: the flagged chunk's symbol range points past a small output buffer
    code_off = out_off[:3].copy()
    code_len = ol.astype(np.int64).copy()
    code_len[2] = 64
    dec = torch.full((300 + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    fd = rc.decode_batch(m, out, dev(code_off), dev(code_len), dec, dev(sym_off))
    torch.cuda.synchronize()
    d = dec.cpu().numpy()
    assert fd.cpu().numpy().tolist() == [0, 0, N.F_TOO_LONG]
    assert np.array_equal(d[:200], syms[:200]) and (d[200:] == 0xEE).all()


def test_chunk_at_the_limit_round_trips(ctx):
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total)
    inv = synth.inverse_cdf(c)
    syms = torch.empty(MAX, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x1234, inv, syms, MAX, 1)
    sym_off = torch.tensor([0, MAX], dtype=torch.int64, device="cuda")
    cap = rc.slot_capacity(MAX, 8.0)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    out_off = torch.tensor([0, cap], dtype=torch.int64, device="cuda")
    out_len, flags = rc.encode_batch(m, syms, sym_off, out, out_off)
    dec = torch.empty_like(syms)
    fd = rc.decode_batch(m, out, out_off[:1], out_len, dec, sym_off)
    torch.cuda.synchronize()
    assert int(flags[0]) == 0 and int(fd[0]) == 0 and torch.equal(dec, syms)
    hs = syms.cpu().numpy()
    f, b, lb = cpu.encode(c, cum, total, hs, cap=cap)
    assert f == 0 and lb == int(out_len[0]) and bytes(out[:lb].cpu().numpy()) == b


def test_encode_chunks_raises_too_long_before_upload(ctx):
    m = _models(ctx)["uniform"]
    with pytest.raises(rc.ChunkTooLongError):
        rc.encode_chunks(m, [np.zeros(MAX + 1, np.uint8)])


def test_host_stream_too_long_chunk(ctx):
    """rc_encode_host / rc_decode_host: the flagged chunk is staged as empty."""
    m = _models(ctx)["zipf"]
    rng = np.random.default_rng(3)
    syms = np.zeros(200 + MAX + 1, np.uint8)
    syms[:200] = rng.integers(0, 256, 200).astype(np.uint8)
    soff = np.array([0, 100, 200, 200 + MAX + 1], np.uint64)
    ooff = np.array([0, 4096, 8192, 12288], np.uint64)
    out, ol, fl = rc.encode_host(m, syms, soff, ooff)
    assert fl.tolist() == [0, 0, N.F_TOO_LONG] and int(ol[2]) == 0
    dec, fd = rc.decode_host(m, out, ooff[:3], np.array([ol[0], ol[1], 64], np.uint64), soff)
    assert fd.tolist() == [0, 0, N.F_TOO_LONG] and np.array_equal(dec[:200], syms[:200])


@pytest.mark.parametrize("direct", ["1", "0"])
def test_host_stream_too_long_chunk_mid_batch(ctx, knob_ctx, direct):
    """A too-long chunk between in-limit chunks of one batch: its input is not staged and its
    output slot is not overwritten, on the direct (mapped) and staged output paths."""
    zc, zcum, zt = synth.zipf_table()
    m = rc.StaticModel(zc, zcum, zt, ctx=knob_ctx(RC_STREAM_DIRECT=direct))
    rng = np.random.default_rng(4)
    n_big = MAX + 1
    syms = np.zeros(200 + n_big + 300, np.uint8)
    syms[:200] = rng.integers(0, 256, 200).astype(np.uint8)
    syms[200 + n_big:] = rng.integers(0, 256, 300).astype(np.uint8)
    e = 200 + n_big
    soff = np.array([0, 100, 200, e, e + 150, e + 300], np.uint64)
    ooff = np.arange(6, dtype=np.uint64) * 4096
    out = np.full(5 * 4096, 0xEE, np.uint8)
    out, ol, fl = rc.encode_host(m, syms, soff, ooff, out=out)
    assert fl.tolist() == [0, 0, N.F_TOO_LONG, 0, 0] and int(ol[2]) == 0
    assert (out[2 * 4096:3 * 4096] == 0xEE).all()  # the flagged slot untouched
    for k in (0, 1, 3, 4):
        f, b, lb = cpu.encode(m.c, m.cum, m.total, syms[int(soff[k]):int(soff[k + 1])])
        assert f == 0 and lb == int(ol[k]) and bytes(out[int(ooff[k]):int(ooff[k]) + lb]) == b
    code_len = ol.astype(np.uint64).copy()
    code_len[2] = 64
    dec = np.full(len(syms), 0xEE, np.uint8)
    dec, fd = rc.decode_host(m, out, ooff[:5], code_len, soff, out=dec)
    assert fd.tolist() == [0, 0, N.F_TOO_LONG, 0, 0]
    assert np.array_equal(dec[:200], syms[:200]) and np.array_equal(dec[e:], syms[e:])
    assert (dec[200:e] == 0xEE).all()  # the flagged chunk's symbols untouched
