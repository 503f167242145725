"""GPU parity of the pipelined host path (rc_stream.hip): rc_encode_host /
rc_decode_host on host-resident numpy arrays against the oracle, byte for byte, across many
small batches (RC_STREAM_BATCH_BYTES lowered), ragged / misaligned / scattered layouts, flagged
chunks, and pageable vs pinned buffers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import cpu  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


@pytest.fixture
def small_batches(knob_ctx):
    """A context whose host pipeline cuts 20,000-byte batches (many batches per call)."""
    return knob_ctx(RC_STREAM_BATCH_BYTES=20000)


def layout(rng, n, lo, hi, gap=False):
    lens = rng.integers(lo, hi + 1, n)
    lens[rng.random(n) < 0.1] = 0
    gaps = rng.integers(0, 40, n) if gap else np.zeros(n, np.int64)
    off = np.zeros(n + 1, np.int64)
    off[0] = int(rng.integers(0, 16)) if gap else 0
    for k in range(n):
        off[k + 1] = off[k] + lens[k] + (gaps[k] if k + 1 < n else 0)
    return lens, off


@pytest.mark.parametrize("gap", [False, True])
def test_encode_host_matches_oracle(ctx, small_batches, gap):
    rng = np.random.default_rng(3 + gap)
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total, ctx=small_batches)
    n = 120
    lens, soff = layout(rng, n, 0, 3000, gap)
    syms = rng.choice(256, int(soff[-1]), p=np.asarray(c, float) / np.sum(c)).astype(np.uint8)
    caps = np.array([rc.slot_capacity(int(L), m.max_bits_per_symbol()) for L in lens])
    ooff = np.concatenate([[int(rng.integers(0, 16)) if gap else 0], caps]).cumsum()
    # chunk k's symbols are [soff[k], soff[k] + lens[k]); with gaps the offsets array has
    # the gap bytes inside chunk k, so encode exactly what the offsets describe
    out, ol, fl = rc.encode_host(m, syms, soff, ooff)
    assert (fl == 0).all()
    for k in range(n):
        ch = syms[soff[k]: soff[k + 1]]
        f, b, L = cpu.encode(c, cum, total, ch)
        assert f == 0 and ol[k] == L and bytes(out[ooff[k]: ooff[k] + L]) == b, k
    # decode from scattered code positions
    counts = np.diff(soff)
    dsoff = np.concatenate([[0], np.cumsum(counts)])
    dec, fd = rc.decode_host(m, out, ooff[:-1], ol, dsoff)
    assert (fd == 0).all()
    assert (dec == syms[soff[0]: soff[-1]]).all()


def test_flags_returned(ctx, small_batches):
    m = rc.StaticModel([1, 5, 2, 0, 2, 2, 1, 1, 1, 1], ctx=small_batches)
    syms = np.array([1, 2, 3, 1, 2, 12], np.uint8)
    soff = np.array([0, 3, 5, 6])
    ooff = np.array([0, 64, 128, 192])
    out, ol, fl = rc.encode_host(m, syms, soff, ooff)
    assert list(fl) == [rc._native.F_ZERO_FREQ, 0, rc._native.F_BAD_SYMBOL]
    f, b, L = cpu.encode([1, 5, 2, 0, 2, 2, 1, 1, 1, 1], [0, 1, 6, 8, 8, 10, 12, 13, 14, 15],
                         16, bytes([1, 2]))
    assert ol[1] == L and bytes(out[64:64 + L]) == b


@pytest.mark.parametrize("pinned", [False, True])
def test_large_round_trip(ctx, pinned):
    n, L = 1200, 65536  # 75 MiB: two batches at the default batch size
    dsyms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    c, cum, total = synth.zipf_table()
    synth.fill(ctx, 21, synth.inverse_cdf(c), dsyms, L, n)
    if pinned:
        hs = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
        hs.copy_(dsyms)
        syms = hs.numpy()
    else:
        syms = dsyms.cpu().numpy()
    m = rc.StaticModel(c, cum, total)
    soff = np.arange(n + 1) * L
    cap = rc.slot_capacity(L, 8.0)
    ooff = np.arange(n + 1) * cap
    out, ol, fl = rc.encode_host(m, syms, soff, ooff)
    ol = ol.astype(np.int64)
    assert (fl == 0).all()
    # same bytes as the device path
    dout = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    dl, df = rc.encode_batch(m, dsyms, torch.from_numpy(soff).cuda(), dout,
                             torch.from_numpy(ooff).cuda())
    assert (dl.cpu().numpy() == ol.astype(np.int64)).all()
    hd = dout.cpu().numpy()
    for k in (0, 1, n // 2, n - 1):
        assert bytes(hd[ooff[k]: ooff[k] + ol[k]]) == bytes(out[ooff[k]: ooff[k] + ol[k]])
    dec, fd = rc.decode_host(m, out, ooff[:-1], ol, soff)
    assert (fd == 0).all() and (dec == syms).all()


def test_cached_pipeline_across_shapes(knob_ctx):
    """The host pipeline is kept with its context: a small call, a larger one (the pipe grows),
    a smaller one again (reused), then rc_ctx_destroy frees it; every call byte-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    own = knob_ctx(RC_STREAM_BATCH_BYTES=50000)
    try:
        c, cum, total = synth.zipf_table()
        m = rc.StaticModel(c, cum, total, ctx=own)
        rng = np.random.default_rng(11)
        p = np.asarray(c, float) / np.sum(c)
        for n, hi in [(7, 500), (90, 4000), (3, 100)]:
            lens, soff = layout(rng, n, 0, hi)
            syms = rng.choice(256, int(soff[-1]), p=p).astype(np.uint8)
            caps = np.array([rc.slot_capacity(int(L), m.max_bits_per_symbol()) for L in lens])
            ooff = np.concatenate([[0], caps]).cumsum()
            out, ol, fl = rc.encode_host(m, syms, soff, ooff)
            assert (fl == 0).all()
            for k in range(n):
                f, b, L = cpu.encode(c, cum, total, syms[soff[k]: soff[k + 1]])
                assert ol[k] == L and bytes(out[ooff[k]: ooff[k] + L]) == b, (n, k)
            dec, fd = rc.decode_host(m, out, ooff[:-1], ol, soff)
            assert (fd == 0).all() and (dec == syms).all(), n
        del m
    finally:
        own.close()


def test_host_multi_device_list_equals_single(ctx):
    """rc_encode_host_multi / rc_decode_host_multi over a list of contexts — here two contexts
    on the one visible device (each with its own streams and pipeline) plus the default one:
    the chunks split three ways give the bytes of one single-device call."""
    c, cum, total = synth.zipf_table()
    inv = synth.inverse_cdf(c)
    n, L = 300, 3000
    syms = np.concatenate([synth.host_chunk(0x77, inv, k, L + (k % 7) * 13) for k in range(n)])
    lens = np.array([L + (k % 7) * 13 for k in range(n)], np.uint64)
    soff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    caps = np.array([rc.slot_capacity(int(x), 8.0) for x in lens], np.uint64)
    ooff = np.concatenate([[0], np.cumsum(caps)]).astype(np.uint64)
    ctxs = [rc.default_context(0), rc.Context(0), rc.Context(0)]
    models = [rc.StaticModel(c, cum, total, ctx=x) for x in ctxs]
    out1, ol1, fl1 = rc.encode_host(models[0], syms, soff, ooff)
    out3, ol3, fl3 = rc.encode_host_multi(models, syms, soff, ooff)
    assert (fl1 == 0).all() and (fl3 == 0).all() and np.array_equal(ol1, ol3)
    for k in range(n):
        assert out1[ooff[k]: ooff[k] + ol1[k]].tobytes() == out3[ooff[k]: ooff[k] + ol3[k]].tobytes()
    dec, fd = rc.decode_host_multi(models, out3, ooff[:-1], ol3, soff)
    assert (fd == 0).all() and np.array_equal(dec, syms)
    for k in (0, n // 2, n - 1):
        f, b, lb = cpu.encode(c, cum, total, syms[soff[k]: soff[k + 1]])
        assert f == 0 and out3[ooff[k]: ooff[k] + lb].tobytes() == b


@pytest.mark.parametrize("dma,direct", [("0", "1"), ("0", "0"), ("1", "1")])
def test_output_copy_paths_on_offset_pinned_buffers(ctx, knob_ctx, dma, direct):
    """Outputs written by the coder straight into mapped host memory (default), staged and moved
    by the copy kernel (RC_STREAM_DIRECT=0), or moved by DMA (RC_STREAM_DMA=1): all byte-exact,
    on pinned buffers used at odd offsets (interior mapped pointers, staging displaced to the
    host address mod 64) across several batches."""
    kc = knob_ctx(RC_STREAM_DMA=dma, RC_STREAM_DIRECT=direct, RC_STREAM_BATCH_BYTES=300000)
    rng = np.random.default_rng(29)
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total, ctx=kc)
    n = 96
    lens, soff = layout(rng, n, 0, 20000, gap=True)
    nsym = int(soff[-1])
    pin_in = torch.empty(nsym + 64, dtype=torch.uint8, pin_memory=True).numpy()
    syms = pin_in[5:5 + nsym]
    syms[:] = rng.choice(256, nsym, p=np.asarray(c, float) / np.sum(c)).astype(np.uint8)
    caps = np.array([rc.slot_capacity(int(L), m.max_bits_per_symbol()) for L in lens])
    ooff = np.concatenate([[0], caps]).cumsum()
    pin_out = torch.empty(int(ooff[-1]) + 64, dtype=torch.uint8, pin_memory=True).numpy()
    out = pin_out[3:3 + int(ooff[-1])]
    out, ol, fl = rc.encode_host(m, syms, soff, ooff, out=out)
    assert (fl == 0).all()
    for k in range(n):
        f, b, L = cpu.encode(c, cum, total, syms[soff[k]: soff[k + 1]])
        assert f == 0 and ol[k] == L and bytes(out[ooff[k]: ooff[k] + L]) == b, k
    pin_dec = torch.empty(nsym - int(soff[0]) + 64, dtype=torch.uint8, pin_memory=True).numpy()
    dsoff = soff - soff[0]
    dec = pin_dec[7:7 + int(dsoff[-1])]
    dec, fd = rc.decode_host(m, out, ooff[:-1], ol, dsoff, out=dec)
    assert (fd == 0).all() and (dec == syms[soff[0]: soff[-1]]).all()


def test_adaptive_model_through_host_path(ctx, knob_ctx):
    """The host pipeline with the adaptive (C4) model: ragged chunks across several batches,
    every stream byte-exact vs the adaptive oracle and the round trip exact."""
    rng = np.random.default_rng(41)
    m = rc.AdaptiveModel(256, 32, 57343, 256, ctx=knob_ctx(RC_STREAM_BATCH_BYTES=40000))
    n = 40
    lens, soff = layout(rng, n, 0, 6000)
    w = 1.0 / np.arange(1, 257) ** 1.2
    syms = rng.choice(256, int(soff[-1]), p=w / w.sum()).astype(np.uint8)
    caps = np.array([rc.slot_capacity(int(L), 16) for L in lens])
    ooff = np.concatenate([[0], caps]).cumsum()
    out, ol, fl = rc.encode_host(m, syms, soff, ooff)
    assert (fl == 0).all()
    for k in range(n):
        f, b, L = cpu.encode_adaptive(256, 32, 57343, 256, syms[soff[k]: soff[k + 1]])
        assert f == 0 and ol[k] == L and bytes(out[ooff[k]: ooff[k] + L]) == b, k
    dec, fd = rc.decode_host(m, out, ooff[:-1], ol, soff)
    assert (fd == 0).all() and (dec == syms).all()
