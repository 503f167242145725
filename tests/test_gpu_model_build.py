"""GPU parity of model construction: rc_histogram against numpy
counts (exact integers), build_model's table against the oracle quantizer, rc_ideal_bits
against oracle/model_build.ideal_bits (f64; relative tolerance 1e-12: the GPU accumulates four
bins per lane with fma and adds the 64 lanes by a butterfly, the oracle adds in bin order with
separate multiply and add; 256 positive terms stay within ~3e-14 either way)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import model_build as O  # noqa: E402
from gpu_helpers import dev  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


def ragged(rng, n, lo, hi, base=0, zipf=False):
    lens = rng.integers(lo, hi + 1, n)
    lens[rng.random(n) < 0.1] = 0  # empty chunks
    tot = int(lens.sum())
    if zipf:
        c, _, _ = synth.zipf_table()
        data = rng.choice(256, tot + base, p=np.asarray(c, float) / np.sum(c)).astype(np.uint8)
    else:
        data = rng.integers(0, 256, tot + base).astype(np.uint8)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + base
    return data, off


@pytest.mark.parametrize("base", [0, 3, 13])
@pytest.mark.parametrize("zipf", [False, True])
def test_histogram_matches_numpy(ctx, base, zipf):
    rng = np.random.default_rng(base + 10 * zipf)
    data, off = ragged(rng, 300, 0, 5000, base, zipf)
    hist, ch = rc.histogram(dev(data), dev(off), per_chunk=True)
    torch.cuda.synchronize()
    ch = ch.cpu().numpy()
    for k in range(len(off) - 1):
        want = np.bincount(data[off[k]:off[k + 1]], minlength=256)
        assert (ch[k] == want).all(), k
    assert (hist.cpu().numpy() == np.bincount(data[off[0]:off[-1]], minlength=256)).all()


def test_histogram_large_chunks_and_accumulation(ctx):
    n, L = 2048, 65536
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    c, _, _ = synth.zipf_table()
    synth.fill(ctx, 0x5EED0001, synth.inverse_cdf(c), syms, L, n)
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    hist, ch = rc.histogram(syms, off, per_chunk=True)
    want = torch.bincount(syms, minlength=256)
    assert torch.equal(hist, want.to(torch.int64))
    assert torch.equal(ch.sum(0, dtype=torch.int64), want.to(torch.int64))
    assert int(ch.sum(1).min()) == L and int(ch.sum(1).max()) == L
    # hist accumulates: a second call adds
    h2 = hist.clone()
    ctx._lib.rc_histogram(ctx.handle, rc.api._ptr(syms), rc.api._ptr(off), n, None,
                          rc.api._ptr(h2))
    torch.cuda.synchronize()
    assert torch.equal(h2, 2 * hist)


def _data(rng, kind, tot):
    if kind == "uniform":
        return rng.integers(0, 256, tot).astype(np.uint8)
    if kind == "zipf":
        c, _, _ = synth.zipf_table()
        return rng.choice(256, tot, p=np.asarray(c, float) / np.sum(c)).astype(np.uint8)
    if kind == "constant":  # every symbol of every lane into one u16 counter
        return np.full(tot, 0xA7, np.uint8)
    # bins b and b + 128 share a counter dword (low and high halves)
    return np.where(rng.random(tot) < 0.5, 0x05, 0x85).astype(np.uint8)


def _check_hist(data, off):
    hist, ch = rc.histogram(dev(data), dev(off), per_chunk=True)
    torch.cuda.synchronize()
    ch = ch.cpu().numpy()
    for k in range(len(off) - 1):
        want = np.bincount(data[off[k]:off[k + 1]], minlength=256)
        assert (ch[k] == want).all(), k
    want_all = np.bincount(data[off[0]:off[-1]], minlength=256)
    assert (hist.cpu().numpy() == want_all).all()
    hist_only, _ = rc.histogram(dev(data), dev(off), per_chunk=False)
    assert (hist_only.cpu().numpy() == want_all).all()


@pytest.mark.parametrize("base", [0, 7])
@pytest.mark.parametrize("kind", ["uniform", "zipf", "constant", "pair"])
def test_histogram_skewed_and_paired_bins(ctx, base, kind):
    """k_histogram's u16 sub-histograms: ragged chunks with unaligned starts, data that puts
    every symbol into one counter, and two bins sharing one counter dword."""
    rng = np.random.default_rng(base + 100 * len(kind))
    lens = rng.integers(0, 70000, 90)
    lens[::9] = 0
    tot = int(lens.sum()) + base
    data = _data(rng, kind, tot)
    _check_hist(data, np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + base)


@pytest.mark.parametrize("kind", ["constant", "pair", "zipf"])
def test_histogram_multi_segment_chunks(ctx, kind):
    """Chunks longer than one counting segment (256 x 8176 symbols, ~2 MiB): the u16 counters
    are read out and cleared between segments, so even a one-symbol chunk of 5 MiB is exact."""
    rng = np.random.default_rng(len(kind))
    seg = 256 * 8176
    lens = np.array([seg - 1, seg, seg + 1, 2 * seg + 17, 5 << 20, 3, 0, seg + 15], np.int64)
    base = 5
    tot = int(lens.sum()) + base
    data = _data(rng, kind, tot)
    _check_hist(data, np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + base)


@pytest.mark.parametrize("T,all_symbols", [(0, False), (1 << 16, True), (4096, False),
                                           (1 << 20, True)])
def test_build_model_table_and_round_trip(ctx, T, all_symbols):
    rng = np.random.default_rng(T)
    data, off = ragged(rng, 64, 100, 3000, 5, zipf=True)
    m = rc.build_model(dev(data), dev(off), target_total=T, all_symbols=all_symbols)
    want = O.quantize_counts(np.bincount(data[off[0]:off[-1]], minlength=256), T,
                             O.Q_ALL_SYMBOLS if all_symbols else 0)
    assert list(m.c) == want[0] and list(m.cum) == want[1] and m.total == want[2]
    chunks = [bytes(data[off[k]:off[k + 1]]) for k in range(len(off) - 1)]
    codes = rc.encode_chunks(m, chunks)
    dec = rc.decode_chunks(m, codes, [len(x) for x in chunks])
    assert all(bytes(d) == x for d, x in zip(dec, chunks))


def test_sample_freqtable_built_on_gpu(ctx):
    # examples/sample_impl.rs:74-90: the FreqTable of the test data, from the GPU histogram
    data = np.array([2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5], np.uint8)
    m = rc.build_model(dev(data), dev(np.array([0, 16], np.int64)), target_total=0,
                       n_symbols=10, all_symbols=False)
    assert list(m.c) == [1, 5, 2, 0, 2, 2, 1, 1, 1, 1] and m.total == 16
    code = rc.encode_chunks(m, [bytes(data)])[0]
    assert code.hex() == "64475f8970365a2f83b20246c0"  # K1


@pytest.mark.parametrize("n", [1, 255, 256, 1000])
def test_ideal_bits_matches_oracle(ctx, n):
    rng = np.random.default_rng(n)
    data, off = ragged(rng, n, 0, 2000, 0, zipf=True)
    _, ch = rc.histogram(dev(data), dev(off), per_chunk=True, batch=False)
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total)
    bits = rc.ideal_bits(m, ch).cpu().numpy()
    want = O.ideal_bits(ch.cpu().numpy(), list(c), total)
    np.testing.assert_allclose(bits, want, rtol=1e-12, atol=0)


def test_ideal_bits_inf_for_zero_frequency(ctx):
    c = np.array([1, 5, 2, 0, 2, 2, 1, 1, 1, 1], np.uint32)
    m = rc.StaticModel(c)
    h = np.zeros((3, 256), np.int32)
    h[0, :10] = 1
    h[0, 3] = 0
    h[1, 3] = 2   # c == 0
    h[2, 12] = 1  # outside the alphabet
    bits = rc.ideal_bits(m, dev(h)).cpu().numpy()
    assert abs(bits[0] - sum(math.log2(16 / x) for x in c if x)) < 1e-12
    assert math.isinf(bits[1]) and math.isinf(bits[2])


def test_code_length_vs_ideal(ctx):
    # the entropy report: coded bytes against the ideal code length of the same model
    n, L = 256, 65536
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    c, cum, total = synth.zipf_table()
    synth.fill(ctx, 7, synth.inverse_cdf(c), syms, L, n)
    off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    m = rc.StaticModel(c, cum, total)
    _, ch = rc.histogram(syms, off, per_chunk=True, batch=False)
    ideal = rc.ideal_bits(m, ch)
    cap = rc.slot_capacity(L, 8.0)
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    out_len, fl = rc.encode_batch(m, syms, off, out,
                                  torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap)
    over = (out_len.double() * 8 - ideal).cpu().numpy()
    # a range coder with 64-bit state pays its 8-byte flush plus a few bits per chunk
    assert (over > 0).all() and (over < 64 + 0.01 * L).all()
