"""GPU parity tests: the HIP kernels (librc_amd.so, through the C ABI) against the CPU oracle.

Bar: bit-exact bytes, lengths and flags for every chunk (integer/byte work).  Small cases are
compared chunk by chunk with oracle/rc_oracle.c; full-size cases use encode -> decode round
trips plus a seeded sample of chunks checked against the oracle.
"""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import cpu  # noqa: E402
from gpu_helpers import cum_of, dev, run_decode, run_encode  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


# ----------------------------------------------------------------------------- tests
def test_known_answer_vectors_gpu(ctx):
    kats = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))
    for k in kats:
        m = rc.StaticModel(k["c"], k["cum"], k["total"])
        code = rc.encode_chunks(m, [bytes(k["symbols"])])[0]
        assert code.hex() == k["encoded_hex"], k["name"]
        dec = rc.decode_chunks(m, [code], [len(k["symbols"])])[0]
        assert list(dec) == k["symbols"], k["name"]


def test_sample_impl_gpu(ctx):
    """examples/sample_impl.rs:72-128 through the mirrored Encoder/Decoder/FreqTable API."""
    test_data = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]
    sd = rc.FreqTable(10)
    for i in test_data:
        sd.add_alphabet_freq(i)
    sd.calc_cum()
    encoder = rc.Encoder()
    for i in test_data:
        encoder.encode(sd, i)
    code = encoder.finish()
    assert code.hex() == "64475f8970365a2f83b20246c0"
    decoder = rc.Decoder(code, len(test_data))
    decodeds = [decoder.decode(sd) for _ in test_data]
    assert decodeds == test_data


def test_fixtures_gpu(ctx):
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")))
    for e in fx:
        if e["config"] == "C4_adaptive":
            continue
        m = rc.StaticModel(e["c"], None, e["total"])
        syms = bytes.fromhex(e["symbols_hex"])
        code = rc.encode_chunks(m, [syms])[0]
        assert code.hex() == e["encoded_hex"]
        assert bytes(rc.decode_chunks(m, [code], [len(syms)])[0]) == syms


def _random_model(rng, kind):
    n = int(rng.choice([1, 2, 3, 7, 10, 64, 200, 255, 256]))
    if kind == "pow2":
        bits = int(rng.integers(max(1, int(np.ceil(np.log2(n)))), 17))
        total = 1 << bits
        w = rng.pareto(1.1, n) + 0.05
        c = np.maximum(1, np.floor(w / w.sum() * total)).astype(np.int64)
        c[int(np.argmax(c))] += total - c.sum()
        if c.min() < 1:
            c = np.ones(n, np.int64)
            c[0] += total - n
    elif kind == "big":
        c = rng.integers(1, 1 << 23, n)
    else:
        c = rng.integers(1, 300, n)
    c = c.astype(np.int64)
    if n > 2 and kind != "pow2":
        z = rng.random(n) < 0.15
        z[int(np.argmax(c))] = False
        c[z] = 0
    return c.astype(np.uint32)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("kind", ["pow2", "small", "big"])
def test_random_models_vs_oracle(ctx, seed, kind):
    rng = np.random.default_rng(1000 * seed + {"pow2": 1, "small": 2, "big": 3}[kind])
    c = _random_model(rng, kind)
    cum = cum_of(c)
    total = int(c.astype(np.uint64).sum())
    m = rc.StaticModel(c, cum, total)
    nz = np.nonzero(c)[0]
    p = c[nz] / c[nz].sum()
    lens = list(rng.choice([0, 1, 2, 7, 15, 16, 17, 31, 33, 100, 257, 1000, 4099], 70))
    chunks = [rng.choice(nz, L, p=p).astype(np.uint8) for L in lens]
    bits = m.max_bits_per_symbol()
    caps = [rc.slot_capacity(L, bits + 1) for L in lens]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=(seed % 2 == 1), seed=seed)
    codes = []
    for k, ch in enumerate(chunks):
        f, b, L = cpu.encode(c, cum, total, ch)
        assert (fl[k], ol[k]) == (f, L), (k, fl[k], f, ol[k], L)
        got = bytes(out[out_off[k]: out_off[k] + ol[k]])
        assert got == b, k
        codes.append(b)
    dec, fd = run_decode(m, codes, lens, misalign=(seed % 2 == 0), seed=seed + 1)
    for k, ch in enumerate(chunks):
        assert fd[k] == 0
        assert (dec[k] == ch).all(), k


@pytest.mark.parametrize("total", [256, 300, 384, 511, 512])
def test_wide_direct_lut_models(ctx, total):
    """256 <= total <= 512 decodes through 16-B direct LUT entries {cum, c, s} (direct == 2):
    pow2 and magic-division totals, zero frequencies, short alphabets; encode bytes, lengths
    and decoded symbols against the oracle, and garbage streams decode like find_index."""
    rng = np.random.default_rng(total)
    n = int(rng.choice([3, 17, 200, 256]))
    c = np.zeros(n, np.int64)
    c[rng.choice(n, max(2, n - n // 6), replace=False)] = 1
    while c.sum() < total:
        c[int(rng.choice(np.nonzero(c)[0]))] += 1
    c = c.astype(np.uint32)
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, total)
    nz = np.nonzero(c)[0]
    p = c[nz] / c[nz].sum()
    lens = list(rng.choice([0, 1, 15, 16, 63, 64, 65, 127, 128, 129, 1000, 4099], 64))
    chunks = [rng.choice(nz, L, p=p).astype(np.uint8) for L in lens]
    caps = [rc.slot_capacity(L, m.max_bits_per_symbol() + 1) for L in lens]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=total)
    codes = []
    for k, ch in enumerate(chunks):
        f, b, L = cpu.encode(c, cum, total, ch)
        assert (fl[k], ol[k]) == (f, L), k
        assert bytes(out[out_off[k]: out_off[k] + ol[k]]) == b, k
        codes.append(b)
    dec, fd = run_decode(m, codes, lens, misalign=True, seed=total + 1)
    for k, ch in enumerate(chunks):
        assert fd[k] == 0 and (dec[k] == ch).all(), k
    garbage = [rng.integers(0, 256, int(rng.integers(8, 400))).astype(np.uint8).tobytes()
               for _ in range(64)]
    counts = [int(rng.integers(0, 300)) for _ in garbage]
    dec, fd = run_decode(m, garbage, counts, misalign=False, seed=total + 2)
    for k in range(len(garbage)):
        f, d = cpu.decode(c, cum, total, garbage[k], counts[k])
        assert fd[k] == f, k
        if f == 0:
            assert (dec[k] == d).all(), k


@pytest.mark.parametrize("total", [2049, 4096, 10000, 16384, 16385, 32769, 65535, 65536])
@pytest.mark.parametrize("shape", ["zipf", "runs"])
def test_small_bucket_models(ctx, total, shape):
    """2048 < total <= 2^16 decodes through the small bucket-model decoder (LUT 4): up to 2^11
    buckets in 256-lane workgroups for total <= 2^14, 2^12 buckets in 512-lane ones above
    (rc_static.h SMB_WG), across the boundary and with pow2 and magic-division totals.  "zipf":
    a Zipf(1.2) table; "runs": runs of c = 1 and c = 2 symbols between large ones, so buckets
    hold three or more symbol starts and the candidate pair misses (the exact fix-up).  Encode
    bytes and decoded symbols against the oracle; garbage streams decode like find_index."""
    rng = np.random.default_rng(total * 7 + (shape == "runs"))
    n = 256
    if shape == "zipf":
        w = 1.0 / np.arange(1, n + 1) ** 1.2
        c = np.maximum(1, np.floor(w / w.sum() * total)).astype(np.int64)
    else:
        c = rng.choice([1, 1, 2, 3], n).astype(np.int64)
        c[::37] = total // 16
    c[int(np.argmax(c))] += total - c.sum()
    assert c.min() >= 1 and c.sum() == total
    c = c.astype(np.uint32)
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, total)
    p = c / c.sum()
    lens = list(rng.choice([0, 1, 15, 16, 63, 64, 65, 1000, 4099], 48))
    chunks = [rng.choice(n, L, p=p).astype(np.uint8) for L in lens]
    # runs: also sequences of the rarest symbols, which keep range small and the fix-ups busy
    if shape == "runs":
        rare = np.nonzero(c <= 2)[0]
        chunks += [rng.choice(rare, 2000).astype(np.uint8) for _ in range(8)]
        lens += [2000] * 8
    caps = [rc.slot_capacity(L, m.max_bits_per_symbol() + 1) for L in lens]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=total)
    codes = []
    for k, ch in enumerate(chunks):
        f, b, L = cpu.encode(c, cum, total, ch)
        assert (fl[k], ol[k]) == (f, L), k
        assert bytes(out[out_off[k]: out_off[k] + ol[k]]) == b, k
        codes.append(b)
    dec, fd = run_decode(m, codes, lens, misalign=True, seed=total + 1)
    for k, ch in enumerate(chunks):
        assert fd[k] == 0 and (dec[k] == ch).all(), k
    garbage = [rng.integers(0, 256, int(rng.integers(8, 400))).astype(np.uint8).tobytes()
               for _ in range(64)]
    counts = [int(rng.integers(0, 300)) for _ in garbage]
    dec, fd = run_decode(m, garbage, counts, misalign=False, seed=total + 2)
    for k in range(len(garbage)):
        f, d = cpu.decode(c, cum, total, garbage[k], counts[k])
        assert fd[k] == f, k
        if f == 0:
            assert (dec[k] == d).all(), k


@pytest.mark.parametrize("total,c_big", [(65536, 65536 - 255), (32768, 32768 - 255),
                                         (4096, 4096 - 255), (65536, 1 << 15)])
@pytest.mark.parametrize("misalign", [False, True])
def test_rare_heavy_models(ctx, total, c_big, misalign):
    """Small models whose coded symbols are nearly all c = 1 of a large total: every symbol
    narrows range by up to 2^16, so 2-3 bytes settle per symbol and range_reduction_expansion
    runs often, back to back (the encoder's ring margin between flush checks, the decoders' rare
    paths and ring checks).  Whole 64-symbol tiles and ragged tails, against the oracle."""
    rng = np.random.default_rng(total + c_big + misalign)
    c = np.ones(256, np.int64)
    c[0] = c_big
    c[1] = total - c_big - 254
    c = c.astype(np.uint32)
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, total)
    lens = [64, 640, 4096, 4099, 65536, 1000, 127, 0] * 4
    # symbols 2..255 only (c = 1), with a few runs of the big symbol between them
    chunks = []
    for L in lens:
        ch = rng.integers(2, 256, L)
        ch[rng.random(L) < 0.05] = 0
        chunks.append(ch.astype(np.uint8))
    caps = [rc.slot_capacity(L, m.max_bits_per_symbol() + 1) for L in lens]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=misalign, seed=total)
    codes = []
    for k, ch in enumerate(chunks):
        f, b, L = cpu.encode(c, cum, total, ch)
        assert (fl[k], ol[k]) == (f, L), k
        assert bytes(out[out_off[k]: out_off[k] + ol[k]]) == b, k
        codes.append(b)
    dec, fd = run_decode(m, codes, lens, misalign=misalign, seed=total + 1)
    for k, ch in enumerate(chunks):
        assert fd[k] == 0 and (dec[k] == ch).all(), k


@pytest.mark.parametrize("seed", range(4))
def test_garbage_streams_decode_like_oracle(ctx, seed):
    """find_index on arbitrary bytes (data < lower_bound wraps, rfreq >= total) must pick the
    same index as the reference's binary search, and flag where the reference would hang."""
    rng = np.random.default_rng(seed)
    for kind in ["pow2", "small", "big"]:
        c = _random_model(rng, kind)
        cum = cum_of(c)
        total = int(c.astype(np.uint64).sum())
        m = rc.StaticModel(c, cum, total)
        codes = [rng.integers(0, 256, int(rng.integers(8, 400))).astype(np.uint8).tobytes()
                 for _ in range(64)]
        counts = [int(rng.integers(0, 300)) for _ in codes]
        dec, fd = run_decode(m, codes, counts, misalign=True, seed=seed)
        for k in range(len(codes)):
            f, d = cpu.decode(c, cum, total, codes[k], counts[k])
            assert fd[k] == f, (kind, k, fd[k], f)
            if f == 0:
                assert (dec[k] == d).all(), (kind, k)


def test_error_flags_gpu(ctx):
    c = np.array([1, 5, 2, 0, 2, 2, 1, 1, 1, 1], np.uint32)
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, 16)
    chunks = [np.array([1, 3, 2], np.uint8), np.array([1, 10], np.uint8),
              np.array([], np.uint8), np.array([3, 10], np.uint8),
              np.array([1, 2, 4, 5] * 10, np.uint8)]
    caps = [64, 64, 64, 64, 5]  # the last slot overflows; run_encode checks the sentinel after it
    for mis in (False, True):
        out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=mis)
        assert list(fl) == [rc.api.N.F_ZERO_FREQ, rc.api.N.F_BAD_SYMBOL, 0,
                            rc.api.N.F_ZERO_FREQ, rc.api.N.F_CAPACITY]
        f, full, L = cpu.encode(c, cum, 16, chunks[4])
        assert ol[4] == L and bytes(out[out_off[4]:out_off[4] + 5]) == full[:5]
        assert bytes(out[out_off[2]:out_off[2] + 8]) == bytes(8) and ol[2] == 8
    # decoder: truncated streams and short codes
    codes = [full[:7], full[:-1], full, full[:8]]
    counts = [1, 40, 40, 40]
    dec, fd = run_decode(m, codes, counts)
    for k in range(len(codes)):
        assert fd[k] == cpu.decode(c, cum, 16, codes[k], counts[k])[0]
    assert fd[0] == rc.api.N.F_TRUNCATED and fd[1] == rc.api.N.F_TRUNCATED and fd[2] == 0
    with pytest.raises(rc.ZeroFrequencyError):
        rc.encode_chunks(m, [bytes([1, 3])])
    with pytest.raises(rc.TruncatedStreamError):
        rc.decode_chunks(m, [full[:-1]], [40])
    with pytest.raises(ValueError):
        rc.StaticModel([1, 2], [0, 2], 3)  # cum[1] != cum[0] + c[0]


def test_error_flags_sm_gpu(ctx):
    """256 <= total <= 2^16 (the SM kernels): zero-frequency and out-of-alphabet symbols, both
    orders in one chunk (the first error wins), flagged chunks among clean ones."""
    rng = np.random.default_rng(11)
    c = rng.integers(1, 400, 200).astype(np.uint32)
    c[[5, 77, 150]] = 0
    total = int(c.sum())
    assert 256 <= total <= 65536
    m = rc.StaticModel(c, cum_of(c), total)
    good = [i for i in range(200) if c[i]]
    chunks = []
    for k in range(64):
        ch = rng.choice(good, size=int(rng.integers(50, 3000))).astype(np.uint8)
        kind = k % 8
        if kind == 1:
            ch[len(ch) // 2] = 77            # zero frequency
        elif kind == 2:
            ch[len(ch) // 3] = 230           # outside the alphabet
        elif kind == 3:
            ch[10], ch[20] = 5, 201          # zero frequency first
        elif kind == 4:
            ch[10], ch[20] = 255, 150        # outside the alphabet first
        chunks.append(ch)
    caps = [rc.slot_capacity(len(ch), 16) for ch in chunks]
    for mis in (False, True):
        out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=mis, seed=3)
        for k, ch in enumerate(chunks):
            f, want, L = cpu.encode(c, cum_of(c), total, ch)
            assert fl[k] == f, (k, fl[k], f)
            if f == 0:
                assert ol[k] == L and bytes(out[out_off[k]:out_off[k] + L]) == want


def test_bad_models_rejected_by_abi(ctx):
    """rc_model_create_static validates the PModel snapshot itself (not only the Python layer)."""
    import ctypes
    N = rc.api.N
    lib = N.load()

    def create(c, cum, total, n=None):
        c = np.ascontiguousarray(c, np.uint32)
        cum = np.ascontiguousarray(cum, np.uint32)
        h = ctypes.c_void_p()
        st = lib.rc_model_create_static(ctx.handle, len(c) if n is None else n,
                                        c.ctypes.data_as(ctypes.c_void_p),
                                        cum.ctypes.data_as(ctypes.c_void_p), total,
                                        ctypes.byref(h))
        if st == N.RC_OK:
            assert lib.rc_model_destroy(h) == N.RC_OK
        else:
            assert h.value is None
        return st

    assert create([1, 5, 2], [0, 1, 6], 8) == N.RC_OK
    assert create([0, 3], [0, 0], 3) == N.RC_OK  # zero-frequency symbols are allowed
    assert create([1, 5, 2], [1, 2, 7], 8) == N.RC_E_BAD_MODEL  # cum[0] != 0
    assert create([1, 5, 2], [0, 1, 7], 8) == N.RC_E_BAD_MODEL  # cum not the prefix sum
    assert create([1, 5, 2], [0, 1, 6], 9) == N.RC_E_BAD_MODEL  # total != sum(c)
    assert create([0, 0], [0, 0], 0) == N.RC_E_BAD_MODEL  # total 0
    assert create([1] * 257, np.arange(257), 257) == N.RC_E_BAD_MODEL  # alphabet > 256
    assert create([1], [0], 1, n=0) == N.RC_E_BAD_MODEL
    big = [0xFFFFFFFF, 1]  # sum overflows u32: rejected, not wrapped
    assert create(big, [0, 0xFFFFFFFF], 0) == N.RC_E_BAD_MODEL


def test_synth_matches_host(ctx):
    for (c, _, _), L in ((synth.uniform_table(), 4096), (synth.zipf_table(), 1000)):
        inv = synth.inverse_cdf(c)
        n = 37
        t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        synth.fill(ctx, 0x5EED0001, inv, t, L, n)
        h = t.cpu().numpy()
        for k in (0, 1, 17, 36):
            assert (h[k * L:(k + 1) * L] == synth.host_chunk(0x5EED0001, inv, k, L)).all()


@pytest.mark.parametrize("cfg", ["uniform", "zipf"])
def test_full_size_round_trip(ctx, cfg):
    """64 KiB chunks (BASELINE configs[1]/[2]) at 8192 chunks: GPU round trip over all chunks,
    plus 24 seeded chunks bit-checked against the oracle."""
    c, cum, total = synth.uniform_table() if cfg == "uniform" else synth.zipf_table()
    m = rc.StaticModel(c, cum, total)
    inv = synth.inverse_cdf(c)
    n, L = 8192, 65536
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0001, inv, syms, L, n)
    sym_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    cap = rc.slot_capacity(L, 8.0 if cfg == "uniform" else 6.0, slack=1.05)
    out_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    out_len, flags = rc.encode_batch(m, syms, sym_off, out, out_off)
    dec = torch.empty_like(syms)
    fd = rc.decode_batch(m, out, out_off[:-1].contiguous(), out_len, dec, sym_off)
    torch.cuda.synchronize()
    assert int(flags.abs().sum()) == 0 and int(fd.abs().sum()) == 0
    assert torch.equal(dec, syms)
    ol = out_len.cpu().numpy()
    rng = random.Random(5)
    for k in sorted(rng.sample(range(n), 24)):
        ch = synth.host_chunk(0x5EED0001, inv, k, L)
        f, b, Lb = cpu.encode(c, cum, total, ch)
        assert f == 0 and Lb == ol[k]
        assert bytes(out[k * cap: k * cap + Lb].cpu().numpy()) == b


@pytest.mark.parametrize("cfg", ["uniform", "zipf"])
def test_coresident_workgroups(ctx, cfg):
    """2^17 chunks = 512 workgroups of 256 lanes: at least two workgroups per CU run together
    (the case that exposed the 88-VGPR corruption).  Samples from every part of
    the grid are bit-checked against the oracle; every chunk round-trips."""
    c, cum, total = synth.uniform_table() if cfg == "uniform" else synth.zipf_table()
    m = rc.StaticModel(c, cum, total)
    inv = synth.inverse_cdf(c)
    n, L = 1 << 17, 1024
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0002, inv, syms, L, n)
    sym_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    cap = rc.slot_capacity(L, 8.0, slack=1.05)
    out_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    out_len, flags = rc.encode_batch(m, syms, sym_off, out, out_off)
    dec = torch.empty_like(syms)
    fd = rc.decode_batch(m, out, out_off[:-1].contiguous(), out_len, dec, sym_off)
    torch.cuda.synchronize()
    assert int(flags.abs().sum()) == 0 and int(fd.abs().sum()) == 0
    assert torch.equal(dec, syms)
    ol = out_len.cpu().numpy()
    h = out.cpu().numpy()
    for k in range(0, n, 997):
        ch = synth.host_chunk(0x5EED0002, inv, k, L)
        f, b, lb = cpu.encode(c, cum, total, ch)
        assert f == 0 and lb == ol[k] and bytes(h[k * cap:k * cap + lb]) == b, k


@pytest.mark.parametrize("rank", [3])
def test_n8_rank_shard(ctx, rank):
    """configs[4] at N = 8: one rank's shard of the 2^20 x 64 KiB Zipf(1.2) stream, i.e. 2^17
    chunks of 65536 symbols generated as global chunks [rank * 2^17, (rank + 1) * 2^17) of the
    bench's seed (shard.synth_seed).  512 workgroups: two per CU, the co-residency shape of the
    8-GPU line.  Every chunk round-trips; 16 chunks, one from each 1/16 of the
    grid (both workgroups of a CU included), are bit-checked against the oracle."""
    from range_coder_rust_amd import shard
    c, cum, total = synth.zipf_table()
    m = rc.StaticModel(c, cum, total)
    inv = synth.inverse_cdf(c)
    n, L = 1 << 17, 1 << 16
    lo, hi = shard.shard_range(1 << 20, 8, rank)
    assert hi - lo == n
    seed = shard.synth_seed(0x5EED0001, lo)
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, seed, inv, syms, L, n)
    sym_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    cap = rc.slot_capacity(L, 6.0, slack=1.02)  # Zipf(1.2) codes at ~5.3 bits/symbol
    out_off = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    out_len, flags = rc.encode_batch(m, syms, sym_off, out, out_off)
    dec = torch.empty_like(syms)
    fd = rc.decode_batch(m, out, out_off[:-1].contiguous(), out_len, dec, sym_off)
    torch.cuda.synchronize()
    assert int(flags.abs().sum()) == 0 and int(fd.abs().sum()) == 0
    step = 1 << 30
    for i in range(0, n * L, step):
        assert torch.equal(dec[i:i + step], syms[i:i + step]), i
    ol = out_len.cpu().numpy()
    for j in range(16):
        k = j * (n // 16) + (j * 4099) % (n // 16)
        ch = synth.host_chunk(seed, inv, k, L)
        assert np.array_equal(ch, syms[k * L:(k + 1) * L].cpu().numpy()), k
        f, b, lb = cpu.encode(c, cum, total, ch)
        got = bytes(out[k * cap:k * cap + lb].cpu().numpy())
        assert f == 0 and lb == ol[k] and got == b, k
    del syms, out, dec
    torch.cuda.empty_cache()


def test_cpp_sample_impl(ctx):
    """The reference example (examples/sample_impl.rs) via the C++ host API (include/*.hpp)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                       "sample_impl")
    if not os.path.exists(exe):
        pytest.skip("examples/sample_impl not built")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "output : 0x64475f8970365a2f83b20246c0" in r.stdout
    assert "test passed" in r.stdout


def _pair_models(rng):
    """Models of the pair-bucket decoder (2^15 < total <= 2^16): Zipf, skewed with zero
    frequencies and c = 1 runs (buckets with several symbol starts: the exact fix-up), and the
    extreme totals."""
    zc, _, zt = synth.zipf_table()
    out = [(zc.astype(np.uint32), zt)]
    for total in (32769, 40000, 65535, 65536):
        n = int(rng.choice([2, 3, 50, 200, 256]))
        w = rng.pareto(1.0, n) + 0.01
        c = np.floor(w / w.sum() * total).astype(np.int64)
        if n > 3:
            c[rng.random(n) < 0.2] = 0
            c[rng.choice(n, min(10, n), replace=False)] = 1
        c[int(np.argmax(c))] += total - int(c.sum())
        if c.max() >= 65536:  # one symbol holding everything: no pair table (16-bit fields)
            c[0] -= 1
            c[1] += 1
        out.append((c.astype(np.uint32), total))
    return out


def _pair_decoder_cases(kc):
    rng = np.random.default_rng(77)
    for mi, (c, total) in enumerate(_pair_models(rng)):
        cum = cum_of(c)
        m = rc.StaticModel(c, cum, total, ctx=kc)
        nz = np.nonzero(c)[0]
        p = c[nz] / c[nz].sum()
        lens = list(rng.choice([0, 1, 15, 16, 17, 64, 65, 257, 1000, 4099], 96))
        chunks = [rng.choice(nz, L, p=p).astype(np.uint8) for L in lens]
        codes = [cpu.encode(c, cum, total, ch)[1] for ch in chunks]
        dec, fd = run_decode(m, codes, lens, misalign=(mi % 2 == 0), seed=mi)
        for k, ch in enumerate(chunks):
            assert fd[k] == 0 and (dec[k] == ch).all(), (mi, k)
        garbage = [rng.integers(0, 256, int(rng.integers(8, 400))).astype(np.uint8).tobytes()
                   for _ in range(64)]
        counts = [int(rng.integers(0, 300)) for _ in garbage]
        dec, fd = run_decode(m, garbage, counts, misalign=True, seed=mi + 100)
        for k in range(len(garbage)):
            f, d = cpu.decode(c, cum, total, garbage[k], counts[k])
            assert fd[k] == f, (mi, k, fd[k], f)
            if f == 0:
                assert (dec[k] == d).all(), (mi, k)


@pytest.mark.parametrize("pair", ["512", "1024", "0"])
def test_pair_bucket_decoder_vs_oracle(ctx, knob_ctx, pair):
    """k_decode_static LUT 3 (both candidates of a bucket in one 16-B LDS entry) at both
    workgroup sizes, and the bucket decoder it replaces at low occupancy (RC_DEC_PAIR=0), on the
    same streams: decoded symbols against the oracle's, ragged and misaligned chunks; garbage
    streams decode like the reference's find_index, flags included."""
    _pair_decoder_cases(knob_ctx(RC_DEC_PAIR=pair))

def test_flat_model_garbage_and_truncated_streams(ctx):
    """The flat model (256 symbols, every c = 1: k_decode_static LUT 5, k_encode_static SM 3,
    no table reads) on arbitrary bytes and truncated streams: flags as the oracle's, and the
    decoded symbols where the oracle decodes (find_index is rfreq itself, sample_impl.rs:27-45)."""
    rng = np.random.default_rng(41)
    c = np.ones(256, np.uint32)
    cum = cum_of(c)
    m = rc.StaticModel(c, cum, 256)
    codes = [rng.integers(0, 256, int(rng.integers(8, 600))).astype(np.uint8).tobytes()
             for _ in range(96)]
    counts = [int(rng.integers(0, 700)) for _ in codes]
    dec, fd = run_decode(m, codes, counts, misalign=True, seed=41)
    for k in range(len(codes)):
        f, d = cpu.decode(c, cum, 256, codes[k], counts[k])
        assert fd[k] == f, (k, fd[k], f)
        if f == 0:
            assert (dec[k] == d).all(), k
    # valid streams cut short, and their encoder bytes against the oracle
    chunks = [rng.integers(0, 256, int(rng.integers(1, 3000))).astype(np.uint8) for _ in range(64)]
    caps = [rc.slot_capacity(len(ch), 9) for ch in chunks]
    out, out_off, ol, fl = run_encode(m, chunks, caps, misalign=True, seed=43)
    cut = []
    for k, ch in enumerate(chunks):
        f, b, L = cpu.encode(c, cum, 256, ch)
        assert fl[k] == f == 0 and ol[k] == L and bytes(out[out_off[k]:out_off[k] + L]) == b, k
        cut.append(b[:max(8, L - int(rng.integers(0, 6)))])
    dec, fd = run_decode(m, cut, [len(ch) for ch in chunks], misalign=True, seed=47)
    for k, ch in enumerate(chunks):
        f, d = cpu.decode(c, cum, 256, cut[k], len(ch))
        assert fd[k] == f, (k, fd[k], f)
        if f == 0:
            assert (dec[k] == ch).all(), k
