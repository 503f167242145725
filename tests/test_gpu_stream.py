"""The reference's per-call surface on the GPU (rc_stream_* kernels, rc_resume.hip) against the
oracles: Encoder / Decoder with a PModel the caller changes between calls, encode()'s byte
counts, peek_code, range_coder / data, Decoder without a symbol count, errors at the exact
call; and the batch device entry points against orc_stream_* with random (even inconsistent)
tables, garbage streams, split calls and 64-bit stream positions."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402
from oracle import cpu, ref_literal as R  # noqa: E402
from gpu_helpers import dev  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rc.default_context(0)


SAMPLE = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]


def _sample_table():
    sd = rc.FreqTable(10)
    for i in SAMPLE:
        sd.add_alphabet_freq(i)
    sd.calc_cum()
    return sd


def test_sample_impl_reference_surface(ctx):
    """examples/sample_impl.rs:72-128 verbatim: Decoder::new(code) takes no count."""
    sd = _sample_table()
    encoder = rc.Encoder.new()
    rets = [encoder.encode(sd, i) for i in SAMPLE]
    code = encoder.finish()
    assert code.hex() == "64475f8970365a2f83b20246c0"
    ref = R.Encoder()
    rt = R.FreqTable.from_counts(sd.c)
    assert [int(r) for r in rets] == [ref.encode(rt, i) for i in SAMPLE]
    decoder = rc.Decoder.new(code)
    assert [decoder.decode(sd) for _ in SAMPLE] == SAMPLE


class AdaptiveFreqTable(rc.FreqTable):
    """A caller-side adaptive model: the mirror FreqTable, updated after every symbol with the
    rule of oracle/ref_literal.py AdaptiveModel (what a reference user would write on top of
    the PModel trait)."""

    def __init__(self, n, inc, limit, period):
        super().__init__(n)
        self.c = [1] * n
        self.calc_cum()
        self.inc, self.limit, self.period = inc, limit, period

    def update(self, s, i):
        self.c[s] += self.inc
        if (i + 1) % self.period == 0 and sum(self.c) > self.limit:
            self.c = [(x + 1) >> 1 for x in self.c]
        self.calc_cum()


def _zipfish(n, seed, alpha=256):
    rng = random.Random(seed)
    return [min(alpha - 1, int(rng.paretovariate(1.15))) for _ in range(n)]


def test_model_mutated_between_encode_calls(ctx):
    syms = _zipfish(5000, 1)
    want = R.encode_adaptive_stream(256, 32, 4000, 64, syms)
    m = AdaptiveFreqTable(256, 32, 4000, 64)
    ref_m = R.AdaptiveModel(256, 32, 4000, 64)
    ref = R.Encoder()
    enc = rc.Encoder()
    rets, ref_rets = [], []
    for i, s in enumerate(syms):
        rets.append(enc.encode(m, s))
        ref_rets.append(ref.encode(ref_m, s))
        m.update(s, i)
        ref_m.update(s, i)
        if i in (0, 7, 100, 2047, 4000):  # peek_code / range_coder mid-stream
            assert enc.peek_code() == bytes(ref.code)
            assert enc.range_coder == rc.RangeCoder(ref.range_coder.lower_bound,
                                                    ref.range_coder.range)
    code = enc.finish()
    assert code == want
    assert [int(r) for r in rets] == ref_rets
    with pytest.raises(rc.FinishedError):
        enc.encode(m, 0)


def test_model_mutated_between_decode_calls(ctx):
    syms = _zipfish(4000, 2)
    code = R.encode_adaptive_stream(256, 32, 4000, 64, syms)
    m = AdaptiveFreqTable(256, 32, 4000, 64)
    ref = R.Decoder(code)
    ref_m = R.AdaptiveModel(256, 32, 4000, 64)
    dec = rc.Decoder(code)
    out = []
    for i in range(len(syms)):
        s = dec.decode(m)
        assert s == ref.decode(ref_m)
        out.append(s)
        m.update(s, i)
        ref_m.update(s, i)
        if i in (0, 9, 1000, 3999):
            assert dec.data() == ref.data
            assert dec.range_coder() == rc.RangeCoder(ref.range_coder.lower_bound,
                                                      ref.range_coder.range)
    assert out == syms


def test_static_then_switch_models_mid_stream(ctx):
    """Decode-ahead blocks under one table, then a different table from symbol 3000 on."""
    a = rc.FreqTable.from_counts([1 + (i * 7) % 13 for i in range(256)])
    b = rc.FreqTable.from_counts([1 + (i * 3) % 29 for i in range(256)])
    rng = random.Random(3)
    syms = [rng.randrange(256) for _ in range(6000)]
    enc = rc.Encoder()
    for i, s in enumerate(syms):
        enc.encode(a if i < 3000 else b, s)
    code = enc.finish()
    ref = R.Encoder()
    ra, rb = R.FreqTable.from_counts(a.c), R.FreqTable.from_counts(b.c)
    for i, s in enumerate(syms):
        ref.encode(ra if i < 3000 else rb, s)
    assert code == bytes(ref.finish())
    dec = rc.Decoder(code)
    got = [dec.decode(a) for _ in range(2500)]
    st = dec.range_coder()  # re-derived inside a decode-ahead block
    got += [dec.decode(a) for _ in range(500)]
    got += [dec.decode(b) for _ in range(3000)]
    assert got == syms
    rdec = R.Decoder(code)
    for _ in range(2500):
        rdec.decode(ra)
    assert st == rc.RangeCoder(rdec.range_coder.lower_bound, rdec.range_coder.range)


def test_errors_at_the_reference_call(ctx):
    sd = _sample_table()
    enc = rc.Encoder()
    with pytest.raises(rc.ZeroFrequencyError):
        enc.encode(sd, 3)  # c_freq(3) == 0: the reference never terminates
    with pytest.raises(rc.BadSymbolError):
        enc.encode(sd, 10)  # sample_impl.rs:19 unwrap
    code = rc.Encoder()
    for i in SAMPLE:
        code.encode(sd, i)
    code = code.finish()
    # decoding past the end: the reference panics in shift_left_buffer at some call k
    ref = R.Decoder(code)
    rt = R.FreqTable.from_counts(sd.c)
    k = 0
    while True:
        try:
            ref.decode(rt)
        except R.ReferencePanic:
            break
        k += 1
    dec = rc.Decoder(code)
    for _ in range(k):
        dec.decode(sd)
    with pytest.raises(rc.TruncatedStreamError):
        dec.decode(sd)
    with pytest.raises(rc.TruncatedStreamError):
        rc.Decoder(code[:7])


def _random_triples(rng, n):
    t = []
    for _ in range(n):
        total = rng.choice([256, 65536, rng.randint(1, 2 ** 32 - 1)])
        c = rng.randint(1, total) if rng.random() < 0.97 else rng.randint(0, 2 ** 32 - 1)
        cum = rng.randint(0, total - min(c, total)) if rng.random() < 0.97 else \
            rng.randint(0, 2 ** 32 - 1)
        t.append((c, cum, total if rng.random() < 0.995 else 0))
    return t


def test_batch_stream_encode_split_calls_vs_oracle(ctx):
    rng = random.Random(5)
    ns = 150
    streams = [_random_triples(rng, rng.randint(0, 300)) for _ in range(ns)]
    # oracle: one call each
    want = []
    for t in streams:
        st = cpu.Stream.fresh()
        f, b, nb = cpu.stream_encode(st, t, finish=True)
        want.append((f, b, nb.tolist(), st.tuple()))
    states = rc.stream_states(ns)
    got = [b""] * ns
    counts = [[] for _ in range(ns)]
    cut = [sorted(rng.randint(0, len(t)) for _ in range(2)) for t in streams]
    for part in range(3):
        pieces = []
        for k, t in enumerate(streams):
            lo = 0 if part == 0 else cut[k][part - 1]
            hi = cut[k][part] if part < 2 else len(t)
            pieces.append(t[lo:hi])
        lens = np.array([len(p) for p in pieces], np.int64)
        sym_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        trip = np.array([x for p in pieces for x in p] or [(0, 0, 0)], np.uint32).reshape(-1)
        fin = part == 2
        caps = 12 * lens + (8 if fin else 0) + 3
        out_off = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
        out = torch.full((int(out_off[-1]) + 16,), 0xEE, dtype=torch.uint8, device="cuda")
        nb = torch.zeros(max(int(sym_off[-1]), 1), dtype=torch.uint8, device="cuda")
        ol, fl = rc.stream_encode_batch(ctx, states, dev(trip.view(np.int32)), dev(sym_off), out,
                                        dev(out_off), nbytes=nb, finish=fin)
        torch.cuda.synchronize()
        h, ol, nbh = out.cpu().numpy(), ol.cpu().numpy(), nb.cpu().numpy()
        stt = states.cpu().numpy().view(np.uint64)
        for k in range(ns):
            got[k] += h[out_off[k]: out_off[k] + ol[k]].tobytes()
            nk = int(stt[k, 4]) - len(counts[k])
            counts[k] += nbh[sym_off[k]: sym_off[k] + nk].tolist()
            assert (h[out_off[k] + ol[k]: out_off[k + 1]] == 0xEE).all()
    stt = states.cpu().numpy().view(np.uint64)
    for k in range(ns):
        f, b, nb, tup = want[k]
        assert got[k] == b, k
        assert counts[k] == nb, k
        lo, r, d, pos, n, fs = (int(x) for x in stt[k])
        assert (lo, r, pos, n, fs & 0xFFFFFFFF, fs >> 32) == \
            (tup[0], tup[1], tup[3], tup[4], tup[5], tup[6]), k


def test_batch_stream_decode_split_calls_vs_oracle(ctx):
    rng = random.Random(6)
    ns = 120
    na = 40
    c = np.array([rng.choice([0, 1, rng.randint(1, 900)]) for _ in range(na)], np.uint32)
    cum = np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32)
    total = int(c.sum())
    codes = []
    for k in range(ns):
        if k % 3 == 0:  # valid streams
            syms = [s for s in (rng.randrange(na) for _ in range(400)) if c[s]][:300]
            codes.append(cpu.encode(c, cum, total, np.array(syms, np.uint8))[1])
        else:  # garbage
            codes.append(bytes(rng.randrange(256) for _ in range(rng.randint(0, 90))))
    want = []
    for code in codes:
        st = cpu.Stream.fresh()
        f, s = cpu.stream_decode(st, c, cum, total, code, 320)
        want.append((f, s.tolist(), st.tuple()))
    clen = np.array([len(x) for x in codes], np.int64)
    coff = np.concatenate([[0], np.cumsum(clen)[:-1]]).astype(np.int64)
    blob = np.frombuffer(b"".join(codes) + b"\0" * 16, np.uint8)
    states = rc.stream_states(ns)
    got = [[] for _ in range(ns)]
    for part, m in enumerate((100, 0, 220)):
        sym_off = (np.arange(ns + 1) * m).astype(np.int64)
        syms = torch.full((ns * m + 16,), 0xEE, dtype=torch.uint8, device="cuda")
        before = states.cpu().numpy().view(np.uint64)[:, 4].copy()
        rc.stream_decode_batch(ctx, dev(c.view(np.int32)), dev(cum.view(np.int32)), total,
                               states, dev(blob), dev(coff), dev(clen), syms, dev(sym_off))
        torch.cuda.synchronize()
        after = states.cpu().numpy().view(np.uint64)[:, 4]
        h = syms.cpu().numpy()
        for k in range(ns):
            got[k] += h[k * m: k * m + int(after[k] - before[k])].tolist()
    stt = states.cpu().numpy().view(np.uint64)
    for k in range(ns):
        f, s, tup = want[k]
        assert got[k] == s, k
        lo, r, d, pos, n, fs = (int(x) for x in stt[k])
        assert (lo, r, d, pos, n, fs & 0xFFFFFFFF) == tup[:6], k


def test_stream_positions_are_64_bit(ctx):
    """A decoder whose state sits 2^33 bytes into its stream: code_off points 2^33 before the
    window (u64 wrap-around), so only 64-bit positions address the right bytes."""
    c = np.ones(256, np.uint32)
    cum = np.arange(256, dtype=np.uint32)
    rng = np.random.default_rng(9)
    syms = rng.integers(0, 256, 500).astype(np.uint8)
    code = cpu.encode(c, cum, 256, syms)[1]
    # the oracle's state after Decoder::new + 100 symbols
    st = cpu.Stream.fresh()
    f, _ = cpu.stream_decode(st, c, cum, 256, code, 100)
    assert f == 0
    big = 1 << 33
    states = rc.stream_states(1)
    row = np.array([st.lower_bound, st.range, st.data, st.pos + big, st.n, 1 << 32], np.uint64)
    states[0] = torch.from_numpy(row.view(np.int64)).to("cuda")
    blob = dev(np.frombuffer(code + b"\0" * 16, np.uint8))
    coff = np.array([(-big) & ((1 << 64) - 1)], np.uint64)
    out = torch.zeros(400, dtype=torch.uint8, device="cuda")
    fl = rc.stream_decode_batch(ctx, dev(c.view(np.int32)), dev(cum.view(np.int32)), 256, states,
                                blob, dev(coff.view(np.int64)),
                                dev(np.array([len(code) + big], np.int64)), out,
                                dev(np.array([0, 400], np.int64)))
    torch.cuda.synchronize()
    assert int(fl[0]) == 0
    assert np.array_equal(out.cpu().numpy(), syms[100:])
    assert int(states.cpu().numpy().view(np.uint64)[0, 3]) == big + len(code)


def _xorshift_syms(n, seed):
    """The symbol generator of examples/adaptive_impl.cpp."""
    x, out, M = seed, [], (1 << 64) - 1
    for _ in range(n):
        x ^= (x << 13) & M
        x ^= x >> 7
        x ^= (x << 17) & M
        r = x % 1000
        out.append(r % 4 if r < 500 else (r % 32 if r < 800 else r % 256))
    return out


def test_cpp_caller_adaptive_model(ctx):
    """examples/adaptive_impl.cpp: rc::Encoder / rc::Decoder with a PModel the caller updates
    between calls; its stream equals the literal restatement's."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                       "adaptive_impl")
    if not os.path.exists(exe):
        pytest.skip("examples/adaptive_impl not built")
    n, seed = 3000, 5
    r = subprocess.run([exe, str(n), str(seed)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    want = R.encode_adaptive_stream(256, 32, 4000, 64, _xorshift_syms(n, seed))
    assert r.stdout.strip() == want.hex()


def _canonical_index(c, cum, total, low, rng, data):
    """FreqTable::find_index (sample_impl.rs:27-45), for the test models below."""
    rf = ((data - low) & ((1 << 64) - 1)) // (rng // total)
    left, right = 0, len(c) - 1
    while left < right:
        mid = (left + right) // 2
        if cum[mid + 1] <= rf:
            left = mid + 1
        else:
            right = mid
    return left


class _Linear(rc.FreqTable):
    """find_index overridden by a linear scan (same inverse as the binary search)."""
    calls = 0

    def find_index(self, decoder):
        type(self).calls += 1
        r = decoder.range_coder()
        rf = ((decoder.data() - r.lower_bound()) & ((1 << 64) - 1)) // (r.range() // self.total)
        i = 0
        while i + 1 < len(self.c) and self.cum[i + 1] <= rf:
            i += 1
        return i


class _NextUp(rc.FreqTable):
    """A different inverse: the canonical symbol's successor where that has c > 0."""

    def find_index(self, decoder):
        r = decoder.range_coder()
        i = _canonical_index(self.c, self.cum, self.total, r.lower_bound(), r.range(),
                             decoder.data())
        return i + 1 if i + 1 < len(self.c) and self.c[i + 1] else i


class _RefNextUp(R.FreqTable):
    def find_index(self, decoder):
        rcd = decoder.range_coder
        i = _canonical_index(self.c, self.cum, self.total, rcd.lower_bound, rcd.range,
                             decoder.data)
        return i + 1 if i + 1 < len(self.c) and self.c[i + 1] else i


class _Opted(_Linear):
    canonical_find_index = True  # the override keeps the binary search's semantics


def test_custom_find_index_is_called(ctx):
    """pmodel.rs:12 / decoder.rs:40: a model's own find_index decides every decoded index."""
    sd = _sample_table()
    enc = rc.Encoder()
    for i in SAMPLE:
        enc.encode(sd, i)
    code = enc.finish()
    lin = _Linear(10)
    lin.c = list(sd.c)
    lin.calc_cum()
    _Linear.calls = 0
    dec = rc.Decoder(code)
    assert [dec.decode(lin) for _ in SAMPLE] == SAMPLE
    assert _Linear.calls == len(SAMPLE)
    # opted in: the decode-ahead path, find_index never called
    opt = _Opted(10)
    opt.c = list(sd.c)
    opt.calc_cum()
    _Linear.calls = 0
    dec = rc.Decoder(code)
    assert [dec.decode(opt) for _ in SAMPLE] == SAMPLE and _Linear.calls == 0


def test_custom_find_index_other_inverse_vs_reference(ctx):
    """A find_index with a different inverse decodes other symbols: exactly the reference's,
    symbol by symbol, until the reference panics (then the same error class at that call)."""
    rng = random.Random(11)
    counts = [rng.randint(1, 40) for _ in range(32)]
    syms = [rng.randrange(32) for _ in range(300)]
    m = rc.FreqTable.from_counts(counts)
    enc = rc.Encoder()
    for s in syms:
        enc.encode(m, s)
    code = enc.finish()
    ours = _NextUp(32)
    ours.c = list(counts)
    ours.calc_cum()
    ref_m = _RefNextUp.from_counts(counts)
    ref = R.Decoder(code)
    dec = rc.Decoder(code)
    got, want, ref_err = [], [], None
    for _ in range(len(syms)):
        try:
            want.append(ref.decode(ref_m))
        except (R.ReferencePanic, R.RangeCoderError) as e:
            ref_err = e
            break
        got.append(dec.decode(ours))
    assert got == want and want != syms[:len(want)]
    if ref_err is not None:
        with pytest.raises(rc.RangeCoderError):
            dec.decode(ours)


def test_lower_bound_overflow_payload(ctx):
    """error.rs:5-10: LowerBoundOverflow {lower_bound, add_val, range} at the failing encode."""
    class Bad(rc.PModel):
        def __init__(self):
            self.bad = False

        def alphabet_count(self):
            return 2

        def c_freq(self, i):
            return 1

        def cum_freq(self, i):
            return 0xFFFFFFFF if self.bad else i

        def total_freq(self):
            return 2

    m = Bad()
    enc = rc.Encoder()
    ref = R.Encoder()
    for i in (1, 1, 0, 1):  # a lower bound well above 0
        enc.encode(m, i)
        ref.encode(m, i)
    m.bad = True
    low, rng_ = ref.range_coder.lower_bound, ref.range_coder.range
    r = rng_ // 2
    add, nr = (r * 0xFFFFFFFF) & ((1 << 64) - 1), r
    assert low + add > (1 << 64) - 1  # the reference's overflowing_add fails here
    enc.encode(m, 1)
    with pytest.raises(rc.LowerBoundOverflow) as ei:
        enc.peek_code()
    e = ei.value
    assert (e.lower_bound, e.add_val, e.range) == (low, add, nr)
    with pytest.raises(rc.LowerBoundOverflow):  # the encoder stays failed, as after a panic
        enc.peek_code()


def test_cpp_find_index(ctx):
    """examples/find_index_impl.cpp: an overridden find_index is called per symbol, and
    LowerBoundOverflow carries the reference's payload, through the C++ host API."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                       "find_index_impl")
    if not os.path.exists(exe):
        pytest.skip("examples/find_index_impl not built")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "find_index called 16 times" in r.stdout and "test passed" in r.stdout


def test_threads_share_the_default_context(ctx):
    """Several Python threads code their own streams through the process-wide default context at
    the same time (ctypes releases the GIL in every native call): each stream's staging block
    use is serialised per context (rc_resume.hip), so no thread sees another's bytes.  Static
    tables decode ahead in blocks and encoders flush at every peek_code, so every thread goes
    through the staging block many times."""
    import threading

    n_threads, n_sym = 4, 6000
    tables, streams = [], []
    for k in range(n_threads):
        rng = np.random.default_rng(100 + k)
        counts = [int(x) for x in rng.integers(1, 50, 40 + 20 * k)]
        tables.append(rc.FreqTable.from_counts(counts))
        p = np.asarray(counts, float) / sum(counts)
        streams.append([int(s) for s in rng.choice(len(counts), n_sym, p=p)])
    codes, decoded, errors = [None] * n_threads, [None] * n_threads, []
    start = threading.Barrier(n_threads)

    def work(k):
        try:
            t, syms = tables[k], streams[k]
            start.wait()
            e = rc.Encoder()
            for i, s in enumerate(syms):
                e.encode(t, s)
                if i % 750 == 749:
                    e.peek_code()
            codes[k] = e.finish()
            d = rc.Decoder(codes[k])
            decoded[k] = [d.decode(t) for _ in syms]
        except Exception as exc:  # noqa: BLE001 (reported below)
            errors.append((k, repr(exc)))

    threads = [threading.Thread(target=work, args=(k,)) for k in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    for k in range(n_threads):
        c = np.asarray(tables[k].c, np.uint32)
        cum = np.asarray(tables[k].cum, np.uint32)
        f, b, _ = cpu.encode(c, cum, tables[k].total, np.asarray(streams[k], np.uint8))
        assert f == 0 and bytes(codes[k]) == bytes(b), k
        assert decoded[k] == streams[k], k


# ---- the stream service (rc_resume.hip): small host calls through a persistent wave ----------

def _adaptive_round_trip(ctx_, n=1500, seed=11):
    syms = _zipfish(n, seed)
    m = AdaptiveFreqTable(256, 32, 4000, 64)
    enc = rc.Encoder(ctx=ctx_)
    rets = []
    for i, s in enumerate(syms):
        rets.append(enc.encode(m, s))
        m.update(s, i)
        if i % 97 == 0:
            enc.peek_code()  # a flush: one small encode call
    code = enc.finish()
    m = AdaptiveFreqTable(256, 32, 4000, 64)
    dec = rc.Decoder(code, ctx=ctx_)
    out = []
    for i in range(n):
        s = dec.decode(m)  # the table changes every symbol: one decode call per symbol
        out.append(s)
        m.update(s, i)
    return syms, code, [int(r) for r in rets], out


@pytest.mark.parametrize("service", ["1", "0"])
def test_service_and_launch_paths_vs_reference(ctx, knob_ctx, service):
    """The same caller-adaptive round trip through the service (default) and through the
    launch path (a context created with RC_STREAM_SERVICE=0), against ref_literal's bytes and
    encode() counts."""
    syms, code, rets, out = _adaptive_round_trip(knob_ctx(RC_STREAM_SERVICE=service))
    assert code == R.encode_adaptive_stream(256, 32, 4000, 64, syms)
    ref = R.Encoder()
    ref_m = R.AdaptiveModel(256, 32, 4000, 64)
    want = []
    for i, s in enumerate(syms):
        want.append(ref.encode(ref_m, s))
        ref_m.update(s, i)
    assert rets == want
    assert out == syms


def test_service_restarts_after_idle_and_stops_on_destroy(ctx):
    """The wave leaves after its idle time; the next call starts a new one.  rc_ctx_destroy
    with a wave running returns promptly, and torch.cuda.synchronize() is not held up for
    longer than the idle time."""
    import time
    c2 = rc.Context(0)
    try:
        sd = _sample_table()
        for rep in range(3):
            enc = rc.Encoder(ctx=c2)
            for i in SAMPLE:
                enc.encode(sd, i)
            assert enc.finish().hex() == "64475f8970365a2f83b20246c0"
            dec = rc.Decoder(bytes.fromhex("64475f8970365a2f83b20246c0"), ctx=c2)
            assert [dec.decode(sd) for _ in SAMPLE] == SAMPLE
            time.sleep(0.02)  # > the idle time: the wave has left, the next call relaunches
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 1.0
        enc = rc.Encoder(ctx=c2)
        enc.encode(sd, 1)
        enc.peek_code()  # a wave is running now
    finally:
        t0 = time.perf_counter()
        c2.close()
        assert time.perf_counter() - t0 < 1.0


def _set_idle_ticks(ticks):
    L = rc._native.load()
    L.rc_svc_set_idle_ticks_.argtypes = [ctypes.c_uint64]
    L.rc_svc_set_idle_ticks_.restype = ctypes.c_int
    assert L.rc_svc_set_idle_ticks_(ticks) == 0


def test_service_wave_leaving_as_requests_arrive():
    """a wave that leaves between the host's publication of a request and its
    check must not read as a device fault.  With an idle time of 1 tick (10 ns) every wave
    leaves right after its request, so nearly every call races a leaving wave; all of them must
    return the reference's bytes and symbols (and no RC_E_DEVICE)."""
    c2 = rc.Context(0)
    _set_idle_ticks(1)
    try:
        syms, code, rets, out = _adaptive_round_trip(c2, n=400, seed=3)
        assert code == R.encode_adaptive_stream(256, 32, 4000, 64, syms)
        assert out == syms
    finally:
        _set_idle_ticks(0)
        c2.close()


def test_batch_launches_while_the_service_is_busy(ctx):
    """while another thread keeps the context's service wave busy, batch encode /
    decode launches on torch's default stream and on a second torch stream finish in their
    usual time: they do not queue behind the wave (which shares a hardware queue with some
    stream of the process)."""
    import threading
    import time
    c2 = rc.Context(0)
    c, cum, total = synth.zipf_table()
    n, L = 2048, 4096
    inv = synth.inverse_cdf(c)
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0001, inv, syms, L, n)
    cap = rc.slot_capacity(L, 8.0)
    so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    dec = torch.empty_like(syms)
    ref = _adaptive_round_trip(c2, n=200, seed=5)

    def batch(m):
        t0 = time.perf_counter()
        ol, fe = rc.encode_batch(m, syms, so, out, oo)
        fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert int(fe.abs().sum()) == 0 and int(fd.abs().sum()) == 0 and torch.equal(dec, syms)
        return dt

    m_default = rc.StaticModel(c, cum, total, ctx=ctx)
    m_c2 = rc.StaticModel(c, cum, total, ctx=c2)
    base = max(batch(m_default), batch(m_c2))  # unloaded (and warmed up)
    stop, errs, rounds = threading.Event(), [], [0]

    def busy():
        try:
            while not stop.is_set():
                if _adaptive_round_trip(c2, n=200, seed=5) != ref:
                    errs.append("mismatch")
                rounds[0] += 1
        except Exception as e:  # (reported below)
            errs.append(repr(e))

    th = threading.Thread(target=busy)
    th.start()
    try:
        time.sleep(0.3)
        times = []
        for m in (m_default, m_c2):
            times.append(batch(m))
            side = torch.cuda.Stream()
            with torch.cuda.stream(side):
                times.append(batch(m))
    finally:
        stop.set()
        th.join()
        c2.close()
    assert not errs, errs
    assert rounds[0] >= 1
    # the library's launches ask the wave to leave first (rc_svc_yield_all_), and a wave lives
    # 1 ms at most (SVC_LIFE_US), so a batch waits for it a millisecond at worst; before round 6
    # the same launches waited 1.7-4.0 s (profiles/r06/service_busy.json)
    assert max(times) < 5 * base + 0.005, (times, base)
