"""The Python mirror's per-call logic (api.py Encoder / Decoder) on the CPU: the two one-stream
entry points it calls (rc_stream_encode_host / rc_stream_decode_host) are stood in for by the C
oracle's resumable coder (orc_stream_encode / orc_stream_decode, oracle/rc_oracle.c) behind a
fake context, so what is tested is the mirror itself: staging and flushing (small flushes through
reused buffers, large ones through numpy arrays), the decode-ahead blocks that double while the
table holds, re-deriving the state when the caller's table changes or range_coder() / data() are
asked mid-block, the find_index override path (pmodel.rs:12), and the reference's errors at the
call that hits them.  Expected values come from oracle/ref_literal.py, the literal restatement.
The GPU suite (tests/test_gpu_stream.py) runs the same surface on the kernels.  The C++ mirror
(include/range_coder.hpp) gets the same treatment: the examples (examples/*.cpp) are built with
g++ against tests/native/oracle_backed_rc.cpp, which implements those two entry points over the
oracle, and their output is checked as the GPU suite checks it.

The fake reads the caller's buffers only inside the call, after allocating and filling scratch
arrays of the same sizes, so a buffer the mirror let go of before the call (a temporary whose
pointer outlived it) is likely to be overwritten and show up as wrong bytes."""
import ctypes
import random

import numpy as np
import pytest

import range_coder_rust_amd as rc
from range_coder_rust_amd import _native as N
from oracle import cpu, ref_literal as R


def _addr(p):
    if isinstance(p, ctypes.Array):
        return ctypes.addressof(p)
    if isinstance(p, ctypes.c_void_p):
        return p.value or 0
    if isinstance(p, (bytes, bytearray)):
        return None
    return int(p)


class _OracleLib:
    """rc_stream_*_host over the C oracle (host memory in, host memory out)."""

    def __init__(self):
        self.calls = {"encode": 0, "decode": 0}
        self.sizes = []

    @staticmethod
    def _scratch(nbytes):  # reuse bait for a freed caller buffer
        return [np.full(max(int(nbytes), 1), 0xA5, np.uint8) for _ in range(4)]

    def rc_stream_encode_host(self, h, st_ref, trip, n, out, cap, out_len_ref, nb, finish, fl_ref):
        self.calls["encode"] += 1
        self.sizes.append(int(n))
        bait = self._scratch(12 * n)
        t = np.frombuffer(ctypes.string_at(_addr(trip), 12 * n), np.uint32).reshape(-1, 3) \
            if n else np.zeros((0, 3), np.uint32)
        del bait
        st = st_ref._obj
        ost = cpu.Stream.from_buffer_copy(st)
        f, b, cnt = cpu.stream_encode(ost, t, finish=bool(finish), cap=int(cap))
        ctypes.memmove(ctypes.addressof(st), ctypes.addressof(ost), ctypes.sizeof(ost))
        if b:
            ctypes.memmove(_addr(out), b, len(b))
        if len(cnt):
            ctypes.memmove(_addr(nb), cnt.astype(np.uint8).tobytes(), len(cnt))
        out_len_ref._obj.value = len(b)
        fl_ref._obj.value = f
        return N.RC_E_CHUNK if f else N.RC_OK

    def rc_stream_decode_host(self, h, c, cum, na, total, st_ref, code, code_len, out, n, fl_ref):
        self.calls["decode"] += 1
        cc = np.frombuffer(c, np.uint32)[:na] if isinstance(c, bytes) else \
            np.frombuffer(ctypes.string_at(_addr(c), 4 * na), np.uint32)
        cm = np.frombuffer(cum, np.uint32)[:na] if isinstance(cum, bytes) else \
            np.frombuffer(ctypes.string_at(_addr(cum), 4 * na), np.uint32)
        bait = self._scratch(code_len)
        code_b = ctypes.string_at(_addr(code), int(code_len)) if code_len else b""
        del bait
        st = st_ref._obj
        ost = cpu.Stream.from_buffer_copy(st)
        f, s = cpu.stream_decode(ost, cc, cm, int(total), code_b, int(n))
        ctypes.memmove(ctypes.addressof(st), ctypes.addressof(ost), ctypes.sizeof(ost))
        if len(s):
            ctypes.memmove(_addr(out), s.astype(np.uint8).tobytes(), len(s))
        fl_ref._obj.value = f
        return N.RC_E_CHUNK if f else N.RC_OK


class _Ctx:
    def __init__(self):
        self._lib = _OracleLib()
        self.handle = ctypes.c_void_p(1)


SAMPLE = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]


class Adaptive(rc.FreqTable):
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


def test_sample_round_trip_and_bytes():
    ctx = _Ctx()
    sd = rc.FreqTable(10)
    for i in SAMPLE:
        sd.add_alphabet_freq(i)
    sd.calc_cum()
    enc = rc.Encoder(ctx)
    rets = [enc.encode(sd, i) for i in SAMPLE]
    code = enc.finish()
    assert code.hex() == "64475f8970365a2f83b20246c0"
    ref = R.Encoder()
    rt = R.FreqTable.from_counts(sd.c)
    assert [int(r) for r in rets] == [ref.encode(rt, i) for i in SAMPLE]
    dec = rc.Decoder(code, ctx=ctx)
    assert [dec.decode(sd) for _ in SAMPLE] == SAMPLE


@pytest.mark.parametrize("n,count_every", [(300, 0), (300, 1), (3000, 0), (3000, 7)])
def test_adaptive_encode_flushes(n, count_every):
    """Staged triples flushed at peek_code / a ByteCount's value / finish: small flushes (<= 64
    symbols, reused ctypes buffers) and large ones (numpy arrays) give the reference's bytes."""
    ctx = _Ctx()
    syms = _zipfish(n, n + count_every)
    m = Adaptive(256, 32, 4000, 64)
    ref_m = R.AdaptiveModel(256, 32, 4000, 64)
    ref = R.Encoder()
    enc = rc.Encoder(ctx)
    for i, s in enumerate(syms):
        b = enc.encode(m, s)
        want = ref.encode(ref_m, s)
        if count_every and i % count_every == 0:
            assert int(b) == want, i
        m.update(s, i)
        ref_m.update(s, i)
        if i in (0, 63, 64, 65, 1000):
            assert enc.peek_code() == bytes(ref.code)
    assert enc.finish() == bytes(ref.finish())
    if not count_every and n > 300:
        assert max(ctx._lib.sizes) > 64  # the large-flush path ran


def test_adaptive_decode_rederives_per_symbol():
    ctx = _Ctx()
    syms = _zipfish(2000, 2)
    code = R.encode_adaptive_stream(256, 32, 4000, 64, syms)
    m = Adaptive(256, 32, 4000, 64)
    ref = R.Decoder(code)
    ref_m = R.AdaptiveModel(256, 32, 4000, 64)
    dec = rc.Decoder(code, ctx=ctx)
    for i in range(len(syms)):
        s = dec.decode(m)
        assert s == ref.decode(ref_m) == syms[i], i
        m.update(s, i)
        ref_m.update(s, i)
        if i in (0, 9, 1000, 1999):
            assert dec.data() == ref.data
            assert dec.range_coder() == rc.RangeCoder(ref.range_coder.lower_bound,
                                                      ref.range_coder.range)


def test_static_decode_ahead_blocks_and_midblock_state():
    """A static table decodes ahead in doubling blocks; range_coder() / data() asked inside a
    block re-derive the state there, and a table switch mid-block restarts from it."""
    ctx = _Ctx()
    rng = random.Random(4)
    t1 = rc.FreqTable.from_counts([rng.randint(1, 50) for _ in range(40)])
    t2 = rc.FreqTable.from_counts([rng.randint(1, 50) for _ in range(40)])
    syms = [rng.randrange(40) for _ in range(700)]
    which = [t1 if i < 500 else t2 for i in range(700)]
    ref_e = R.Encoder()
    rt = {id(t1): R.FreqTable.from_counts(t1.c), id(t2): R.FreqTable.from_counts(t2.c)}
    for s, t in zip(syms, which):
        ref_e.encode(rt[id(t)], s)
    code = bytes(ref_e.finish())
    ref = R.Decoder(code)
    dec = rc.Decoder(code, ctx=ctx)
    for i, t in enumerate(which):
        assert dec.decode(t) == ref.decode(rt[id(t)]) == syms[i], i
        if i in (3, 100, 257, 499, 500, 650):
            assert dec.data() == ref.data
            assert dec.range_coder() == rc.RangeCoder(ref.range_coder.lower_bound,
                                                      ref.range_coder.range)
    # far fewer GPU calls than symbols: the blocks doubled
    assert ctx._lib.calls["decode"] < 100


class OwnFindIndex(rc.FreqTable):
    def find_index(self, decoder):  # a linear scan (the canonical inverse, found another way)
        r = decoder.range_coder()
        rf = ((decoder.data() - r.lower_bound()) & ((1 << 64) - 1)) // (r.range() // self.total)
        i = 0
        while i + 1 < len(self.c) and self.cum[i + 1] <= rf:
            i += 1
        return i


def test_own_find_index_is_called_per_symbol():
    ctx = _Ctx()
    rng = random.Random(5)
    counts = [rng.randint(1, 30) for _ in range(20)]
    t = OwnFindIndex(20)
    t.c = list(counts)
    t.calc_cum()
    syms = [rng.randrange(20) for _ in range(300)]
    ref_e = R.Encoder()
    rt = R.FreqTable.from_counts(counts)
    for s in syms:
        ref_e.encode(rt, s)
    dec = rc.Decoder(bytes(ref_e.finish()), ctx=ctx)
    assert [dec.decode(t) for _ in syms] == syms
    assert ctx._lib.calls["decode"] >= len(syms)


def test_errors_at_the_reference_call():
    ctx = _Ctx()
    t = rc.FreqTable.from_counts([3, 0, 5])
    enc = rc.Encoder(ctx)
    with pytest.raises(rc.ZeroFrequencyError):
        enc.encode(t, 1)  # c_freq == 0: the reference would never terminate
    enc.encode(t, 0)
    enc.finish()
    with pytest.raises(rc.FinishedError):
        enc.encode(t, 0)
    with pytest.raises(rc.TruncatedStreamError):
        rc.Decoder(b"\x00" * 7, ctx=ctx)
    dec = rc.Decoder(b"\x00" * 8, ctx=ctx)  # 8 bytes: the data window, no symbol bytes
    t1 = rc.FreqTable.from_counts([1] * 256)
    with pytest.raises(rc.RangeCoderError):
        for _ in range(16):
            dec.decode(t1)  # runs out of code bytes: decoder.rs:33 panics


# ---- the C++ mirror (include/range_coder.hpp), built against the oracle-backed stand-in ----
import os  # noqa: E402
import subprocess  # noqa: E402

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cpp_examples(tmp_path_factory):
    d = tmp_path_factory.mktemp("cpp_mirror")
    exes = {}
    for name in ("sample_impl", "adaptive_impl", "find_index_impl"):
        exe = str(d / name)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(_ROOT, "include"),
                        os.path.join(_ROOT, "examples", name + ".cpp"),
                        os.path.join(_ROOT, "tests", "native", "oracle_backed_rc.cpp"),
                        "-x", "c", os.path.join(_ROOT, "oracle", "rc_oracle.c"),
                        "-o", exe], check=True)
        exes[name] = exe
    return exes


def test_cpp_sample_impl_on_cpu(cpp_examples):
    r = subprocess.run([cpp_examples["sample_impl"]], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "output : 0x64475f8970365a2f83b20246c0" in r.stdout and "test passed" in r.stdout


def _xorshift_syms(n, seed):  # examples/adaptive_impl.cpp's symbol generator
    x, out, M = seed, [], (1 << 64) - 1
    for _ in range(n):
        x ^= (x << 13) & M
        x ^= x >> 7
        x ^= (x << 17) & M
        r = x % 1000
        out.append(r % 4 if r < 500 else (r % 32 if r < 800 else r % 256))
    return out


def test_cpp_caller_adaptive_model_on_cpu(cpp_examples):
    n, seed = 3000, 5
    r = subprocess.run([cpp_examples["adaptive_impl"], str(n), str(seed)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == R.encode_adaptive_stream(256, 32, 4000, 64,
                                                        _xorshift_syms(n, seed)).hex()


def test_cpp_find_index_on_cpu(cpp_examples):
    r = subprocess.run([cpp_examples["find_index_impl"]], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "find_index called 16 times" in r.stdout and "test passed" in r.stdout
