"""The resumable-stream oracle (orc_stream_encode / orc_stream_decode, the restatement behind the
rc_stream_* entry points) against the literal Python restatement (oracle/ref_literal.py) with the
reference's per-call PModel semantics: models changed by the caller between calls, arbitrary
(even inconsistent) tables, garbage streams, and every panic / endless loop of the reference
mapped to its flag."""
import random

import numpy as np
import pytest

from oracle import cpu, ref_literal as R


class Table:
    """A PModel over fixed (c, cum, total) lists, with FreqTable::find_index (sample_impl.rs:27-45)
    — the tables need not be consistent."""

    def __init__(self, c, cum, total):
        self.c, self.cum, self.total = list(c), list(cum), total

    def alphabet_count(self):
        return len(self.c)

    def c_freq(self, i):
        return self.c[i]

    def cum_freq(self, i):
        return self.cum[i]

    def total_freq(self):
        return self.total

    find_index = R.FreqTable.find_index


def _flag_of(exc):
    """The rc flag a ref_literal exception maps to."""
    msg = str(exc)
    if isinstance(exc, ZeroDivisionError) or isinstance(exc, R.RangeCoderError) or \
            "UpperBoundOverflow" in msg:
        return cpu.F_BAD_MODEL
    if "does not terminate" in msg:
        return "endless"
    if "pop_front" in msg:
        return cpu.F_TRUNCATED
    raise exc


def _ref_encode(models_and_syms):
    """ref_literal Encoder with the model given per call: (bytes, counts, flag)."""
    enc = R.Encoder()
    counts = []
    for m, s in models_and_syms:
        try:
            counts.append(enc.encode(m, s))
        except Exception as e:  # noqa: BLE001 — a reference panic
            f = _flag_of(e)
            return bytes(enc.code), counts, cpu.F_ZERO_FREQ if f == "endless" else f, enc
    return bytes(enc.code), counts, 0, enc


def test_caller_adaptive_model_encode_matches_reference():
    rng = random.Random(1)
    syms = [min(255, int(rng.paretovariate(1.2))) for _ in range(3000)]
    m = R.AdaptiveModel(256, 32, 57343, 256)
    trip, pairs = [], []
    for i, s in enumerate(syms):
        trip.append((m.c_freq(s), m.cum_freq(s), m.total_freq()))
        pairs.append((R.FreqTable.from_counts(list(m.c)), s))
        m.update(s, i)
    code, counts, f, enc = _ref_encode(pairs)
    assert f == 0
    st = cpu.Stream.fresh()
    fl, got, nb = cpu.stream_encode(st, trip, finish=True)
    assert fl == 0 and got == bytes(enc.finish()) == R.encode_adaptive_stream(256, 32, 57343,
                                                                              256, syms)
    assert nb.tolist() == counts
    # resumable: the same stream coded in random pieces
    st2 = cpu.Stream.fresh()
    out, nbs, i = b"", [], 0
    while i < len(trip):
        j = min(len(trip), i + rng.randint(0, 400))
        f2, b2, n2 = cpu.stream_encode(st2, trip[i:j])
        assert f2 == 0
        out, i = out + b2, j
        nbs += n2.tolist()
    f2, b2, _ = cpu.stream_encode(st2, np.zeros((0, 3)), finish=True)
    assert f2 == 0 and out + b2 == got and nbs == counts and st2.tuple() == st.tuple()


def test_caller_adaptive_model_decode_matches_reference():
    rng = random.Random(2)
    syms = [min(255, int(rng.paretovariate(1.1))) for _ in range(2000)]
    code = R.encode_adaptive_stream(256, 32, 57343, 256, syms)
    m = R.AdaptiveModel(256, 32, 57343, 256)
    st = cpu.Stream.fresh()
    out = []
    for i in range(len(syms)):
        f, s = cpu.stream_decode(st, m.c, m.cum, m.total, code, 1)
        assert f == 0
        out.append(int(s[0]))
        m.update(out[-1], i)
    assert out == syms
    assert st.pos == len(code)  # every byte consumed, as the reference's deque empties


@pytest.mark.parametrize("seed", range(30))
def test_random_tables_encode_vs_reference(seed):
    """Arbitrary per-symbol triples: bytes, counts, state and the panic flags agree."""
    rng = random.Random(seed)
    n = rng.randint(1, 60)
    trip = []
    for _ in range(n):
        kind = rng.random()
        total = rng.choice([1, 2, 255, 256, 65536, rng.randint(1, 2 ** 32 - 1)])
        if kind < 0.05:
            total = 0
        c = rng.randint(0, total) if kind > 0.1 else rng.randint(0, 2 ** 32 - 1)
        cum = rng.randint(0, max(0, total - c)) if kind > 0.2 else rng.randint(0, 2 ** 32 - 1)
        if kind > 0.3 and c == 0:
            c = 1
        trip.append((c, cum, total))
    pairs = [(Table([c], [cum], t), 0) for c, cum, t in trip]
    code, counts, f, enc = _ref_encode(pairs)
    st = cpu.Stream.fresh()
    fl, got, nb = cpu.stream_encode(st, trip)
    assert fl == f and got == code and nb.tolist() == counts
    assert (st.lower_bound, st.range) == (enc.range_coder.lower_bound, enc.range_coder.range) \
        or f  # after a panic the reference state is torn; ours stops before the symbol
    assert st.n == len(counts)


@pytest.mark.parametrize("seed", range(30))
def test_random_tables_decode_vs_reference(seed):
    """Garbage code, random (possibly inconsistent) tables: symbols and the panic flags agree."""
    rng = random.Random(100 + seed)
    na = rng.randint(1, 12)
    code = bytes(rng.randrange(256) for _ in range(rng.randint(8, 40)))
    dec = R.Decoder(code)
    st = cpu.Stream.fresh()
    for _ in range(rng.randint(1, 30)):
        c = [rng.choice([0, 1, rng.randint(0, 1000)]) for _ in range(na)]
        if rng.random() < 0.6:
            cum = list(np.concatenate([[0], np.cumsum(c)[:-1]]))
            total = int(sum(c)) + rng.choice([0, 0, 1])
        else:
            cum = sorted(rng.randint(0, 2000) for _ in range(na))
            total = rng.randint(0, 2000)
        t = Table(c, [int(x) for x in cum], total)
        try:
            want, wf = dec.decode(t), 0
        except Exception as e:  # noqa: BLE001
            want, wf = None, _flag_of(e)
            wf = cpu.F_CORRUPT if wf == "endless" else wf
        f, got = cpu.stream_decode(st, c, t.cum, total, code, 1)
        assert f == wf
        if wf:
            break
        assert int(got[0]) == want
        assert (st.lower_bound, st.range, st.data) == \
            (dec.range_coder.lower_bound, dec.range_coder.range, dec.data)


def test_stream_flags_are_sticky_and_finish_consumes():
    st = cpu.Stream.fresh()
    f, b, _ = cpu.stream_encode(st, [(1, 0, 2)], finish=True)
    assert f == 0 and len(b) == 8 and st.stage == 2  # no byte settles, then finish
    f, b, _ = cpu.stream_encode(st, [(1, 0, 2)])
    assert f == cpu.F_FINISHED and b == b""
    st = cpu.Stream.fresh()
    assert cpu.stream_encode(st, [(0, 0, 2)])[0] == cpu.F_ZERO_FREQ
    assert cpu.stream_encode(st, [(1, 0, 2)])[0] == cpu.F_ZERO_FREQ and st.n == 0
    st = cpu.Stream.fresh()  # capacity: refused without a change, not sticky
    f, b, _ = cpu.stream_encode(st, [(1, 0, 2)] * 3, cap=20)
    assert f == cpu.F_CAPACITY and st.flags == 0 and st.n == 0
    st = cpu.Stream.fresh()
    assert cpu.stream_decode(st, [1], [0], 1, b"\0" * 7, 1)[0] == cpu.F_TRUNCATED
