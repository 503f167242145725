"""Host logic of the Python mirror that needs no GPU: ByteCount's numeric behaviour (the u32
that Encoder::encode returns, encoder.rs:34-36), the reference errors a flagged symbol maps to
(error.rs:3-13 with param_update's arithmetic, range_coder.rs:53-81, :138-146), and which models
keep the decode-ahead path (pmodel.rs:12)."""
import pytest

import range_coder_rust_amd as rc
from range_coder_rust_amd import api
from range_coder_rust_amd import _native as N

M64 = (1 << 64) - 1


class _Counts:
    def __init__(self, counts):
        self.counts = counts

    def _count(self, i):
        return self.counts[i]


def test_bytecount_behaves_like_the_u32():
    enc = _Counts([0, 2, 3])
    z, two, three = (rc.ByteCount(enc, i) for i in range(3))
    assert not z and bool(two)
    assert two + 1 == 3 and 1 + two == 3 and two - 1 == 1 and 5 - two == 3
    assert two * 3 == 6 and 3 * two == 6 and three // 2 == 1 and float(three) == 3.0
    assert sum([two, three]) == 5 and two < three and int(three) == 3 and [9, 8, 7][two] == 7


def test_lower_bound_overflow_mapping():
    low, rng = 0xCFFFFFFFFFFFFFFD, 0x0FFFFFFFFFFFFFFF
    with pytest.raises(rc.LowerBoundOverflow) as ei:
        api._raise_bad_model(low, rng, 1, 0xFFFFFFFF, 2, "t")
    r = rng // 2
    assert (ei.value.lower_bound, ei.value.add_val, ei.value.range) == \
        (low, (r * 0xFFFFFFFF) & M64, r)
    assert isinstance(ei.value, rc.BadModelError)


def test_upper_bound_overflow_mapping():
    # no lower-bound overflow, but low + add + r*c wraps: c > total - cum
    low, rng = 1 << 62, 1 << 63
    with pytest.raises(rc.UpperBoundOverflow) as ei:
        api._raise_bad_model(low, rng, 3, 1, 2, "t")
    r = rng // 2
    assert (ei.value.lower_bound, ei.value.range) == (low + r, (r * 3) & M64)


def test_divide_by_zero_mapping():
    with pytest.raises(rc.BadModelError, match="divide by zero"):
        api._raise_bad_model(0, M64, 1, 0, 0, "t")


def test_decode_error_uses_the_reference_index():
    """The decode-side payload comes from the index FreqTable::find_index picks at the failing
    state (here: a table whose last entry's cum overflows the lower bound)."""
    st = N.StreamState(0xF000000000000000, 0x0800000000000000, 0xF7F0000000000000, 8, 0, 0, 1)
    c, cum, total = (1, 1, 2), (0, 1, 0xFFFFFFFF), 3
    sig = (c, cum, total)
    rf = api._find_index_rfreq(st, total)
    with pytest.raises(rc.BadModelError) as ei:
        api._decode_error(st, sig, N.F_BAD_MODEL, "t")
    # the binary search of sample_impl.rs:31-44 over cum with rf
    idx = 0 if rf < 1 else (1 if rf < 0xFFFFFFFF else 2)
    r = st.range // total
    if isinstance(ei.value, rc.LowerBoundOverflow):
        assert ei.value.add_val == (r * cum[idx]) & M64
    with pytest.raises(rc.TruncatedStreamError):
        api._decode_error(st, sig, N.F_TRUNCATED, "t")


class _Own(rc.FreqTable):
    def find_index(self, decoder):
        return 0


class _OwnCanonical(rc.FreqTable):
    canonical_find_index = True

    def find_index(self, decoder):
        return 0


class _Sub(_Own):
    pass


class _Duck:
    def find_index(self, decoder):
        return 0


def test_which_models_keep_the_decode_ahead_path():
    assert api._canonical_find_index(rc.FreqTable(4))
    assert not api._canonical_find_index(_Own(4))
    assert api._canonical_find_index(_OwnCanonical(4))
    assert not api._canonical_find_index(_Sub(4))  # inherits a non-canonical override
    assert not api._canonical_find_index(_Duck())

    class P(rc.PModel):
        pass

    assert api._canonical_find_index(P())


def test_canonical_check_follows_a_class_patched_after_first_decode():
    """the per-class cache is keyed by what the class resolves now, so setting
    find_index (or the flag) on a class after its first check is seen."""
    class Q(rc.FreqTable):
        pass

    assert api._canonical_find_index(Q(4))
    Q.find_index = lambda self, decoder: 0
    assert not api._canonical_find_index(Q(4))
    Q.canonical_find_index = True
    assert api._canonical_find_index(Q(4))
    del Q.find_index
    del Q.canonical_find_index
    assert api._canonical_find_index(Q(4))
