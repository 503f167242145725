"""CPU tests of model construction: the library's host quantizer
(rc_quantize_counts, called through the C ABI without a GPU) against the oracle restatement
(oracle/model_build.py), and the oracle against the reference's own sample table."""
import math

import numpy as np
import pytest

from oracle import model_build as O
from range_coder_rust_amd import api
from range_coder_rust_amd.model_build import quantize_counts

# examples/sample_impl.rs:74 test data; its FreqTable (add_alphabet_freq + calc_cum, :85-90)
SAMPLE = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]


def test_oracle_exact_table_is_the_samples_freqtable():
    counts = O.histogram(SAMPLE, 10)
    assert list(counts) == [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    c, cum, total = O.quantize_counts(counts, 0)
    assert cum == [0, 1, 6, 8, 8, 10, 12, 13, 14, 15] and total == 16  # K1's table
    t = api.FreqTable(10)
    for s in SAMPLE:
        t.add_alphabet_freq(s)
    t.calc_cum()
    assert t.c == c and t.cum == cum and t.total == total


def test_library_exact_table_matches():
    c, cum, total = quantize_counts(O.histogram(SAMPLE, 10), 0)
    assert list(c) == [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    assert list(cum) == [0, 1, 6, 8, 8, 10, 12, 13, 14, 15] and total == 16


def _cases():
    rng = np.random.default_rng(7)
    out = []
    for n in (1, 2, 3, 10, 255, 256):
        for kind in ("uniform", "zipf", "sparse", "huge", "zeros"):
            if kind == "uniform":
                cnt = rng.integers(0, 1000, n)
            elif kind == "zipf":
                cnt = (1e7 / np.arange(1, n + 1) ** 1.2).astype(np.int64)
            elif kind == "sparse":
                cnt = rng.integers(0, 5, n) * (rng.random(n) < 0.2)
            elif kind == "huge":
                cnt = rng.integers(0, 1 << 40, n)
            else:
                cnt = np.zeros(n, np.int64)
            for T in (0, n, 256, 4096, 1 << 16, (1 << 16) + 7, 1 << 31, (1 << 32) - 1, 1 << 32):
                for fl in (0, O.Q_ALL_SYMBOLS):
                    out.append((cnt.astype(np.uint64), T, fl))
    return out


@pytest.mark.parametrize("idx", range(0, 540, 1))
def test_library_quantizer_matches_oracle(idx):
    cases = _cases()
    if idx >= len(cases):
        pytest.skip("beyond case list")
    cnt, T, fl = cases[idx]
    want = O.quantize_counts(cnt, T, fl)
    if want is None:
        with pytest.raises(ValueError):
            quantize_counts(cnt, T, bool(fl))
        return
    c, cum, total = quantize_counts(cnt, T, bool(fl))
    assert list(c) == want[0] and list(cum) == want[1] and total == want[2]
    if T:
        assert total == T
        assert all(ci >= 1 for ci, k in zip(c, cnt) if k > 0 or fl)


def test_quantized_tables_are_valid_models():
    # every scaled table is a valid rc_model table: cum[0] == 0, cum[i+1] == cum[i] + c[i]
    for cnt, T, fl in _cases()[::7]:
        r = O.quantize_counts(cnt, T, fl)
        if r is None:
            continue
        c, cum, total = r
        assert cum[0] == 0 and all(cum[i + 1] == cum[i] + c[i] for i in range(len(c) - 1))
        assert cum[-1] + c[-1] == total


def test_ideal_code_length_oracle_matches_pmodel():
    t = api.FreqTable.from_counts([1, 5, 2, 0, 2, 2, 1, 1, 1, 1])
    for i in range(10):
        o = O.ideal_code_length(t.c[i], t.total)
        if t.c[i] == 0:
            assert o is None
            with pytest.raises(api.RangeCoderError):
                t.ideal_code_length(i)
        else:
            assert o == t.ideal_code_length(i)
    assert O.ideal_code_length(1, 16) == 4.0


def test_ideal_bits_oracle():
    c = [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    h = np.zeros((2, 256), np.int64)
    for s in SAMPLE:
        h[0, s] += 1
    h[1, 3] = 1  # c == 0: no code length
    bits = O.ideal_bits(h, c, 16)
    want = sum(math.log2(16 / c[s]) for s in SAMPLE)
    assert abs(bits[0] - want) < 1e-12 * want and math.isinf(bits[1])
