"""range_par_total (range_coder.rs:38-40) on the device, in the three forms the static coders use
(rc_static.h): the small-model f64 two-step (256 <= total <= 2^16, not a power of two), the
64 x 64 magic product and the power-of-two shift, under the decoders' f32 rounding mode, run by
the library's internal test hook (rc_test_range_par_total_, rc_kernels.hip) and compared with
exact integer division on the edge cases tests/test_div_f64.py restates in Python: the full
64-bit span, exact multiples of total and their neighbours, every total's extremes (ADVICE r04:
the restatement cannot see the device's rounding, __umul24's operand truncation or the
compiler's contraction of the f64 ops)."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SMALL = [257, 300, 1000, 2049, 10000, 16385, 32769, 65521, 65533, 65535]
LARGE = [1, 3, 255, 65537, 1 << 20 | 1, 0xFFFFFFFF, 0x80000001]
POW2 = [1, 2, 256, 1 << 12, 1 << 16, 1 << 24, 1 << 31]


def _cases(t, rnd, n=3000):
    top = 2 ** 64 - 1
    m = t * (2 ** 64 // t)
    cases = [top, top - 1, 2 ** 32, 2 ** 32 - 1, 2 ** 63, m, m - 1, t, t - 1, t + 1, 1 << 48,
             (1 << 48) - 1, ((2 ** 32 - 1) << 32) | 0xFFFFFFFF, (2 ** 32 - 1) << 32]
    for _ in range(n):
        k = rnd.choice([64, 63, 56, 48, 40, 33])
        cases.append(rnd.getrandbits(k))
        mm = rnd.getrandbits(64) // t * t
        cases += [mm, max(mm - 1, 0), min(mm + t - 1, top)]
    return [c for c in cases if 0 <= c <= top]


def _run(totals_cases):
    import range_coder_rust_amd as rc
    from range_coder_rust_amd import _native as N
    ctx = rc.default_context(0)
    L = ctx._lib
    L.rc_test_range_par_total_.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p]
    L.rc_test_range_par_total_.restype = ctypes.c_int
    ranges = np.array([r for _, r in totals_cases], dtype=np.uint64)
    totals = np.array([t for t, _ in totals_cases], dtype=np.uint32)
    out = np.zeros(3 * len(ranges), dtype=np.uint64)
    N.check(L.rc_test_range_par_total_(ctx.handle, ranges.ctypes.data, totals.ctypes.data,
                                       len(ranges), out.ctypes.data), "rc_test_range_par_total_")
    return out.reshape(-1, 3)


def test_small_model_f64_form_on_device():
    rnd = random.Random(5)
    tc = [(t, r) for t in SMALL for r in _cases(t, rnd)]
    got = _run(tc)
    bad = [(t, r, int(g)) for (t, r), g in zip(tc, got[:, 0]) if int(g) != r // t]
    assert not bad, bad[:5]
    bad = [(t, r) for (t, r), g in zip(tc, got[:, 1]) if int(g) != r // t]
    assert not bad, bad[:5]


def test_magic_form_on_device():
    rnd = random.Random(6)
    tc = [(t, r) for t in LARGE + SMALL for r in _cases(t, rnd, 1500)]
    got = _run(tc)
    bad = [(t, r, int(g)) for (t, r), g in zip(tc, got[:, 1]) if int(g) != r // t]
    assert not bad, bad[:5]


def test_pow2_form_on_device():
    rnd = random.Random(7)
    tc = [(t, r) for t in POW2 for r in _cases(t, rnd, 500)]
    got = _run(tc)
    bad = [(t, r, int(g)) for (t, r), g in zip(tc, got[:, 2]) if int(g) != r // t]
    assert not bad, bad[:5]
