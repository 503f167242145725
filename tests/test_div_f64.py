"""range_par_total (range_coder.rs:38-40) for small non-power-of-two models as the decoders and the
encoder compute it (rc_static.h range_par_total, SM branch): two f64 steps with 1/total rounded
up.  Restated here in Python floats (IEEE f64, round to nearest, as the kernels run f64) and
checked against exact integer division on ranges that stress the bound: the full 64-bit span,
exact multiples of total and their neighbours, every total's extremes."""
import math
import random
from fractions import Fraction

import pytest


def inv_up(t):
    u = 1.0 / t  # rc_kernels.hip: nextafter when fma(u, t, -1) < 0
    if Fraction(u) * t < 1:
        u = math.nextafter(u, 2.0)
    return u


def range_par_total_f64(rng, t, u):
    rh, rl = rng >> 32, rng & 0xFFFFFFFF
    q1 = int(rh * u)                                  # v_mul_f64, v_cvt_u32_f64
    assert q1 < 1 << 24                               # the 24-bit multiply's operand range
    rem = (rh - ((q1 * t) & 0xFFFFFFFF)) & 0xFFFFFFFF  # __umul24, v_sub_u32
    q0 = int(float(rem * 2 ** 32 + rl) * u)           # the fma is exact: n < 2^48
    assert q0 < 1 << 32
    return (q1 << 32) | q0


@pytest.mark.parametrize("t", [257, 300, 1000, 2049, 10000, 16385, 32769, 65521, 65533, 65535])
def test_matches_integer_division(t):
    rnd = random.Random(t)
    u = inv_up(t)
    cases = [2 ** 64 - 1, 2 ** 32, 2 ** 32 - 1, t * (2 ** 64 // t), t * (2 ** 64 // t) - 1]
    for _ in range(4000):
        k = rnd.choice([64, 63, 56, 48, 40, 33])
        cases.append(rnd.getrandbits(k))
        m = rnd.getrandbits(64) // t * t
        cases += [m, max(m - 1, 0), min(m + t - 1, 2 ** 64 - 1)]
    for r in cases:
        assert range_par_total_f64(r, t, u) == r // t, (r, t)


def test_inv_up_rounds_up():
    for t in range(257, 65536, 97):
        assert Fraction(inv_up(t)) * t >= 1
