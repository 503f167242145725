"""Literal pure-Python restatement of diegodox/range_coder_rust (TEST INFRASTRUCTURE ONLY).

This is a second, independent oracle used to cross-check ``oracle/rc_oracle.c`` on small
inputs.  It follows the Rust source statement by statement, keeping the reference's data
structures (``VecDeque`` -> ``collections.deque``), its explicit ``overflowing_add`` checks
(raised as ``RangeCoderError``) and its panics (raised as ``ReferencePanic``).  Rust release
semantics apply to unchecked u64 arithmetic (wrap modulo 2**64).  Only tests/ import it.

Parity status: the Rust reference cannot be built in this image (no rustc/cargo), so this file
is a restatement, not an execution of the reference.  See oracle/rc_oracle.h.
"""
from collections import deque

U64 = (1 << 64) - 1


class RangeCoderError(Exception):
    """error.rs:3-13"""


class ReferencePanic(Exception):
    """A point where the Rust reference panics (unwrap on None / Err)."""


class RangeCoder:
    """range_coder.rs:7-147"""

    TOP8 = 1 << (64 - 8)  # :23
    TOP16 = 1 << (64 - 16)  # :24

    def __init__(self):  # Default, :13-20
        self.lower_bound = 0
        self.range = U64

    def range_par_total(self, total_freq):  # :38-40
        return self.range // total_freq

    def param_update(self, c_freq, cum_freq, total_freq, max_iter=1 << 12):  # :53-92
        out_bytes = deque()
        range_par_total = self.range_par_total(total_freq)
        self.range = (range_par_total * c_freq) & U64  # :65
        add = (range_par_total * cum_freq) & U64
        if self.lower_bound + add > U64:  # :68-81 overflowing_add
            raise RangeCoderError("LowerBoundOverflow")
        self.lower_bound = self.lower_bound + add
        it = 0
        while True:  # :83-85
            b = self.no_carry_expansion()
            if b is None:
                break
            out_bytes.append(b)
            it += 1
            if it > max_iter:  # the reference never terminates here (c_freq == 0)
                raise ReferencePanic("no_carry_expansion does not terminate")
        while True:  # :87-89
            b = self.range_reduction_expansion()
            if b is None:
                break
            out_bytes.append(b)
        return out_bytes

    def left_shift(self):  # :95-100
        tmp = (self.lower_bound >> (64 - 8)) & 0xFF
        self.range = (self.range << 8) & U64
        self.lower_bound = (self.lower_bound << 8) & U64
        return tmp

    def no_carry_expansion(self):  # :110-116
        if self.lower_bound ^ self.upper_bound() < self.TOP8:
            return self.left_shift()
        return None

    def range_reduction_expansion(self):  # :126-135
        if self.range < self.TOP16:
            self.range = (~self.lower_bound & U64) & (self.TOP16 - 1)
            return self.left_shift()
        return None

    def upper_bound(self):  # :138-146
        s = self.lower_bound + self.range
        if s > U64:
            raise ReferencePanic("UpperBoundOverflow unwrap")
        return s


class Encoder:
    """encoder.rs:7-55"""

    def __init__(self):
        self.range_coder = RangeCoder()
        self.code = deque()

    def encode(self, pmodel, index):  # :24-37
        outbytes = self.range_coder.param_update(
            pmodel.c_freq(index), pmodel.cum_freq(index), pmodel.total_freq())
        n = len(outbytes)
        self.code.extend(outbytes)
        return n

    def finish(self):  # :40-46
        for _ in range(8):
            self.code.append(self.range_coder.left_shift())
        return self.code


class Decoder:
    """decoder.rs:6-55"""

    def __init__(self, code):  # :14-23
        self.range_coder = RangeCoder()
        self.data = 0
        self.buffer = deque(code)
        self.shift_left_buffer(8)

    def shift_left_buffer(self, n):  # :31-35
        for _ in range(n):
            if not self.buffer:
                raise ReferencePanic("pop_front on empty buffer")
            self.data = ((self.data << 8) & U64) | self.buffer.popleft()

    def decode(self, pmodel):  # :38-54
        idx = pmodel.find_index(self)
        n = len(self.range_coder.param_update(
            pmodel.c_freq(idx), pmodel.cum_freq(idx), pmodel.total_freq()))
        self.shift_left_buffer(n)
        return idx


class FreqTable:
    """examples/sample_impl.rs:4-70"""

    def __init__(self, alphabet_count):  # :49-54
        self.total = 0
        self.c = [0] * alphabet_count
        self.cum = [0] * alphabet_count

    def alphabet_count(self):  # :55-57
        return len(self.c)

    def add_alphabet_freq(self, i):  # :58-60
        self.c[i] += 1

    def calc_cum(self):  # :61-69
        t = 0
        for i in range(len(self.c)):
            self.cum[i] = t
            t += self.c[i]
        self.total = t

    def c_freq(self, i):  # :18-20
        if i >= len(self.c):
            raise ReferencePanic("get(index).unwrap()")
        return self.c[i]

    def cum_freq(self, i):  # :21-23
        if i >= len(self.cum):
            raise ReferencePanic("get(index).unwrap()")
        return self.cum[i]

    def total_freq(self):  # :24-26
        return self.total

    def find_index(self, decoder):  # :27-45
        rc = decoder.range_coder
        rfreq = ((decoder.data - rc.lower_bound) & U64) // rc.range_par_total(self.total)
        left, right = 0, self.alphabet_count() - 1
        while left < right:
            mid = (left + right) // 2
            if self.cum_freq(mid + 1) <= rfreq:
                left = mid + 1
            else:
                right = mid
        return left

    @classmethod
    def from_counts(cls, counts):
        t = cls(len(counts))
        t.c = list(counts)
        t.calc_cum()
        return t


def encode_stream(table, symbols):
    enc = Encoder()
    for s in symbols:
        enc.encode(table, s)
    return bytes(enc.finish())


def decode_stream(table, code, n):
    dec = Decoder(code)
    return [dec.decode(table) for _ in range(n)]


class AdaptiveModel(FreqTable):
    """The build-defined adaptive order-0 model (not in the reference), as a
    PModel on top of FreqTable: c[i] = 1 initially; after the i-th coded symbol s (0-based),
    c[s] += inc and, every period-th symbol, halve all counts (rounding up) if the total
    exceeds limit.  Same rule as orc_encode_adaptive / orc_decode_adaptive in rc_oracle.c."""

    def __init__(self, alphabet_count, inc, limit, period):
        super().__init__(alphabet_count)
        self.inc, self.limit, self.period = inc, limit, period
        self.c = [1] * alphabet_count
        self.calc_cum()

    def update(self, s, i):
        self.c[s] += self.inc
        if (i + 1) % self.period == 0 and sum(self.c) > self.limit:
            self.c = [(x + 1) >> 1 for x in self.c]
        self.calc_cum()


def encode_adaptive_stream(n_alpha, inc, limit, period, symbols):
    m = AdaptiveModel(n_alpha, inc, limit, period)
    enc = Encoder()
    for i, s in enumerate(symbols):
        enc.encode(m, s)
        m.update(s, i)
    return bytes(enc.finish())


def decode_adaptive_stream(n_alpha, inc, limit, period, code, n):
    m = AdaptiveModel(n_alpha, inc, limit, period)
    dec = Decoder(code)
    out = []
    for i in range(n):
        s = dec.decode(m)
        m.update(s, i)
        out.append(s)
    return out
