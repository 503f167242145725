"""Host-side API of the MI355X range coder, mirroring the reference crate's public surface.

Reference surface (diegodox/range_coder_rust, src/lib.rs:1-13) and what replaces it here:

  trait PModel (src/pmodel.rs:4-41)        -> class PModel (same method names/meaning)
  FreqTable example model (sample_impl.rs)  -> class FreqTable
  Encoder::{new, encode, finish, peek_code} -> class Encoder: encode() reads the model at the
    (src/encoder.rs:14-46)                     call and stages the triple; the resumable stream
                                               kernel codes staged symbols when a result is needed
  Decoder::{new, decode, range_coder, data} -> class Decoder(code): decode() reads the model at
    (src/decoder.rs:14-54)                     the call; symbols are decoded ahead on the GPU while
                                               the table is unchanged; a PModel with its own
                                               find_index is called per symbol (see Decoder)
  error::RangeCoderError (src/error.rs)     -> RangeCoderError and subclasses (raised where
                                               the reference panics or never terminates), with
                                               LowerBoundOverflow / UpperBoundOverflow payloads

The hot path proper is the batch API (encode_batch / decode_batch / encode_chunks /
decode_chunks): many independent chunks per launch, one chunk per GPU lane, through the C ABI
of librc_amd.so (include/range_coder.h).  Tensors are torch CUDA(HIP) tensors; PyTorch is
used only for device memory and streams.  There is no CPU fallback.
"""
import ctypes
import struct
import math

import numpy as np

from . import _native as N

M64 = (1 << 64) - 1

__all__ = [
    "Context", "StaticModel", "PModel", "FreqTable", "Encoder", "Decoder", "RangeCoderError",
    "ZeroFrequencyError", "BadSymbolError", "TruncatedStreamError", "CorruptStreamError",
    "CapacityError", "ChunkTooLongError", "BadModelError", "FinishedError", "RangeCoder",
    "LowerBoundOverflow", "UpperBoundOverflow",
    "ByteCount", "encode_host_multi", "decode_host_multi", "stream_states", "stream_encode_batch", "stream_decode_batch", "encode_batch", "decode_batch", "encode_chunks", "decode_chunks",
    "default_context", "flag_names", "slot_capacity",
]


# ----------------------------------------------------------------------------- errors
class RangeCoderError(Exception):
    """src/error.rs:3-13 analogue; raised where the reference returns Err / panics."""


class ZeroFrequencyError(RangeCoderError):
    """Encoding a c_freq == 0 symbol (the reference never terminates: range_coder.rs:83-85)."""


class BadSymbolError(RangeCoderError):
    """Symbol index >= alphabet size (the reference panics: sample_impl.rs:19)."""


class TruncatedStreamError(RangeCoderError):
    """Decoder ran out of code bytes (the reference panics: decoder.rs:33)."""


class CorruptStreamError(RangeCoderError):
    """Decoder selected a zero-frequency symbol (the reference never terminates)."""


class CapacityError(RangeCoderError):
    """An encoded chunk did not fit its output slot."""


class BadModelError(RangeCoderError):
    """A (c_freq, cum_freq, total_freq) on which the reference panics: total 0 (division by
    zero, range_coder.rs:38-40), LowerBoundOverflow (:68-81) or UpperBoundOverflow
    (upper_bound().unwrap(), :138-146)."""


class LowerBoundOverflow(BadModelError):
    """RangeCoderError::LowerBoundOverflow (error.rs:5-10): lower_bound + add_val overflowed in
    param_update (range_coder.rs:68-81).  range is the narrowed range, as the reference reports
    it (self.range was updated first, :65)."""

    def __init__(self, msg, lower_bound, add_val, range_):
        super().__init__(msg)
        self.lower_bound, self.add_val, self.range = lower_bound, add_val, range_


class UpperBoundOverflow(BadModelError):
    """RangeCoderError::UpperBoundOverflow (error.rs:11): lower_bound + range overflowed in
    upper_bound() (range_coder.rs:138-146), which no_carry_expansion unwraps (a panic)."""

    def __init__(self, msg, lower_bound, range_):
        super().__init__(msg)
        self.lower_bound, self.range = lower_bound, range_


class FinishedError(RangeCoderError):
    """encode() after finish(): Encoder::finish takes the encoder by value (encoder.rs:40)."""


class ChunkTooLongError(RangeCoderError):
    """A batch chunk of more than RC_MAX_CHUNK_SYMBOLS (2^25) symbols (32-bit in-chunk stream
    positions; the stream API -- Encoder / Decoder -- has no such limit)."""


_FLAG_ERRORS = [
    (N.F_ZERO_FREQ, ZeroFrequencyError), (N.F_BAD_SYMBOL, BadSymbolError),
    (N.F_CAPACITY, CapacityError), (N.F_TRUNCATED, TruncatedStreamError),
    (N.F_CORRUPT, CorruptStreamError), (N.F_TOO_LONG, ChunkTooLongError),
    (N.F_BAD_MODEL, BadModelError), (N.F_FINISHED, FinishedError),
]


def flag_names(f):
    names = {N.F_ZERO_FREQ: "ZERO_FREQ", N.F_BAD_SYMBOL: "BAD_SYMBOL", N.F_CAPACITY: "CAPACITY",
             N.F_TRUNCATED: "TRUNCATED", N.F_CORRUPT: "CORRUPT", N.F_TOO_LONG: "TOO_LONG",
             N.F_BAD_MODEL: "BAD_MODEL", N.F_FINISHED: "FINISHED"}
    return [v for k, v in names.items() if f & k]


def _raise_for_flag(f, where):
    for bit, exc in _FLAG_ERRORS:
        if f & bit:
            raise exc(f"{where}: {'|'.join(flag_names(f))}")


def _raise_bad_model(low, range_, c, cum, total, where):
    """The reference's error for a flagged (RC_F_BAD_MODEL) symbol, with its payload.  The stream
    kernels stop before the failing symbol, so (low, range) is the state param_update started
    from; the payload is param_update's own arithmetic (range_coder.rs:53-81, :138-146), u64
    products wrapping as in a release build."""
    if total == 0:
        raise BadModelError(f"{where}: range_par_total: attempt to divide by zero")
    r = range_ // total
    nr = (r * c) & M64
    add = (r * cum) & M64
    if low + add > M64:
        raise LowerBoundOverflow(
            f"{where}: Overflow happend while lower_bound uppdating {low} + {add} , {nr}",
            low, add, nr)
    nl = low + add
    if nl + nr > M64:
        raise UpperBoundOverflow(
            f"{where}: Overflow happend when calc upper_bound {nl} + {nr}", nl, nr)
    raise BadModelError(f"{where}: BAD_MODEL")


# ----------------------------------------------------------------------------- torch glue
def _torch():
    import torch
    return torch


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _check_dev(t, name, dtype=None):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name} must be a torch tensor on a HIP device")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype not in dtype:
        raise TypeError(f"{name}: dtype {t.dtype} not in {dtype}")


class Context:
    """rc_ctx: one device, launches on the current torch stream of that device."""

    def __init__(self, device=0):
        self._lib = N.load()
        torch = _torch()
        if not torch.cuda.is_available():
            raise N.RCError(N.RC_E_NO_DEVICE, "rc_ctx_create")
        self.device = int(device)
        h = ctypes.c_void_p()
        N.check(self._lib.rc_ctx_create(self.device, ctypes.byref(h)), "rc_ctx_create")
        self.handle = h

    def bind_stream(self):
        """Point the context at torch's current stream for this device (stream-ordered)."""
        torch = _torch()
        s = torch.cuda.current_stream(self.device).cuda_stream
        N.check(self._lib.rc_ctx_set_stream(self.handle, ctypes.c_void_p(s)), "rc_ctx_set_stream")

    def synchronize(self):
        N.check(self._lib.rc_ctx_synchronize(self.handle), "rc_ctx_synchronize")

    def info(self):
        buf = ctypes.create_string_buffer(256)
        N.check(self._lib.rc_device_info(self.device, buf, 256), "rc_device_info")
        return buf.value.decode()

    def close(self):
        if getattr(self, "handle", None):
            self._lib.rc_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device=None):
    torch = _torch()
    if device is None:
        device = torch.cuda.current_device()
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


# ----------------------------------------------------------------------------- models
class PModel:
    """trait PModel (src/pmodel.rs:4-41)."""

    def c_freq(self, index):  # pmodel.rs:6
        raise NotImplementedError

    def cum_freq(self, index):  # pmodel.rs:8
        raise NotImplementedError

    def total_freq(self):  # pmodel.rs:10
        raise NotImplementedError

    def find_index(self, decoder):  # pmodel.rs:12
        """Not overridden: the decoder runs FreqTable::find_index (sample_impl.rs:27-45) itself,
        on the GPU.  Override it to decode with your own rule: Decoder.decode then calls it at
        every symbol with the decoder (range_coder() / data()), as decoder.rs:40 does, and
        applies param_update to the index it returns.  A subclass that overrides it but keeps
        FreqTable's binary-search semantics can set canonical_find_index = True to keep the
        decode-ahead path."""
        raise NotImplementedError

    def ideal_code_length(self, index):  # pmodel.rs:14-40
        p = float(self.c_freq(index))
        if p == 0.0:
            raise RangeCoderError("code length is undefind when probability is zero")
        if math.isnan(p) or math.isinf(p):
            raise RangeCoderError(
                f"code length is undefind when probability is nan or infinite as {p!r}")
        if p < 0:
            raise RangeCoderError(f"code length is undefind when probability is negative as {p}")
        return (math.log(float(self.total_freq())) - math.log(p)) / math.log(2.0)

    def alphabet_count(self):
        """Alphabet size.  Not a trait method in the reference (FreqTable::alphabet_count,
        sample_impl.rs:55-57); the GPU snapshot needs it."""
        raise NotImplementedError


class FreqTable(PModel):
    """The static frequency table of examples/sample_impl.rs:4-70."""

    def __init__(self, alphabet_count):  # FreqTable::new, :49-54
        self.total = 0
        self.c = [0] * int(alphabet_count)
        self.cum = [0] * int(alphabet_count)

    @classmethod
    def from_counts(cls, counts):
        t = cls(len(counts))
        t.c = [int(x) for x in counts]
        t.calc_cum()
        return t

    def alphabet_count(self):  # :55-57
        return len(self.c)

    def add_alphabet_freq(self, index):  # :58-60
        self.c[index] += 1

    def calc_cum(self):  # :61-69
        t = 0
        for i, ci in enumerate(self.c):
            self.cum[i] = t
            t += ci
        self.total = t

    def c_freq(self, index):  # :18-20
        if not 0 <= index < len(self.c):
            raise BadSymbolError(f"index {index} out of alphabet ({len(self.c)})")
        return self.c[index]

    def cum_freq(self, index):  # :21-23
        if not 0 <= index < len(self.cum):
            raise BadSymbolError(f"index {index} out of alphabet ({len(self.cum)})")
        return self.cum[index]

    def total_freq(self):  # :24-26
        return self.total

    def find_index(self, decoder):  # :27-45 — evaluated by the GPU decoders themselves
        raise NotImplementedError("FreqTable.find_index runs inside the GPU decode kernel")

    def _rc_table(self):
        """(c, cum, total) as read through c_freq / cum_freq / total_freq (fast path)."""
        return tuple(self.c), tuple(self.cum), self.total


class StaticModel:
    """rc_model: device snapshot of a PModel's (c_freq, cum_freq, total_freq) table."""

    def __init__(self, c_freq, cum_freq=None, total_freq=None, ctx=None):
        self.ctx = ctx or default_context()
        c = np.ascontiguousarray(c_freq, dtype=np.uint32)
        if cum_freq is None:
            cum = np.concatenate([[0], np.cumsum(c, dtype=np.uint64)[:-1]]).astype(np.uint32)
        else:
            cum = np.ascontiguousarray(cum_freq, dtype=np.uint32)
        if total_freq is None:
            total_freq = int(np.sum(c, dtype=np.uint64))
        if len(c) != len(cum):
            raise ValueError("c_freq and cum_freq differ in length")
        self.c = c
        self.cum = cum
        self.total = int(total_freq)
        self.n_symbols = len(c)
        h = ctypes.c_void_p()
        rc = self.ctx._lib.rc_model_create_static(
            self.ctx.handle, self.n_symbols, ctypes.c_void_p(c.ctypes.data),
            ctypes.c_void_p(cum.ctypes.data), ctypes.c_uint32(self.total & 0xFFFFFFFF),
            ctypes.byref(h))
        if rc == N.RC_E_BAD_MODEL:
            raise ValueError("frequency table rejected: need 1..256 symbols, cum[0] == 0, "
                             "cum[i+1] == cum[i] + c[i], total == sum(c) < 2^32")
        N.check(rc, "rc_model_create_static")
        self.handle = h

    @classmethod
    def from_pmodel(cls, pmodel, n_symbols=None, ctx=None):
        """Snapshot any PModel via c_freq/cum_freq/total_freq (pmodel.rs:6-10)."""
        n = pmodel.alphabet_count() if n_symbols is None else int(n_symbols)
        c = [pmodel.c_freq(i) for i in range(n)]
        cum = [pmodel.cum_freq(i) for i in range(n)]
        return cls(c, cum, pmodel.total_freq(), ctx=ctx)

    def max_bits_per_symbol(self):
        nz = self.c[self.c > 0]
        return math.log2(self.total / float(nz.min()))

    def close(self):
        if getattr(self, "handle", None):
            self.ctx._lib.rc_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# config C4's adaptive model parameters (include/range_coder.h, rc_model_create_adaptive)
ADAPTIVE_DEFAULTS = dict(increment=32, limit=57343, period=256)


class AdaptiveModel:
    """rc_model of the build-defined adaptive order-0 model: per chunk,
    c[i] = 1 initially; after the i-th coded symbol s, c[s] += increment and, every period-th
    symbol, all counts are halved (rounding up) if the total exceeds limit.  Each chunk starts
    from the initial counts, on the GPU as in the oracle (orc_encode_adaptive)."""

    def __init__(self, n_symbols=256, increment=32, limit=57343, period=256, ctx=None):
        self.ctx = ctx or default_context()
        self.n_symbols, self.increment = int(n_symbols), int(increment)
        self.limit, self.period = int(limit), int(period)
        h = ctypes.c_void_p()
        rc = self.ctx._lib.rc_model_create_adaptive(self.ctx.handle, self.n_symbols,
                                                    self.increment, self.limit, self.period,
                                                    ctypes.byref(h))
        if rc == N.RC_E_BAD_MODEL:
            raise ValueError("adaptive model rejected: need 1..256 symbols, increment >= 1, "
                             "period a power of two, n + increment*period <= limit <= "
                             "65535 - increment*period")
        N.check(rc, "rc_model_create_adaptive")
        self.handle = h

    def max_bits_per_symbol(self):
        # the rarest symbol has c >= 1 of a total < 2^16
        return 16.0

    close = StaticModel.close
    __del__ = StaticModel.__del__


# ----------------------------------------------------------------------------- batch API
def slot_capacity(n_symbols, bits_per_symbol, slack=1.02):
    """A per-chunk output slot size (16-B multiple) for n symbols at a given worst bit cost."""
    return int(math.ceil((n_symbols * bits_per_symbol / 8.0) * slack + 64)) + 15 & ~15


def encode_batch(model, syms, sym_off, out, out_off, out_len=None, flags=None):
    """rc_encode_batch on torch tensors (async on torch's current stream).

    syms uint8[...]; sym_off int64/uint64[n+1]; out uint8[...]; out_off int64/uint64[n+1].
    Returns (out_len int64[n], flags int32[n]) device tensors."""
    torch = _torch()
    _check_dev(syms, "syms", (torch.uint8,))
    _check_dev(out, "out", (torch.uint8,))
    _check_dev(sym_off, "sym_off", (torch.int64, torch.uint64))
    _check_dev(out_off, "out_off", (torch.int64, torch.uint64))
    n = sym_off.numel() - 1
    if out_off.numel() != n + 1:
        raise ValueError("out_off must have n_chunks + 1 entries")
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int64, device=syms.device)
    if flags is None:
        flags = torch.empty(max(n, 1), dtype=torch.int32, device=syms.device)
    ctx = model.ctx
    ctx.bind_stream()
    N.check(ctx._lib.rc_encode_batch(ctx.handle, model.handle, _ptr(syms), _ptr(sym_off), n,
                                     _ptr(out), _ptr(out_off), _ptr(out_len), _ptr(flags)),
            "rc_encode_batch")
    return out_len[:n], flags[:n]


def decode_batch(model, code, code_off, code_len, syms_out, sym_off, flags=None):
    """rc_decode_batch on torch tensors (async on torch's current stream).  Returns flags."""
    torch = _torch()
    _check_dev(code, "code", (torch.uint8,))
    _check_dev(syms_out, "syms_out", (torch.uint8,))
    for name, t in (("code_off", code_off), ("code_len", code_len), ("sym_off", sym_off)):
        _check_dev(t, name, (torch.int64, torch.uint64))
    n = sym_off.numel() - 1
    if code_off.numel() < n or code_len.numel() < n:
        raise ValueError("code_off/code_len need n_chunks entries")
    if flags is None:
        flags = torch.empty(max(n, 1), dtype=torch.int32, device=code.device)
    ctx = model.ctx
    ctx.bind_stream()
    N.check(ctx._lib.rc_decode_batch(ctx.handle, model.handle, _ptr(code), _ptr(code_off),
                                     _ptr(code_len), _ptr(syms_out), _ptr(sym_off), n,
                                     _ptr(flags)), "rc_decode_batch")
    return flags[:n]


def encode_chunks(model, chunks, raise_on_error=True):
    """Encode a list of symbol sequences (bytes / uint8 arrays), one chunk each.

    Host-resident convenience: uploads, encodes on the GPU, re-encodes chunks that overflowed
    their first slot with their exact length, downloads.  Returns a list of bytes."""
    torch = _torch()
    dev = torch.device("cuda", model.ctx.device)
    arrs = [np.frombuffer(bytes(c), dtype=np.uint8) if not isinstance(c, np.ndarray)
            else np.ascontiguousarray(c, dtype=np.uint8) for c in chunks]
    n = len(arrs)
    if n == 0:
        return []
    lens = np.array([len(a) for a in arrs], dtype=np.int64)
    if int(lens.max()) > N.MAX_CHUNK_SYMBOLS:
        raise ChunkTooLongError(f"chunk of {int(lens.max())} symbols: the batch API takes at "
                                f"most {N.MAX_CHUNK_SYMBOLS} per chunk (use Encoder for longer "
                                f"streams)")
    sym_off = np.zeros(n + 1, dtype=np.int64)
    sym_off[1:] = np.cumsum(lens)
    bits = model.max_bits_per_symbol()
    caps = np.array([slot_capacity(int(L), bits) for L in lens], dtype=np.int64)
    syms_d = torch.from_numpy(np.concatenate(arrs) if sym_off[-1] else np.zeros(1, np.uint8)).to(dev)
    soff_d = torch.from_numpy(sym_off).to(dev)
    for attempt in range(2):
        out_off = np.zeros(n + 1, dtype=np.int64)
        out_off[1:] = np.cumsum(caps)
        out_d = torch.empty(int(out_off[-1]), dtype=torch.uint8, device=dev)
        ool_d = torch.from_numpy(out_off).to(dev)
        out_len, flags = encode_batch(model, syms_d, soff_d, out_d, ool_d)
        fl = flags.cpu().numpy()
        ol = out_len.cpu().numpy()
        if attempt == 0 and np.any(fl == N.F_CAPACITY):
            caps = np.where(fl == N.F_CAPACITY, (ol + 15) // 16 * 16, caps)
            continue
        break
    host = out_d.cpu().numpy()
    res = []
    for k in range(n):
        if fl[k] and raise_on_error:
            _raise_for_flag(int(fl[k]), f"chunk {k}")
        res.append(bytes(host[out_off[k]: out_off[k] + min(ol[k], caps[k])]))
    return res


def decode_chunks(model, codes, counts, raise_on_error=True):
    """Decode a list of code streams; counts[k] symbols each (the count is out-of-band,
    as in the reference: sample_impl.rs:113-120).  Returns a list of uint8 numpy arrays."""
    torch = _torch()
    dev = torch.device("cuda", model.ctx.device)
    n = len(codes)
    if n == 0:
        return []
    codes = [bytes(c) for c in codes]
    clen = np.array([len(c) for c in codes], dtype=np.int64)
    coff = np.zeros(n, dtype=np.int64)
    coff[1:] = np.cumsum(clen)[:-1]
    counts = np.asarray(counts, dtype=np.int64)
    if int(counts.max()) > N.MAX_CHUNK_SYMBOLS:
        raise ChunkTooLongError(f"chunk of {int(counts.max())} symbols: the batch API takes at "
                                f"most {N.MAX_CHUNK_SYMBOLS} per chunk (use Decoder for longer "
                                f"streams)")
    sym_off = np.zeros(n + 1, dtype=np.int64)
    sym_off[1:] = np.cumsum(counts)
    blob = np.frombuffer(b"".join(codes) + b"\0" * 16, dtype=np.uint8)
    code_d = torch.from_numpy(blob.copy()).to(dev)
    syms_d = torch.empty(max(int(sym_off[-1]), 1), dtype=torch.uint8, device=dev)
    flags = decode_batch(model, code_d, torch.from_numpy(coff).to(dev),
                         torch.from_numpy(clen).to(dev), syms_d, torch.from_numpy(sym_off).to(dev))
    fl = flags.cpu().numpy()
    host = syms_d.cpu().numpy()
    res = []
    for k in range(n):
        if fl[k] and raise_on_error:
            _raise_for_flag(int(fl[k]), f"chunk {k}")
        res.append(host[sym_off[k]: sym_off[k + 1]].copy())
    return res


# ----------------------------------------------------------------------------- stream API


class RangeCoder:
    """RangeCoder (src/range_coder.rs:7-146): the public accessors of one coder state.

    A snapshot: a stream's state lives with its GPU call between calls (rc_stream_state), so
    Encoder.range_coder and Decoder.range_coder() return a copy.  param_update / left_shift are
    pub(crate) in the reference and run only inside the kernels."""

    TOP8 = 1 << (64 - 8)  # range_coder.rs:23
    TOP16 = 1 << (64 - 16)  # range_coder.rs:24

    def __init__(self, lower_bound=0, range_=M64):  # Default (:13-20)
        self._low, self._range = int(lower_bound), int(range_)

    @classmethod
    def new(cls):  # :26-28
        return cls()

    def lower_bound(self):  # :30-32
        return self._low

    def range(self):  # :33-35
        return self._range

    def range_par_total(self, total_freq):  # :38-40
        if int(total_freq) == 0:
            raise BadModelError("range_par_total: attempt to divide by zero")
        return self._range // int(total_freq)

    def upper_bound(self):  # :138-146
        s = self._low + self._range
        if s > M64:
            raise RangeCoderError(f"UpperBoundOverflow {{ lower_bound: {self._low}, "
                                  f"range: {self._range} }}")
        return s

    def __eq__(self, other):
        return (isinstance(other, RangeCoder) and
                (self._low, self._range) == (other._low, other._range))

    def __repr__(self):
        return f"RangeCoder(lower_bound={self._low:#x}, range={self._range:#x})"


class ByteCount:
    """The value Encoder.encode returns: the number of bytes that symbol settled
    (encoder.rs:34-36).  Symbols are staged and coded on the GPU in batches, so the count is
    known once the symbol is flushed: int(), comparisons and arithmetic flush on demand (one
    launch for everything staged); code that ignores the value, as sample_impl.rs:96 does,
    never waits for it."""

    __slots__ = ("_enc", "_i")

    def __init__(self, enc, i):
        self._enc, self._i = enc, i

    def __int__(self):
        return self._enc._count(self._i)

    __index__ = __int__

    def __eq__(self, other):
        return int(self) == other

    def __ne__(self, other):
        return int(self) != other

    def __lt__(self, other):
        return int(self) < other

    def __le__(self, other):
        return int(self) <= other

    def __gt__(self, other):
        return int(self) > other

    def __ge__(self, other):
        return int(self) >= other

    def __hash__(self):
        return hash(int(self))

    def __bool__(self):
        return int(self) != 0

    def __float__(self):
        return float(int(self))

    def __add__(self, other):
        return int(self) + other

    __radd__ = __add__

    def __sub__(self, other):
        return int(self) - other

    def __rsub__(self, other):
        return other - int(self)

    def __mul__(self, other):
        return int(self) * other

    __rmul__ = __mul__

    def __floordiv__(self, other):
        return int(self) // other

    def __repr__(self):
        return repr(int(self))


def _u32(v, what):
    v = int(v)
    if not 0 <= v <= 0xFFFFFFFF:
        raise RangeCoderError(f"{what} = {v} is not a u32")
    return v


def _canonical_find_index(pmodel):
    """True when decoding may use FreqTable::find_index's binary search (sample_impl.rs:27-45):
    the model does not override find_index (pmodel.rs:12), or says its override has those
    semantics (canonical_find_index = True in the class that defines the override)."""
    t = type(pmodel)
    # (cached per class and per the find_index / canonical_find_index the class resolves to
    # now: the MRO scan is ~1 us of every decode call, and a class patched after its first
    # decode gets a new key)
    key = (t, getattr(t, "find_index", None), getattr(t, "canonical_find_index", None))
    hit = _CANONICAL.get(key)
    if hit is None:
        owner = next((k for k in t.__mro__ if "find_index" in vars(k)), None)
        hit = (owner is None or owner is PModel or owner is FreqTable or
               bool(vars(owner).get("canonical_find_index", False)))
        if len(_CANONICAL) > 4096:
            _CANONICAL.clear()
        _CANONICAL[key] = hit
    return hit


_CANONICAL = {}  # (class, find_index, flag) -> whether find_index keeps FreqTable's semantics


def _find_index_rfreq(st, total):
    """rfreq of FreqTable::find_index (sample_impl.rs:29): (data - lower_bound) / range_par_total.
    Only for error reports (the decode itself ran on the GPU)."""
    return ((st.data - st.lower_bound) & M64) // (st.range // total)


def _decode_error(st, sig, flags, where):
    """Raise the reference's error for a decode that stopped at state st under table sig."""
    if flags & N.F_BAD_MODEL:
        c, cum, total = sig
        if total == 0 or not c:
            raise BadModelError(f"{where}: range_par_total: attempt to divide by zero")
        rf = _find_index_rfreq(st, total)
        left, right = 0, len(c) - 1  # the binary search of sample_impl.rs:31-44
        while left < right:
            mid = (left + right) // 2
            if cum[mid + 1] <= rf:
                left = mid + 1
            else:
                right = mid
        _raise_bad_model(st.lower_bound, st.range, c[left], cum[left], total, where)
    _raise_for_flag(flags, where)


_U32_PACK = {}  # alphabet size -> struct.Struct of that many little-endian u32


def _table_of(pmodel):
    """(c, cum, total) of a PModel, read through c_freq / cum_freq / total_freq over its
    alphabet, as the reference's decode reads them (decoder.rs:38-50, sample_impl.rs:27-45)."""
    fast = getattr(pmodel, "_rc_table", None)
    if fast is not None:
        return fast()
    n = pmodel.alphabet_count()
    return (tuple(int(pmodel.c_freq(i)) for i in range(n)),
            tuple(int(pmodel.cum_freq(i)) for i in range(n)), int(pmodel.total_freq()))


class Encoder:
    """Encoder (src/encoder.rs:7-55) for ONE stream, with the reference's per-call semantics.

    encode(pmodel, index) reads (c_freq(index), cum_freq(index), total_freq()) at that call, as
    encoder.rs:24-31 does, so a model the caller changes between calls (an adaptive PModel) is
    coded exactly as the reference codes it.  The triples are staged and coded on the GPU by the
    resumable stream kernel (rc_stream_encode_host) when a result is needed: peek_code(),
    range_coder, finish(), the int value of encode()'s ByteCount, or every 2^20 symbols.  A
    stream has no length limit.  Errors the reference panics on surface as RangeCoderError
    subclasses at the call that flushes them; the encoder is then unusable, as after a panic."""

    FLUSH_AT = 1 << 20
    SMALL = 64  # flushes of up to this many symbols use reused ctypes buffers

    def __init__(self, ctx=None):
        self._ctx = ctx
        self._bufs = None          # (triples, output, counts) ctypes buffers of the small flushes
        self._state = N.StreamState.fresh()
        self._code = bytearray()
        self._trip = []            # staged (c, cum, total), flat
        self._counts = bytearray()  # encode() return values of the flushed symbols
        self._staged0 = 0          # index of the first staged symbol
        self._finished = False
        self._exc = None           # the error of the failing symbol, raised again after it

    @classmethod
    def new(cls):  # encoder.rs:14-16
        return cls()

    def encode(self, pmodel, index):  # encoder.rs:24-37
        if self._finished:
            raise FinishedError("encode after finish")
        c = _u32(pmodel.c_freq(index), "c_freq")
        cum = _u32(pmodel.cum_freq(index), "cum_freq")
        total = _u32(pmodel.total_freq(), "total_freq")
        if c == 0:  # range_coder.rs:83-85 would never terminate
            raise ZeroFrequencyError(f"encode({index}): c_freq == 0")
        if total == 0:  # range_coder.rs:38-40 divides by zero
            raise BadModelError(f"encode({index}): total_freq == 0")
        self._trip += (c, cum, total)
        i = self._staged0 + len(self._trip) // 3 - 1
        if len(self._trip) >= 3 * self.FLUSH_AT:
            self._flush()
        return ByteCount(self, i)

    def peek_code(self):  # encoder.rs:18-20: the bytes emitted so far
        self._flush()
        return bytes(self._code)

    @property
    def range_coder(self):  # the pub field of encoder.rs:8 (a snapshot)
        self._flush()
        return RangeCoder(self._state.lower_bound, self._state.range)

    def finish(self):  # encoder.rs:40-46
        if self._finished:
            raise FinishedError("finish twice")
        self._flush(finish=True)
        self._finished = True
        return bytes(self._code)

    def _count(self, i):
        if i >= self._staged0:
            self._flush()
        if i >= len(self._counts):
            raise RangeCoderError(f"symbol {i} was not coded (an earlier symbol failed)")
        return self._counts[i]

    def _flush(self, finish=False):
        if self._state.flags:  # the reference panicked at an earlier call
            if self._exc is not None:
                raise self._exc
            _raise_for_flag(self._state.flags, "encode")
        n = len(self._trip) // 3
        if n == 0 and not finish:
            return
        ctx = self._ctx or default_context()
        cap = N.stream_max_bytes(n, finish)
        small = n <= self.SMALL
        if small:  # (numpy arrays and their .ctypes cost ~1 us each per call)
            if self._bufs is None:
                self._bufs = ((ctypes.c_uint32 * (3 * self.SMALL))(),
                              ctypes.create_string_buffer(N.stream_max_bytes(self.SMALL, True)),
                              ctypes.create_string_buffer(self.SMALL))
            tb, out, nb = self._bufs
            tb[: 3 * n] = self._trip
            args = (tb, out, nb)
        else:
            out = np.empty(max(cap, 1), np.uint8)
            nb = np.empty(max(n, 1), np.uint8)
            trip = np.array(self._trip, dtype=np.uint32)  # (held: _np_ptr keeps no reference)
            args = (_np_ptr(trip), _np_ptr(out), _np_ptr(nb))
        out_len = ctypes.c_uint64()
        fl = ctypes.c_uint32()
        n0 = self._state.n
        rc = ctx._lib.rc_stream_encode_host(ctx.handle, ctypes.byref(self._state), args[0], n,
                                            args[1], cap, ctypes.byref(out_len), args[2],
                                            1 if finish else 0, ctypes.byref(fl))
        if rc not in (N.RC_OK, N.RC_E_CHUNK):
            N.check(rc, "rc_stream_encode_host")
        done = self._state.n - n0
        if small:
            self._code += out.raw[: out_len.value]
            self._counts += nb.raw[:done]
        else:
            self._code += out[: out_len.value].tobytes()
            self._counts += nb[:done].tobytes()
        failed = self._trip[3 * done: 3 * done + 3]
        self._staged0 += n
        self._trip = []
        if fl.value:
            where = f"encode (symbol {self._state.n})"
            try:
                if fl.value & N.F_BAD_MODEL and len(failed) == 3:
                    _raise_bad_model(self._state.lower_bound, self._state.range, *failed, where)
                _raise_for_flag(fl.value, where)
            except RangeCoderError as e:
                self._exc = e
                raise


class Decoder:
    """Decoder (src/decoder.rs:6-55) for ONE stream, with the reference's per-call semantics.

    Decoder(code) runs Decoder::new (the first 8 bytes; a shorter code raises as the reference
    panics).  decode(pmodel) reads the model's table at that call (c_freq / cum_freq /
    total_freq over alphabet_count()) and decodes with FreqTable::find_index's binary search
    and param_update (sample_impl.rs:27-45, decoder.rs:38-54), evaluated on the GPU by the
    resumable stream kernel.  Symbols are decoded ahead in blocks that double while the table
    stays the same; when the caller's table changes (an adaptive PModel), the state at that
    symbol is re-derived and decoding continues under the new table, so every symbol is decoded
    with the table the caller held at its call.

    A PModel that overrides find_index (pmodel.rs:12) gets it called, as decoder.rs:40 does:
    once per symbol, with this decoder (range_coder(), data() give the exact state), and the
    index it returns is what param_update uses (one GPU step per symbol, with the table cut to
    that index's (c_freq, cum_freq)).  That path is launch-latency-bound; a subclass whose
    override keeps FreqTable's binary-search semantics can set canonical_find_index = True to
    stay on the decode-ahead path.  n_symbols (optional, out-of-band as in
    sample_impl.rs:113-120) only bounds the decode-ahead."""

    MAX_BLOCK = 1 << 20
    SMALL = 64  # calls of up to this many symbols decode into a reused buffer

    def __init__(self, code, n_symbols=None, ctx=None):
        self._ctx = ctx or default_context()
        self._code = np.frombuffer(bytes(code), dtype=np.uint8)
        self._code_ptr = _np_ptr(self._code)  # (the array lives as long as the decoder)
        self._small = ctypes.create_string_buffer(self.SMALL)  # output of the short calls
        self._fl = ctypes.c_uint32()
        self._limit = None if n_symbols is None else int(n_symbols)
        self._arrays = (None, None)  # table signature -> (c, cum) uint32 arrays
        st = N.StreamState.fresh()
        if len(self._code) < 8:  # Decoder::new panics (decoder.rs:21, :33)
            raise TruncatedStreamError("code shorter than 8 bytes")
        self._run(st, ((1,), (0,), 1), 0)  # Decoder::new: prime the data window
        self._start = st            # state at the first symbol of the current block
        self._end = st              # state after the block (before a failing symbol)
        self._buf = np.zeros(0, np.uint8)
        self._bpos = 0
        self._sig = None
        self._err = 0               # flag of the symbol after the block, if it failed
        self._block = 1
        self._taken = 0             # symbols returned

    @classmethod
    def new(cls, code):  # decoder.rs:14-23
        return cls(code)

    def _run(self, st, sig, n):
        """Decode n symbols from state st (updated) under table sig; returns (symbols, flags)."""
        na = len(sig[0])
        if not 1 <= na <= 256 or len(sig[1]) != na:
            raise RangeCoderError(f"alphabet of {na} symbols (the GPU decoders take 1..256)")
        if self._arrays[0] != sig:  # the table as packed u32 (struct: ~2 us, numpy ~10-28 us)
            pk = _U32_PACK.get(na) or _U32_PACK.setdefault(na, struct.Struct(f"<{na}I"))
            try:
                self._arrays = (sig, (pk.pack(*sig[0]), pk.pack(*sig[1])))
            except struct.error as e:
                raise RangeCoderError(f"table entry outside u32: {e}") from None
        c, cum = self._arrays[1]
        small = n <= self.SMALL
        out = self._small if small else np.empty(n, np.uint8)
        fl = self._fl
        n0 = st.n
        ctx = self._ctx
        rc = ctx._lib.rc_stream_decode_host(ctx.handle, c, cum, na,
                                            _u32(sig[2], "total_freq"), ctypes.byref(st),
                                            self._code_ptr, len(self._code),
                                            out if small else _np_ptr(out), n, ctypes.byref(fl))
        if rc not in (N.RC_OK, N.RC_E_CHUNK):
            N.check(rc, "rc_stream_decode_host")
        got = st.n - n0
        return (out.raw[:got] if small else out[:got]), fl.value

    @staticmethod
    def _copy(st):
        return N.StreamState.from_buffer_copy(st)

    def _here(self):
        """The state at the current symbol (re-derived inside a block; the block then starts
        here, so the next call needs no re-derivation)."""
        if self._bpos == 0:
            return self._start
        if self._bpos == len(self._buf):
            st = self._copy(self._end)
            st.flags = 0
            return st
        st = self._copy(self._start)
        self._run(st, self._sig, self._bpos)
        self._start, self._buf, self._bpos = st, self._buf[self._bpos:], 0
        return st

    def decode(self, pmodel):  # decoder.rs:38-54
        if not _canonical_find_index(pmodel):
            return self._decode_by_find_index(pmodel)
        sig = _table_of(pmodel)
        same = sig == self._sig
        used = self._bpos == len(self._buf)
        if same and not used:
            s = self._buf[self._bpos]
            self._bpos += 1
            self._taken += 1
            return int(s)
        if same and self._err:  # the reference panics / hangs at this symbol
            _decode_error(self._end, sig, self._err, f"decode (symbol {self._taken})")
        self._block = min(2 * self._block, self.MAX_BLOCK) if same and used else 1
        if used and self._bpos:  # (the block used up: its end state, as _here gives it, once)
            st = self._copy(self._end)
            st.flags = 0
        else:
            st = self._copy(self._here())
        n = self._block
        if self._limit is not None:
            n = max(1, min(n, self._limit - self._taken))
        start = self._copy(st)
        syms, fl = self._run(st, sig, n)
        self._start, self._end, self._buf, self._bpos = start, st, syms, 0
        self._sig, self._err = sig, fl
        if len(syms) == 0:
            _decode_error(st, sig, fl, f"decode (symbol {self._taken})")
        self._bpos = 1
        self._taken += 1
        return int(syms[0])

    def _decode_by_find_index(self, pmodel):
        """decoder.rs:38-54 with the caller's find_index: the index it returns at this state,
        then param_update and shift_left_buffer on the GPU (a one-entry table (c, cum) of that
        index, so the kernel's search has nothing to choose)."""
        st = self._copy(self._here())
        self._start, self._end, self._bpos = st, st, 0
        self._buf, self._sig, self._err = np.zeros(0, np.uint8), None, 0
        idx = int(pmodel.find_index(self))  # reads range_coder() / data(): the state st
        where = f"decode (symbol {self._taken})"
        sig = ((_u32(pmodel.c_freq(idx), "c_freq"),), (_u32(pmodel.cum_freq(idx), "cum_freq"),),
               _u32(pmodel.total_freq(), "total_freq"))
        nxt = self._copy(st)
        syms, fl = self._run(nxt, sig, 1)
        if len(syms) == 0:
            if fl & N.F_BAD_MODEL:
                _raise_bad_model(st.lower_bound, st.range, sig[0][0], sig[1][0], sig[2], where)
            _raise_for_flag(fl, where)
        self._start = self._end = nxt
        self._taken += 1
        return idx

    def range_coder(self):  # decoder.rs:24-26 (a snapshot)
        st = self._here()
        return RangeCoder(st.lower_bound, st.range)

    def data(self):  # decoder.rs:27-29
        return int(self._here().data)


def stream_states(n, device=None):
    """n fresh rc_stream_state on the device (RC_STREAM_STATE_INIT), as an int64 tensor of shape
    (n, 6): lower_bound, range, data, pos, n, flags | stage << 32."""
    torch = _torch()
    st = torch.zeros((n, 6), dtype=torch.int64, device=device or "cuda")
    st[:, 1] = -1  # range = u64::MAX
    return st


def stream_encode_batch(ctx, states, triples, sym_off, out, out_off, out_len=None, nbytes=None,
                        finish=False, flags=None):
    """rc_stream_encode on torch tensors (async on torch's current stream): n = states.shape[0]
    streams, triples uint32/int32 (3 per symbol), sym_off int64[n+1] indexing the triples, out
    uint8 with slots out_off int64[n+1].  Returns (out_len, flags)."""
    torch = _torch()
    n = states.shape[0]
    _check_dev(states, "states", (torch.int64,))
    _check_dev(triples, "triples", (torch.int32, torch.uint32))
    _check_dev(out, "out", (torch.uint8,))
    for name, t in (("sym_off", sym_off), ("out_off", out_off)):
        _check_dev(t, name, (torch.int64, torch.uint64))
        if t.numel() != n + 1:
            raise ValueError(f"{name} must have n_streams + 1 entries")
    if nbytes is not None:
        _check_dev(nbytes, "nbytes", (torch.uint8,))
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int64, device=states.device)
    if flags is None:
        flags = torch.empty(max(n, 1), dtype=torch.int32, device=states.device)
    ctx.bind_stream()
    N.check(ctx._lib.rc_stream_encode(ctx.handle, _ptr(states), _ptr(triples), _ptr(sym_off), n,
                                      _ptr(out), _ptr(out_off), _ptr(out_len), _ptr(nbytes),
                                      1 if finish else 0, _ptr(flags)), "rc_stream_encode")
    return out_len[:n], flags[:n]


def stream_decode_batch(ctx, c, cum, total, states, code, code_off, code_len, syms, sym_off,
                        flags=None):
    """rc_stream_decode on torch tensors: one (c, cum, total) table (uint32/int32 device
    tensors) for every stream's next sym_off[k+1] - sym_off[k] symbols.  Returns flags."""
    torch = _torch()
    n = states.shape[0]
    _check_dev(states, "states", (torch.int64,))
    for name, t in (("c", c), ("cum", cum)):
        _check_dev(t, name, (torch.int32, torch.uint32))
    _check_dev(code, "code", (torch.uint8,))
    _check_dev(syms, "syms", (torch.uint8,))
    for name, t in (("code_off", code_off), ("code_len", code_len), ("sym_off", sym_off)):
        _check_dev(t, name, (torch.int64, torch.uint64))
    if flags is None:
        flags = torch.empty(max(n, 1), dtype=torch.int32, device=states.device)
    ctx.bind_stream()
    rc = ctx._lib.rc_stream_decode(ctx.handle, _ptr(c), _ptr(cum), c.numel(),
                                   ctypes.c_uint32(int(total) & 0xFFFFFFFF), _ptr(states),
                                   _ptr(code), _ptr(code_off), _ptr(code_len), _ptr(syms),
                                   _ptr(sym_off), n, _ptr(flags))
    N.check(rc, "rc_stream_decode")
    return flags[:n]


# ----------------------------------------------------------------------------- host streaming
def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def encode_host(model, syms, sym_off, out_off, out=None):
    """rc_encode_host: host-resident numpy arrays through the pipelined H2D / encode / D2H
    stream (rc_stream.hip).  Returns (out uint8[out_off[-1]], out_len uint64[n], flags
    uint32[n]); flags are returned, not raised.  out: optional caller buffer (e.g. a view of
    pinned memory, which skips the per-call page locking)."""
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
    n = len(sym_off) - 1
    if out is None:
        out = np.empty(int(out_off[-1]), np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < int(out_off[-1]):
        raise ValueError("out must be a contiguous uint8 array of out_off[-1] bytes")
    out_len = np.zeros(max(n, 1), np.uint64)
    flags = np.zeros(max(n, 1), np.uint32)
    ctx = model.ctx
    rc = ctx._lib.rc_encode_host(ctx.handle, model.handle, _np_ptr(syms), _np_ptr(sym_off), n,
                                 _np_ptr(out), _np_ptr(out_off), _np_ptr(out_len), _np_ptr(flags))
    if rc not in (N.RC_OK, N.RC_E_CHUNK):
        N.check(rc, "rc_encode_host")
    return out, out_len[:n], flags[:n]


def decode_host(model, code, code_off, code_len, sym_off, out=None):
    """rc_decode_host: the pipelined host path of decode_batch.  Returns (syms, flags).
    out: optional caller buffer for the symbols."""
    code = np.ascontiguousarray(code, dtype=np.uint8)
    code_off = np.ascontiguousarray(code_off, dtype=np.uint64)
    code_len = np.ascontiguousarray(code_len, dtype=np.uint64)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    n = len(sym_off) - 1
    if out is None:
        syms = np.empty(int(sym_off[-1]), np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < int(sym_off[-1]):
        raise ValueError("out must be a contiguous uint8 array of sym_off[-1] bytes")
    else:
        syms = out
    flags = np.zeros(max(n, 1), np.uint32)
    ctx = model.ctx
    rc = ctx._lib.rc_decode_host(ctx.handle, model.handle, _np_ptr(code), _np_ptr(code_off),
                                 _np_ptr(code_len), _np_ptr(syms), _np_ptr(sym_off), n,
                                 _np_ptr(flags))
    if rc not in (N.RC_OK, N.RC_E_CHUNK):
        N.check(rc, "rc_decode_host")
    return syms, flags[:n]


# ----------------------------------------------------------------------------- several devices
def _handles(models):
    ctxs = (ctypes.c_void_p * len(models))(*[m.ctx.handle.value for m in models])
    hs = (ctypes.c_void_p * len(models))(*[m.handle.value for m in models])
    return ctxs, hs


def encode_host_multi(models, syms, sym_off, out_off, out=None):
    """rc_encode_host_multi: encode_host over several devices at once.  models: one model per
    device (context), e.g. [StaticModel(c, cum, total, ctx=Context(d)) for d in devices]; the
    chunks are split into contiguous ranges of about equal bytes, one per model.  Returns
    (out, out_len, flags) like encode_host."""
    if not models:
        raise ValueError("need at least one model")
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
    n = len(sym_off) - 1
    if out is None:
        out = np.empty(int(out_off[-1]), np.uint8)
    out_len = np.zeros(max(n, 1), np.uint64)
    flags = np.zeros(max(n, 1), np.uint32)
    ctxs, hs = _handles(models)
    rc = models[0].ctx._lib.rc_encode_host_multi(ctxs, hs, len(models), _np_ptr(syms),
                                                 _np_ptr(sym_off), n, _np_ptr(out),
                                                 _np_ptr(out_off), _np_ptr(out_len),
                                                 _np_ptr(flags))
    if rc not in (N.RC_OK, N.RC_E_CHUNK):
        N.check(rc, "rc_encode_host_multi")
    return out, out_len[:n], flags[:n]


def decode_host_multi(models, code, code_off, code_len, sym_off, out=None):
    """rc_decode_host_multi: decode_host over several devices at once.  Returns (syms, flags)."""
    if not models:
        raise ValueError("need at least one model")
    code = np.ascontiguousarray(code, dtype=np.uint8)
    code_off = np.ascontiguousarray(code_off, dtype=np.uint64)
    code_len = np.ascontiguousarray(code_len, dtype=np.uint64)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    n = len(sym_off) - 1
    syms = np.empty(int(sym_off[-1]), np.uint8) if out is None else out
    flags = np.zeros(max(n, 1), np.uint32)
    ctxs, hs = _handles(models)
    rc = models[0].ctx._lib.rc_decode_host_multi(ctxs, hs, len(models), _np_ptr(code),
                                                 _np_ptr(code_off), _np_ptr(code_len),
                                                 _np_ptr(syms), _np_ptr(sym_off), n,
                                                 _np_ptr(flags))
    if rc not in (N.RC_OK, N.RC_E_CHUNK):
        N.check(rc, "rc_decode_host_multi")
    return syms, flags[:n]
