"""Host-side API of the MI355X range coder, mirroring the reference crate's public surface.

Reference surface (diegodox/range_coder_rust, src/lib.rs:1-13) and what replaces it here:

  trait PModel (src/pmodel.rs:4-41)        -> class PModel (same method names/meaning)
  FreqTable example model (sample_impl.rs)  -> class FreqTable
  Encoder::{new, encode, finish}            -> class Encoder: encode() stages symbols, finish()
    (src/encoder.rs:14-46)                     encodes the stream on the GPU (one lane)
  Decoder::{new, decode}                    -> class Decoder(code, n_symbols): the first
    (src/decoder.rs:14-54)                     decode() decodes the stream on the GPU
  error::RangeCoderError (src/error.rs)     -> RangeCoderError and subclasses (raised where
                                               the reference panics or never terminates)

The hot path proper is the batch API (encode_batch / decode_batch / encode_chunks /
decode_chunks): many independent chunks per launch, one chunk per GPU lane, through the C ABI
of librc_amd.so (include/range_coder.h).  Tensors are torch CUDA(HIP) tensors; PyTorch is
used only for device memory and streams.  There is no CPU fallback.
"""
import ctypes
import math

import numpy as np

from . import _native as N

__all__ = [
    "Context", "StaticModel", "PModel", "FreqTable", "Encoder", "Decoder", "RangeCoderError",
    "ZeroFrequencyError", "BadSymbolError", "TruncatedStreamError", "CorruptStreamError",
    "CapacityError", "ChunkTooLongError", "encode_batch", "decode_batch", "encode_chunks", "decode_chunks",
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


class ChunkTooLongError(RangeCoderError):
    """A batch chunk of more than RC_MAX_CHUNK_SYMBOLS (2^25) symbols (32-bit in-chunk stream
    positions; the stream API -- Encoder / Decoder -- has no such limit)."""


_FLAG_ERRORS = [
    (N.F_ZERO_FREQ, ZeroFrequencyError), (N.F_BAD_SYMBOL, BadSymbolError),
    (N.F_CAPACITY, CapacityError), (N.F_TRUNCATED, TruncatedStreamError),
    (N.F_CORRUPT, CorruptStreamError), (N.F_TOO_LONG, ChunkTooLongError),
]


def flag_names(f):
    names = {N.F_ZERO_FREQ: "ZERO_FREQ", N.F_BAD_SYMBOL: "BAD_SYMBOL", N.F_CAPACITY: "CAPACITY",
             N.F_TRUNCATED: "TRUNCATED", N.F_CORRUPT: "CORRUPT", N.F_TOO_LONG: "TOO_LONG"}
    return [v for k, v in names.items() if f & k]


def _raise_for_flag(f, where):
    for bit, exc in _FLAG_ERRORS:
        if f & bit:
            raise exc(f"{where}: {'|'.join(flag_names(f))}")


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

    def find_index(self, decoder):  # pmodel.rs:12 — not called by the GPU path (see StaticModel)
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

    def find_index(self, decoder):  # :27-45 — the GPU decoder implements this inverse itself
        raise NotImplementedError("FreqTable.find_index runs inside the GPU decode kernel")


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
class Encoder:
    """Encoder (src/encoder.rs:7-55) for ONE stream.

    encode(pmodel, index) stages the symbol (it cannot return the per-symbol byte count the
    reference returns, encoder.rs:36, because nothing is coded until finish()); finish()
    encodes the whole stream on the GPU and returns its bytes (== the reference's
    VecDeque<u8>).  All symbols of one stream must use the same static model."""

    def __init__(self):
        self._syms = []
        self._model = None

    @classmethod
    def new(cls):
        return cls()

    def encode(self, pmodel, index):
        if self._model is None:
            self._model = pmodel
        elif pmodel is not self._model:
            raise RangeCoderError("one static model per staged stream")
        self._syms.append(int(index))

    def peek_code(self):
        raise RangeCoderError("peek_code: the stream is coded in finish() on the GPU")

    def finish(self):
        if self._model is None:
            # no symbols: the reference emits the 8 bytes of lower_bound == 0
            return bytes(8)
        m = _snapshot(self._model)
        if any(s < 0 or s >= m.n_symbols for s in self._syms):
            raise BadSymbolError("symbol index outside the alphabet")
        return encode_chunks(m, [np.array(self._syms, dtype=np.uint8)])[0]


class Decoder:
    """Decoder (src/decoder.rs:6-55) for ONE stream; n_symbols is the out-of-band count the
    reference's caller also supplies (sample_impl.rs:113-120)."""

    def __init__(self, code, n_symbols=None):
        self._code = bytes(code)
        if len(self._code) < 8:  # Decoder::new panics (decoder.rs:21,33)
            raise TruncatedStreamError("code shorter than 8 bytes")
        self._n = n_symbols
        self._out = None
        self._pos = 0

    def decode(self, pmodel):
        if self._out is None:
            if self._n is None:
                raise RangeCoderError("Decoder(code, n_symbols): the symbol count is out-of-band")
            m = _snapshot(pmodel)
            self._out = decode_chunks(m, [self._code], [self._n])[0]
        if self._pos >= len(self._out):
            raise RangeCoderError("more decode() calls than n_symbols")
        s = int(self._out[self._pos])
        self._pos += 1
        return s


_snap_cache = {}


def _snapshot(pmodel):
    if isinstance(pmodel, StaticModel):
        return pmodel
    key = id(pmodel)
    n = pmodel.alphabet_count()
    sig = (tuple(pmodel.c_freq(i) for i in range(n)), tuple(pmodel.cum_freq(i) for i in range(n)),
           pmodel.total_freq())
    hit = _snap_cache.get(key)
    if hit is not None and hit[0] == sig:
        return hit[1]
    m = StaticModel(sig[0], sig[1], sig[2])
    _snap_cache[key] = (sig, m)
    return m


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
