"""ctypes binding of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker or as the timed CPU baseline.  The product never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64

F_ZERO_FREQ = 1
F_BAD_SYMBOL = 2
F_CAPACITY = 4
F_TRUNCATED = 8
F_CORRUPT = 16
F_BAD_MODEL = 64
F_FINISHED = 128


class Stream(ctypes.Structure):
    """orc_stream (rc_oracle.h) == rc_stream_state (include/range_coder.h)."""
    _fields_ = [(n, _U64) for n in ("lower_bound", "range", "data", "pos", "n")] + \
               [("flags", _U32), ("stage", _U32)]

    @classmethod
    def fresh(cls):
        return cls(0, (1 << 64) - 1, 0, 0, 0, 0, 0)

    def tuple(self):
        return (self.lower_bound, self.range, self.data, self.pos, self.n, self.flags, self.stage)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_encode.argtypes = [_P, _P, _U32, _U32, _P, _U64, _P, _U64, ctypes.POINTER(_U64)]
        L.orc_encode.restype = _U32
        L.orc_decode.argtypes = [_P, _P, _U32, _U32, _P, _U64, _U64, _P]
        L.orc_decode.restype = _U32
        L.orc_encode_batch.argtypes = [_P, _P, _U32, _U32, _P, _P, _U32, _P, _P, _P, _P, ctypes.c_int]
        L.orc_encode_batch.restype = None
        L.orc_decode_batch.argtypes = [_P, _P, _U32, _U32, _P, _P, _P, _P, _P, _U32, _P, ctypes.c_int]
        L.orc_decode_batch.restype = None
        L.orc_encode_adaptive.argtypes = [_U32, _U32, _U32, _U32, _P, _U64, _P, _U64,
                                          ctypes.POINTER(_U64)]
        L.orc_encode_adaptive.restype = _U32
        L.orc_decode_adaptive.argtypes = [_U32, _U32, _U32, _U32, _P, _U64, _U64, _P]
        L.orc_decode_adaptive.restype = _U32
        L.orc_stream_encode.argtypes = [ctypes.POINTER(Stream), _P, _U64, _P, _U64,
                                        ctypes.POINTER(_U64), _P, ctypes.c_int]
        L.orc_stream_encode.restype = _U32
        L.orc_stream_decode.argtypes = [ctypes.POINTER(Stream), _P, _P, _U32, _U32, _P, _U64, _P,
                                        _U64, ctypes.POINTER(_U64)]
        L.orc_stream_decode.restype = _U32
        L.orc_fnv1a64.argtypes = [_P, _U64]
        L.orc_fnv1a64.restype = _U64
        _LIB = L
    return _LIB


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def _u8(a):
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8).copy()
    return np.ascontiguousarray(a, dtype=np.uint8)


def _table(c, cum):
    c = np.ascontiguousarray(c, dtype=np.uint32)
    cum = np.ascontiguousarray(cum, dtype=np.uint32)
    return c, cum


def encode(c, cum, total, syms, cap=None):
    """One stream: returns (flags, bytes) where bytes has length min(len, cap)."""
    c, cum = _table(c, cum)
    s = _u8(syms)
    if cap is None:
        cap = 16 * len(s) + 64
    out = np.zeros(max(cap, 1), np.uint8)
    ol = _U64()
    f = lib().orc_encode(_ptr(c), _ptr(cum), len(c), total, _ptr(s), len(s), _ptr(out), cap,
                         ctypes.byref(ol))
    return int(f), bytes(out[: min(ol.value, cap)]), int(ol.value)


def decode(c, cum, total, code, n):
    c, cum = _table(c, cum)
    code = _u8(code)
    out = np.zeros(max(n, 1), np.uint8)
    f = lib().orc_decode(_ptr(c), _ptr(cum), len(c), total, _ptr(code), len(code), n, _ptr(out))
    return int(f), out[:n]


def encode_batch(c, cum, total, syms, sym_off, out_off, threads=1):
    c, cum = _table(c, cum)
    syms = np.ascontiguousarray(syms, dtype=np.uint8)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
    n = len(sym_off) - 1
    out = np.zeros(int(out_off[-1]) if n else 1, np.uint8)
    out_len = np.zeros(max(n, 1), np.uint64)
    flags = np.zeros(max(n, 1), np.uint32)
    lib().orc_encode_batch(_ptr(c), _ptr(cum), len(c), total, _ptr(syms), _ptr(sym_off), n,
                           _ptr(out), _ptr(out_off), _ptr(out_len), _ptr(flags), threads)
    return out, out_len[:n], flags[:n]


def decode_batch(c, cum, total, code, code_off, code_len, sym_off, threads=1):
    c, cum = _table(c, cum)
    code = np.ascontiguousarray(code, dtype=np.uint8)
    code_off = np.ascontiguousarray(code_off, dtype=np.uint64)
    code_len = np.ascontiguousarray(code_len, dtype=np.uint64)
    sym_off = np.ascontiguousarray(sym_off, dtype=np.uint64)
    n = len(sym_off) - 1
    out = np.zeros(max(int(sym_off[-1]), 1), np.uint8)
    flags = np.zeros(max(n, 1), np.uint32)
    lib().orc_decode_batch(_ptr(c), _ptr(cum), len(c), total, _ptr(code), _ptr(code_off),
                           _ptr(code_len), _ptr(out), _ptr(sym_off), n, _ptr(flags), threads)
    return out[: int(sym_off[-1])], flags[:n]


def encode_adaptive(n_alpha, inc, limit, period, syms, cap=None):
    s = _u8(syms)
    if cap is None:
        cap = 16 * len(s) + 64
    out = np.zeros(max(cap, 1), np.uint8)
    ol = _U64()
    f = lib().orc_encode_adaptive(n_alpha, inc, limit, period, _ptr(s), len(s), _ptr(out), cap,
                                  ctypes.byref(ol))
    return int(f), bytes(out[: min(ol.value, cap)]), int(ol.value)


def decode_adaptive(n_alpha, inc, limit, period, code, n):
    code = _u8(code)
    out = np.zeros(max(n, 1), np.uint8)
    f = lib().orc_decode_adaptive(n_alpha, inc, limit, period, _ptr(code), len(code), n,
                                  _ptr(out))
    return int(f), out[:n]


def fnv1a64(b):
    a = _u8(b)
    return int(lib().orc_fnv1a64(_ptr(a), len(a)))


def stream_encode(st, triples, finish=False, cap=None):
    """orc_stream_encode: st (Stream) advances; returns (flags, new bytes, per-symbol counts)."""
    t = np.ascontiguousarray(triples, dtype=np.uint32).reshape(-1)
    n = t.size // 3
    if cap is None:
        cap = 12 * n + (8 if finish else 0)
    out = np.zeros(max(cap, 1), np.uint8)
    nb = np.zeros(max(n, 1), np.uint8)
    ol = _U64()
    n0 = st.n
    f = lib().orc_stream_encode(ctypes.byref(st), _ptr(t), n, _ptr(out), cap, ctypes.byref(ol),
                                _ptr(nb), 1 if finish else 0)
    return int(f), bytes(out[: ol.value]), nb[: st.n - n0].copy()


def stream_decode(st, c, cum, total, code, n):
    """orc_stream_decode over the whole code: returns (flags, decoded symbols)."""
    c, cum = _table(c, cum)
    code = _u8(code)
    out = np.zeros(max(n, 1), np.uint8)
    done = _U64()
    f = lib().orc_stream_decode(ctypes.byref(st), _ptr(c), _ptr(cum), len(c), total, _ptr(code),
                                len(code), _ptr(out), n, ctypes.byref(done))
    return int(f), out[: done.value].copy()
