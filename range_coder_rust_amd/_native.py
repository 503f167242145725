"""ctypes binding of librc_amd.so (the C ABI declared in include/range_coder.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no CPU fallback: if the library is missing this module raises on first use.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RC_LIB_PATH") or os.path.join(_HERE, "librc_amd.so")

RC_OK = 0
RC_E_ARG = -1
RC_E_BAD_MODEL = -2
RC_E_DEVICE = -3
RC_E_NO_DEVICE = -4
RC_E_CHUNK = -5

F_ZERO_FREQ = 1
F_BAD_SYMBOL = 2
F_CAPACITY = 4
F_TRUNCATED = 8
F_CORRUPT = 16
F_TOO_LONG = 32
F_BAD_MODEL = 64
F_FINISHED = 128
MAX_CHUNK_SYMBOLS = 1 << 25  # RC_MAX_CHUNK_SYMBOLS

# every symbol include/range_coder.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "rc_ctx_create", "rc_ctx_destroy", "rc_ctx_set_stream", "rc_ctx_reset_stream",
    "rc_ctx_synchronize",
    "rc_status_string", "rc_last_error", "rc_device_info", "rc_model_create_static",
    "rc_model_create_adaptive", "rc_model_destroy", "rc_encode_batch", "rc_decode_batch", "rc_encode_host",
    "rc_decode_host", "rc_synth_fill", "rc_histogram", "rc_quantize_counts", "rc_ideal_bits",
    "rc_container_pack", "rc_container_info_parse", "rc_container_offsets",
    "rc_stream_encode", "rc_stream_decode", "rc_stream_encode_host", "rc_stream_decode_host",
    "rc_encode_host_multi", "rc_decode_host_multi",
)
RC_E_BAD_CONTAINER = -6
RC_E_CAPACITY = -7
CONTAINER_HEADER_BYTES = 64


class ContainerInfo(ctypes.Structure):
    """rc_container_info (include/range_coder.h)."""
    _fields_ = [(n, ctypes.c_uint32) for n in ("version", "kind", "n_symbols", "total_freq",
                                              "increment", "limit", "period", "reserved")] + \
               [(n, ctypes.c_uint64) for n in ("n_chunks", "n_syms", "payload_bytes", "table_off",
                                              "index_off", "payload_off", "container_bytes")]
Q_ALL_SYMBOLS = 1


class StreamState(ctypes.Structure):
    """rc_stream_state (include/range_coder.h): one reference Encoder / Decoder between calls."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("lower_bound", "range", "data", "pos", "n")] + \
               [("flags", ctypes.c_uint32), ("stage", ctypes.c_uint32)]

    @classmethod
    def fresh(cls):  # RC_STREAM_STATE_INIT
        return cls(0, (1 << 64) - 1, 0, 0, 0, 0, 0)


def stream_max_bytes(n, finish):  # RC_STREAM_MAX_BYTES
    return 12 * int(n) + (8 if finish else 0)

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load():
    """Load librc_amd.so (import torch first so the HIP runtime is shared with PyTorch)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:  # share libamdhip64.so.7 with torch when torch is present
        import torch  # noqa: F401
    except Exception:  # pragma: no cover
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.rc_ctx_create.argtypes = [_I, ctypes.POINTER(_P)]
    L.rc_ctx_destroy.argtypes = [_P]
    L.rc_ctx_set_stream.argtypes = [_P, _P]
    L.rc_ctx_reset_stream.argtypes = [_P]
    L.rc_ctx_synchronize.argtypes = [_P]
    L.rc_status_string.argtypes = [_I]
    L.rc_status_string.restype = ctypes.c_char_p
    L.rc_last_error.argtypes = []
    L.rc_last_error.restype = ctypes.c_char_p
    L.rc_device_info.argtypes = [_I, ctypes.c_char_p, ctypes.c_size_t]
    L.rc_model_create_static.argtypes = [_P, _U32, _P, _P, _U32, ctypes.POINTER(_P)]
    L.rc_model_create_adaptive.argtypes = [_P, _U32, _U32, _U32, _U32, ctypes.POINTER(_P)]
    L.rc_model_destroy.argtypes = [_P]
    L.rc_encode_batch.argtypes = [_P, _P, _P, _P, _U32, _P, _P, _P, _P]
    L.rc_decode_batch.argtypes = [_P, _P, _P, _P, _P, _P, _P, _U32, _P]
    L.rc_encode_host.argtypes = [_P, _P, _P, _P, _U32, _P, _P, _P, _P]
    L.rc_decode_host.argtypes = [_P, _P, _P, _P, _P, _P, _P, _U32, _P]
    L.rc_synth_fill.argtypes = [_P, _U64, _P, _P, _U64, _U32]
    L.rc_histogram.argtypes = [_P, _P, _P, _U32, _P, _P]
    L.rc_quantize_counts.argtypes = [_P, _U32, _U64, _U32, _P, _P, _P]
    L.rc_ideal_bits.argtypes = [_P, _P, _U32, _U32, _P, _U32, _P]
    L.rc_container_pack.argtypes = [_P, _P, _P, _P, _P, _P, _U32, _P, _U64, ctypes.POINTER(_U64)]
    L.rc_container_info_parse.argtypes = [_P, _U64, ctypes.POINTER(ContainerInfo)]
    L.rc_container_offsets.argtypes = [_P, _P, ctypes.POINTER(ContainerInfo), _P, _P, _P]
    SP = ctypes.POINTER(StreamState)
    L.rc_stream_encode.argtypes = [_P, _P, _P, _P, _U32, _P, _P, _P, _P, _U32, _P]
    L.rc_stream_decode.argtypes = [_P, _P, _P, _U32, _U32, _P, _P, _P, _P, _P, _P, _U32, _P]
    L.rc_stream_encode_host.argtypes = [_P, SP, _P, _U64, _P, _U64, ctypes.POINTER(_U64), _P,
                                        _U32, ctypes.POINTER(_U32)]
    L.rc_stream_decode_host.argtypes = [_P, _P, _P, _U32, _U32, SP, _P, _U64, _P, _U64,
                                        ctypes.POINTER(_U32)]
    L.rc_encode_host_multi.argtypes = [_P, _P, _U32, _P, _P, _U32, _P, _P, _P, _P]
    L.rc_decode_host_multi.argtypes = [_P, _P, _U32, _P, _P, _P, _P, _P, _U32, _P]
    for name in EXPORTS:
        if name not in ("rc_status_string", "rc_last_error"):
            getattr(L, name).restype = _I
    _lib = L
    return L


def status_string(code):
    return load().rc_status_string(code).decode()


class RCError(RuntimeError):
    def __init__(self, code, what):
        detail = load().rc_last_error().decode() if code == RC_E_DEVICE else ""
        super().__init__(f"{what}: {status_string(code)} ({code}) {detail}".rstrip())
        self.code = code


def check(code, what):
    if code != RC_OK:
        raise RCError(code, what)
    return code
