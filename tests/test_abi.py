"""CPU checks of the drop-in boundary: librc_amd.so loads, exports every function
include/range_coder.h declares, and behaves per the header without a GPU (no compute calls).
Host-side logic of the Python mirror (range_coder_rust_amd.api) is checked here too."""
import ctypes
import math
import os
import re
import subprocess

import pytest

from range_coder_rust_amd import _native as N
from range_coder_rust_amd import api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "range_coder.h")


def header_text():
    with open(HEADER) as f:
        return f.read()


def declared_functions():
    return sorted(set(re.findall(r"^\s*(?:rc_status|const char\s*\*)\s*(rc_\w+)\s*\(",
                                 header_text(), re.M)))


def test_header_declares_what_the_binding_binds():
    assert declared_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = N.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rc_\w+)", out))
    assert set(declared_functions()) <= exported
    # the ABI is C: no mangled rc_ entry points leak out
    assert not re.search(r"\bT _Z\w*rc_(encode|decode)_batch", out)


def test_header_constants_match_binding():
    h = header_text()
    consts = dict((k, int(v, 0)) for k, v in re.findall(r"#define (RC_\w+)\s+\(?(-?\w+?)u?\)?\s", h)
                  if re.fullmatch(r"-?(0x[0-9a-fA-F]+|\d+)", v))
    assert consts["RC_OK"] == N.RC_OK
    assert consts["RC_E_ARG"] == N.RC_E_ARG
    assert consts["RC_E_BAD_MODEL"] == N.RC_E_BAD_MODEL
    assert consts["RC_E_DEVICE"] == N.RC_E_DEVICE
    assert consts["RC_E_NO_DEVICE"] == N.RC_E_NO_DEVICE
    assert consts["RC_E_CHUNK"] == N.RC_E_CHUNK
    for f in ("ZERO_FREQ", "BAD_SYMBOL", "CAPACITY", "TRUNCATED", "CORRUPT"):
        assert consts["RC_F_" + f] == getattr(N, "F_" + f)


def test_status_strings():
    lib = N.load()
    seen = set()
    for s in (N.RC_OK, N.RC_E_ARG, N.RC_E_BAD_MODEL, N.RC_E_DEVICE, N.RC_E_NO_DEVICE,
              N.RC_E_CHUNK):
        t = lib.rc_status_string(s)
        assert t and t != b"unknown status"
        seen.add(t)
    assert len(seen) == 6
    assert lib.rc_status_string(12345) == b"unknown status"


needs_no_gpu = pytest.mark.skipif(
    os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "x") != "",
    reason="checks the no-device behaviour")


@needs_no_gpu
def test_no_device_is_reported_not_faked():
    """No GPU: context creation fails loudly (no CPU fallback behind the ABI)."""
    lib = N.load()
    h = ctypes.c_void_p()
    assert lib.rc_ctx_create(0, ctypes.byref(h)) == N.RC_E_NO_DEVICE
    assert h.value is None
    buf = ctypes.create_string_buffer(128)
    assert lib.rc_device_info(0, buf, 128) == N.RC_E_NO_DEVICE
    with pytest.raises(N.RCError):
        api.Context(0)


def test_null_arguments_rejected():
    lib = N.load()
    h = ctypes.c_void_p()
    assert lib.rc_ctx_create(0, None) == N.RC_E_ARG
    assert lib.rc_ctx_destroy(None) == N.RC_E_ARG
    assert lib.rc_model_create_static(None, 1, None, None, 1, ctypes.byref(h)) == N.RC_E_ARG
    assert lib.rc_model_destroy(None) == N.RC_E_ARG
    assert lib.rc_encode_batch(None, None, None, None, 0, None, None, None, None) == N.RC_E_ARG
    assert lib.rc_decode_batch(None, None, None, None, None, None, None, 0, None) == N.RC_E_ARG
    assert lib.rc_ctx_set_stream(None, None) == N.RC_E_ARG
    assert lib.rc_synth_fill(None, 0, None, None, 1, 1) == N.RC_E_ARG


# ---- host logic of the Python mirror (no device) ----

def test_freq_table_mirrors_sample_impl():
    """FreqTable::{new, add_alphabet_freq, calc_cum} (sample_impl.rs:49-69) on the sample data."""
    data = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]
    t = api.FreqTable(10)
    for i in data:
        t.add_alphabet_freq(i)
    t.calc_cum()
    assert [t.c_freq(i) for i in range(10)] == [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
    assert [t.cum_freq(i) for i in range(10)] == [0, 1, 6, 8, 8, 10, 12, 13, 14, 15]
    assert t.total_freq() == 16
    assert t.alphabet_count() == 10
    # PModel::ideal_code_length default (pmodel.rs:14-40): log2(total / c)
    assert t.ideal_code_length(1) == pytest.approx(math.log2(16 / 5))
    with pytest.raises(api.BadSymbolError):
        t.c_freq(10)  # Vec::get(..).unwrap() panics (sample_impl.rs:19)


def test_slot_capacity_bounds_worst_case():
    for n in (0, 1, 17, 65536):
        cap = api.slot_capacity(n, 8)
        assert cap % 16 == 0 and cap >= 8 + n  # every symbol at most 8 bits plus finish
    assert api.slot_capacity(65536, 8, 1.02) == 66912


def test_flag_names():
    assert api.flag_names(0) == []
    names = api.flag_names(N.F_CAPACITY | N.F_TRUNCATED)
    assert len(names) == 2


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    """The product path has no fallback: a missing librc_amd.so is an error."""
    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(N.NativeLibraryMissing):
        N.load()


def test_product_package_does_not_import_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/."""
    pkg = os.path.join(ROOT, "range_coder_rust_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".cpp", ".h", ".hpp")):
                with open(os.path.join(dirpath, fn)) as f:
                    src = f.read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", src, re.M), fn
                assert "rc_oracle" not in src, fn
    for fn in ("range_coder.h", "range_coder.hpp"):
        with open(os.path.join(ROOT, "include", fn)) as f:
            assert "oracle" not in f.read().lower()
