"""tools/isa_check.py: the build-time guard against the gfx950 top-register hazard (DESIGN.md
§6).  The instruction class it refuses, on disassembly text, and the shipped library passing."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check  # noqa: E402

LIB = os.path.join(ROOT, "range_coder_rust_amd", "librc_amd.so")


@pytest.mark.parametrize("text", [
    "v_lshlrev_b64 v[4:5], v95, v[6:7]",          # the measured shifts (amount = top)
    "v_lshrrev_b64 v[4:5], v95, v[6:7]",
    "v_ashrrev_i64 v[4:5], v95, v[6:7]",
    "v_lshl_add_u64 v[4:5], v[6:7], v95, v[8:9]",  # 32-bit shift amount of a 64-bit op
    "v_lshl_add_u64 v[4:5], v[6:7], 0, v95",       # (any single-register source)
    "v_mad_u64_u32 v[4:5], s[0:1], v95, v3, 0",
    "v_cvt_f64_u32_e32 v[4:5], v95",
    "v_mad_i64_i32 v[4:5], s[0:1], v95, v3, v[6:7]",
])
def test_hazard_class_flagged(text):
    assert isa_check.hazard(text, 95)


@pytest.mark.parametrize("text", [
    "v_lshlrev_b64 v[4:5], v94, v[6:7]",          # one register lower
    "v_lshlrev_b32_e32 v4, v95, v6",              # 32-bit ops read it safely
    "v_add_u32_e32 v4, v95, v6",
    "v_lshlrev_b64 v[94:95], 3, v[6:7]",          # the last VGPR as (part of) the destination
    "v_lshl_add_u64 v[4:5], v[94:95], 0, v[8:9]",  # as half of a pair source
    "s_lshl_b64 s[0:1], s[2:3], 4",
])
def test_hazard_class_not_flagged(text):
    assert not isa_check.hazard(text, 95)


@pytest.mark.skipif(not os.path.exists(LIB), reason="librc_amd.so not built")
def test_shipped_library_passes():
    res = isa_check.check_library(LIB)
    assert len(res) >= 30
    assert not {k: v for k, v in res.items() if v[2]}


def test_shipped_coders_use_no_scratch():
    """The static coders keep their state and tiles in registers: build() refuses a library in
    which one uses scratch memory (round 5: an array form of the encoder's tile loop put the
    tiles in scratch and halved its rate)."""
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    sizes = isa_check.scratch_sizes(LIB)
    coders = {k: v for k, v in sizes.items() if "k_encode_static" in k or "k_decode_static" in k}
    assert coders, "no coder kernels found"
    assert not {k: v for k, v in coders.items() if v}, coders
