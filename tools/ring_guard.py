"""Scratch RC_RING_GUARD builds of librc_amd.so (part 3).

RC_RING_GUARD makes k_decode_static flag a chunk (RC_F_RING_GUARD = 0x100, scratch builds only)
when a symbol's no_carry_expansion bytes or a range_reduction_expansion byte lie past the bytes
its code ring has staged (rc_decode.inc dec_apply / dec_rare): the read would have taken stale
ring bytes from 64 B earlier.

    python tools/ring_guard.py build      # CPU: variants/librc_guard.so, librc_guard_wide1.so
    python tools/ring_guard.py probe      # GPU: the guard fires where the ring does run short

* variants/librc_guard.so: the shipped ring needs plus the guard.  Run the GPU parity tests with
  RC_LIB_PATH pointing at it: any guard hit makes a chunk's flags non-zero, which those tests
  assert against the oracle's (zero) flags.
* variants/librc_guard_wide1.so: the guard plus a ring need cut to 1 byte for wide models
  (DEC_NEED_WIDE=1, so the decoder may read past its ring).  `probe` decodes wide streams that
  settle 3 bytes per symbol with it and reports how many chunks the guard flagged, and that
  every chunk decoded wrong was flagged (the guard sees the under-runs that happen).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GUARD = os.path.join(ROOT, "variants", "librc_guard.so")
WIDE1 = os.path.join(ROOT, "variants", "librc_guard_wide1.so")
F_RING_GUARD = 0x100


def build():
    import __graft_entry__ as g
    g.build_variant(GUARD, ["-DRC_RING_GUARD"])
    g.build_variant(WIDE1, ["-DRC_RING_GUARD", "-DDEC_NEED_WIDE=1u"])


def probe():
    import numpy as np
    os.environ["RC_LIB_PATH"] = WIDE1
    import torch
    import range_coder_rust_amd as rc
    from oracle import cpu
    from gpu_helpers import run_decode

    rc.default_context(0)
    rng = np.random.default_rng(4)
    out = {}
    for total in (1 << 24, 1 << 20):
        c = np.ones(256, np.uint32)
        c[0] = total - 255
        cum = np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32)
        m = rc.StaticModel(c, cum, total)
        lens = [int(x) for x in rng.integers(200, 3000, 512)]
        chunks = [rng.integers(1, 256, L).astype(np.uint8) for L in lens]
        codes = [cpu.encode(c, cum, total, ch)[1] for ch in chunks]
        dec, fd = run_decode(m, codes, lens, misalign=True, seed=total)
        wrong = [k for k, ch in enumerate(chunks) if not (dec[k] == ch).all()]
        flagged = [k for k in range(len(chunks)) if fd[k] & F_RING_GUARD]
        out[str(total)] = dict(chunks=len(chunks), guard_flagged=len(flagged),
                               decoded_wrong=len(wrong),
                               wrong_unflagged=len(set(wrong) - set(flagged)))
        torch.cuda.synchronize()
    print(json.dumps(out))
    for v in out.values():
        assert v["guard_flagged"] > 0 and v["wrong_unflagged"] == 0, out


if __name__ == "__main__":
    {"build": build, "probe": probe}[sys.argv[1]]()
