"""bench.py's legs on models whose total is NOT a power of two (scratch measurement of the
DIV_MAGIC decoders and encoder): "uniform" becomes a 256-symbol model of total 300 (44 symbols of
frequency 2, the rest 1; LUT 2), "zipf" becomes Zipf(1.2) over total 65521 (LUT 4).
  python3 tools/div_probe.py [bench.py options, e.g. --no-cpu-baseline --no-adaptive ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def table(cfg):
    from range_coder_rust_amd import synth
    if cfg == "uniform":
        c = np.ones(256, dtype=np.uint32)
        c[:44] = 2
        return c, np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32), int(c.sum())
    return synth.zipf_table(total=65521)


if __name__ == "__main__":
    bench.table = table
    sys.exit(bench.main())
