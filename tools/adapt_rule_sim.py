"""Code length of adaptive order-0 rules that fit a u8-leaf tree.

The C4 decoder's 255-node u16 tree takes 510 B per lane, so LDS holds 5 waves per CU.  A tree
of <= 320 B per lane (8 waves per CU) keeps the 192 nodes that span one or two symbols in u8 and
the 63 others in u16 (318 B).  That needs every pair of adjacent counts to sum below 256, i.e.
counts <= 127: a different rule than C4's (counts up to 2^16).  This computes, on the bench's
C4 data (Zipf(1.2), 16 KiB chunks, the synth stream of bench.py's adaptive leg), the ideal code
length sum(-log2(c[s] / total)) of C4 and of capped rules (the range coder's own overhead,
~0.002 bits per symbol, is the same for all), so the bytes-per-symbol criterion (<= +1% over
C4) can be checked before any kernel is written.

    python tools/adapt_rule_sim.py [n_chunks]  -> one JSON line
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from range_coder_rust_amd import synth  # noqa: E402

SEED_ADAPTIVE = 0x5EED0001  # bench.py SEED; the adaptive leg's stream (shard.synth_seed(SEED, 0))


def c4_bits(chunk, n=256, inc=32, limit=57343, period=256):
    c = [1] * n
    total = n
    bits = 0.0
    for i, s in enumerate(chunk):
        bits -= math.log2(c[s] / total)
        c[s] += inc
        total += inc
        if (i + 1) % period == 0 and total > limit:
            c = [(x + 1) >> 1 for x in c]
            total = sum(c)
    return bits


def capped_bits(chunk, n=256, inc=1, cap=127):
    """c[s] += inc; when c[s] would pass cap, every count is halved first ((c + 1) >> 1)."""
    c = [1] * n
    total = n
    bits = 0.0
    for s in chunk:
        bits -= math.log2(c[s] / total)
        if c[s] + inc > cap:
            c = [(x + 1) >> 1 for x in c]
            total = sum(c)
        c[s] += inc
        total += inc
    return bits


def main():
    n_chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    L = 16384
    c, _, _ = synth.zipf_table()
    inv = synth.inverse_cdf(c)
    from range_coder_rust_amd import shard
    seed = shard.synth_seed(SEED_ADAPTIVE, 0)
    chunks = [synth.host_chunk(seed, inv, k, L).tolist() for k in range(n_chunks)]
    N = n_chunks * L
    res = {"sample": f"{n_chunks} x 16 KiB chunks of the Zipf(1.2) stream", "bits_per_symbol": {}}
    base = sum(c4_bits(ch) for ch in chunks) / N
    res["bits_per_symbol"]["C4 (inc 32, limit 57343, period 256; u16 tree, 510 B/lane)"] = round(base, 5)
    for inc in (1, 2, 4, 8, 16):
        b = sum(capped_bits(ch, inc=inc) for ch in chunks) / N
        res["bits_per_symbol"][f"cap 127, inc {inc} (u8 span-1/2 nodes, 318 B/lane)"] = round(b, 5)
        res.setdefault("vs_C4", {})[f"inc {inc}"] = round(b / base - 1, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
