"""Synthetic workloads of BASELINE.json's configs.

 * uniform-256 static model: c[i] = 1, total = 256                     (configs[1])
 * Zipf(s=1.2) 256-symbol static model quantised to total 2^16          (configs[2], [4]):
   c[i] = round(65536 * w_i / sum(w)), w_i = (i+1)^-1.2, clamped >= 1, the rounding remainder
   folded into c[0]  (c[0] == 16623, min c == 21).
Symbols are generated on the GPU (rc_synth_fill) from a 2^16-entry inverse CDF with a
counter-based splitmix64 stream, so any chunk can be regenerated bit-identically on the host
(``host_chunk``) without storing the 64 GiB inputs anywhere else.
"""
import ctypes

import numpy as np

from . import _native as N

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def uniform_table(n=256):
    c = np.ones(n, dtype=np.uint32)
    return c, np.arange(n, dtype=np.uint32), n


def zipf_table(s=1.2, n=256, total=1 << 16):
    w = (np.arange(1, n + 1, dtype=np.float64)) ** (-s)
    c = np.maximum(np.rint(total * w / w.sum()), 1).astype(np.int64)
    c[0] += total - int(c.sum())
    c = c.astype(np.uint32)
    cum = np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32)
    return c, cum, total


def inverse_cdf(c):
    """65536-entry inverse CDF of the distribution c (any total), quantised to 2^16."""
    c = np.asarray(c, dtype=np.float64)
    q = np.floor(np.cumsum(c) / c.sum() * 65536.0 + 1e-9).astype(np.int64)
    q[-1] = 65536
    inv = np.zeros(65536, dtype=np.uint8)
    lo = 0
    for s, hi in enumerate(q):
        inv[lo:hi] = s
        lo = max(lo, hi)
    return inv


def _mix64(z):
    z = z.astype(np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def host_chunk(seed, inv, chunk, chunk_len):
    """Numpy restatement of k_synth for one chunk (regenerate any chunk on the host)."""
    nw = (chunk_len + 3) // 4
    j = np.arange(nw, dtype=np.uint64)
    with np.errstate(over="ignore"):
        ctr = (np.uint64(chunk) << np.uint64(32)) + j + np.uint64(1)
        z = np.uint64(seed) + np.uint64(GOLDEN) * ctr
        w = _mix64(z)
    lanes = np.stack([(w >> np.uint64(16 * q)) & np.uint64(0xFFFF) for q in range(4)], axis=1)
    return inv[lanes.reshape(-1).astype(np.int64)][:chunk_len].copy()


def fill(ctx, seed, inv, syms_dev, chunk_len, n_chunks):
    """rc_synth_fill into a torch uint8 device tensor (chunk k at k * chunk_len)."""
    inv = np.ascontiguousarray(inv, dtype=np.uint8)
    assert inv.size == 65536
    assert syms_dev.numel() >= chunk_len * n_chunks
    ctx.bind_stream()
    N.check(ctx._lib.rc_synth_fill(ctx.handle, ctypes.c_uint64(seed & M64),
                                   ctypes.c_void_p(inv.ctypes.data),
                                   ctypes.c_void_p(syms_dev.data_ptr()),
                                   ctypes.c_uint64(chunk_len), n_chunks), "rc_synth_fill")
