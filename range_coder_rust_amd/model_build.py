"""Model construction on the GPU — the step before encode.

The reference builds its model by counting (FreqTable::new + add_alphabet_freq per symbol,
examples/sample_impl.rs:49-60) and scanning (calc_cum, :61-69); PModel::ideal_code_length
(src/pmodel.rs:14-40) prices one symbol.  Here:

  histogram(syms, sym_off)        rc_histogram: per-chunk and/or batch symbol counts (HIP)
  quantize_counts(counts, T)      rc_quantize_counts: counts -> (c, cum, total) table
  build_model(syms, sym_off, T)   histogram -> table -> StaticModel, in one call
  ideal_bits(model, chunk_hist)   rc_ideal_bits: per-chunk sum of ideal code lengths (HIP)
"""
import ctypes

import numpy as np

from . import _native as N
from .api import StaticModel, _check_dev, _ptr, _torch, default_context


def quantize_counts(counts, target_total=0, all_symbols=False):
    """rc_quantize_counts (host): counts (len n <= 256) -> (c, cum, total).

    target_total 0 keeps calc_cum's exact table; otherwise counts are scaled to that total
    (each modelled symbol keeps c >= 1).  all_symbols gives absent symbols c >= 1 too."""
    L = N.load()
    cnt = np.ascontiguousarray(counts, dtype=np.uint64)
    n = len(cnt)
    c = np.zeros(max(n, 1), np.uint32)
    cum = np.zeros(max(n, 1), np.uint32)
    total = ctypes.c_uint32()
    rc = L.rc_quantize_counts(ctypes.c_void_p(cnt.ctypes.data), n, int(target_total),
                              N.Q_ALL_SYMBOLS if all_symbols else 0,
                              ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(cum.ctypes.data),
                              ctypes.byref(total))
    if rc == N.RC_E_BAD_MODEL:
        raise ValueError("no frequency table for these counts and target")
    N.check(rc, "rc_quantize_counts")
    return c[:n], cum[:n], int(total.value)


def histogram(syms, sym_off, per_chunk=False, batch=True, ctx=None):
    """rc_histogram on torch tensors (async, torch's current stream).

    Returns (hist, chunk_hist): hist int64[256] (the batch) or None, chunk_hist int32[n, 256]
    (one row per chunk) or None."""
    torch = _torch()
    _check_dev(syms, "syms", (torch.uint8,))
    _check_dev(sym_off, "sym_off", (torch.int64, torch.uint64))
    ctx = ctx or default_context(syms.device.index)
    n = sym_off.numel() - 1
    hist = torch.zeros(256, dtype=torch.int64, device=syms.device) if batch else None
    chunk_hist = (torch.empty((max(n, 1), 256), dtype=torch.int32, device=syms.device)
                  if per_chunk else None)
    ctx.bind_stream()
    N.check(ctx._lib.rc_histogram(ctx.handle, _ptr(syms), _ptr(sym_off), n, _ptr(chunk_hist),
                                  _ptr(hist)), "rc_histogram")
    return hist, (chunk_hist[:n] if per_chunk else None)


def build_model(syms, sym_off, target_total=1 << 16, n_symbols=256, all_symbols=True, ctx=None):
    """Histogram of the batch on the GPU, then a StaticModel of its (scaled) table."""
    hist, _ = histogram(syms, sym_off, ctx=ctx)
    counts = hist.cpu().numpy().astype(np.uint64)
    if n_symbols < 256 and counts[n_symbols:].any():
        raise ValueError(f"symbols >= {n_symbols} present")
    c, cum, total = quantize_counts(counts[:n_symbols], target_total, all_symbols)
    return StaticModel(c, cum, total, ctx=ctx or default_context(syms.device.index))


def ideal_bits(model, chunk_hist):
    """rc_ideal_bits: float64[n] tensor, per chunk sum of log2(total / c[s]) over its symbols
    (inf if the chunk holds a symbol with c == 0).  model: a StaticModel (its host table)."""
    torch = _torch()
    _check_dev(chunk_hist, "chunk_hist", (torch.int32,))
    n = chunk_hist.shape[0] if chunk_hist.dim() == 2 else 0
    if chunk_hist.dim() != 2 or chunk_hist.shape[1] != 256:
        raise ValueError("chunk_hist must be [n_chunks, 256]")
    bits = torch.empty(max(n, 1), dtype=torch.float64, device=chunk_hist.device)
    ctx = model.ctx
    ctx.bind_stream()
    c = np.ascontiguousarray(model.c, dtype=np.uint32)
    N.check(ctx._lib.rc_ideal_bits(ctx.handle, ctypes.c_void_p(c.ctypes.data), len(c),
                                   model.total, _ptr(chunk_hist), n, _ptr(bits)),
            "rc_ideal_bits")
    return bits[:n]
