"""CPU restatement of model construction (TEST INFRASTRUCTURE ONLY).

Checker for librc_amd.so's rc_histogram / rc_quantize_counts / rc_ideal_bits.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it; the product never does.

  histogram        FreqTable::new + add_alphabet_freq per symbol (examples/sample_impl.rs:49-60)
  calc_cum         FreqTable::calc_cum (sample_impl.rs:61-69): exclusive scan, total = sum
  quantize_counts  build-defined scaling of counts to a target total (include/range_coder.h,
                   rc_quantize_counts); with target 0 it is calc_cum's exact table
  ideal_code_length  PModel::ideal_code_length (src/pmodel.rs:14-40), f64
  ideal_bits       per chunk: sum over the chunk's symbols of ideal_code_length

Parity of the exact-table mode and ideal_code_length follows the reference's code directly;
the scaled mode and the batching are not in the reference (parity pinned only against this
restatement).
"""
import math

import numpy as np

Q_ALL_SYMBOLS = 1


def histogram(syms, n_symbols=256):
    """add_alphabet_freq for every symbol (sample_impl.rs:58-60), as counts[0..n)."""
    a = np.asarray(syms, dtype=np.uint8)
    return np.bincount(a, minlength=n_symbols).astype(np.uint64)[:max(n_symbols, int(a.max(initial=0)) + 1)]


def calc_cum(c):
    """FreqTable::calc_cum (sample_impl.rs:61-69): cum = exclusive prefix sum, total = sum."""
    cum, t = [], 0
    for x in c:
        cum.append(t)
        t += int(x)
    return cum, t


def quantize_counts(counts, target_total=0, qflags=0):
    """Returns (c, cum, total) lists, or None where rc_quantize_counts returns RC_E_BAD_MODEL."""
    counts = [int(x) for x in counts]
    n = len(counts)
    all_sym = bool(qflags & Q_ALL_SYMBOLS)
    N = sum(counts)
    if target_total == 0:
        c = [x + (1 if all_sym and x == 0 else 0) for x in counts]
    else:
        T = int(target_total)
        need = sum(1 for x in counts if all_sym or x > 0)
        if N == 0:
            if not all_sym:
                return None
            need = n
        if T < need or T > 0xFFFFFFFF:
            return None
        c = []
        for x in counts:
            if N == 0:
                c.append(1)
            elif x == 0 and not all_sym:
                c.append(0)
            else:
                c.append(max(1, (x * T + N // 2) // N))
        s = sum(c)
        if s < T:
            m = max(range(n), key=lambda i: (c[i], -i))  # largest, lowest index on ties
            c[m] += T - s
        elif s > T:
            excess = s - T
            for i in sorted(range(n), key=lambda i: (-c[i], i)):  # stable: largest first
                if excess == 0 or c[i] <= 1:
                    break
                take = min(excess, c[i] - 1)
                c[i] -= take
                excess -= take
            if excess:
                return None
    cum, total = calc_cum(c)
    if total == 0 or total > 0xFFFFFFFF:
        return None
    return c, cum, total


def ideal_code_length(c_i, total):
    """PModel::ideal_code_length (pmodel.rs:14-40); None where the reference returns Err."""
    p = float(c_i)
    if p == 0.0:
        return None
    return (math.log(float(total)) - math.log(p)) / math.log(2.0)


def ideal_bits(chunk_hist, c, total):
    """Per chunk, sum over bins in order 0..255 of count * ideal_code_length (inf where c == 0).
    The GPU accumulates with fma; this sums products, so compare with a relative tolerance."""
    icl = [ideal_code_length(c[i], total) if i < len(c) else None for i in range(256)]
    out = []
    for row in np.asarray(chunk_hist):
        acc = 0.0
        for i in range(256):
            h = int(row[i])
            if h:
                acc = acc + float(h) * icl[i] if icl[i] is not None else math.inf
        out.append(acc)
    return np.array(out, dtype=np.float64)
