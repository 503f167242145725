"""Randomised parity soak of the batch coders against the C oracle (GPU box), for a time budget.

Every iteration draws a static model and a batch, encodes and decodes it with the HIP kernels
(rc_encode_batch / rc_decode_batch, the drop-in for Encoder::encode / Decoder::decode,
encoder.rs:24-46, decoder.rs:14-54) and with oracle/rc_oracle.c (orc_encode_batch /
orc_decode_batch, 16 host threads), and requires the same bytes, lengths and flags chunk for
chunk, and the GPU decode of the GPU bytes to return the input.  The draws cover what the
kernels specialise on:
  model   uniform 256; Zipf(s) over 256 with s in [0.3, 2.5]; random counts over n in [1, 256]
          symbols, some with zero frequencies (never drawn in the data); totals quantised to a
          power of two (2^8 .. 2^16), a non-power-of-two in [257, 2^16), small totals below 256,
          and wide totals up to 2^24 (the paths: DIV_POW2 / DIV_MAGIC, direct tables, LUT 4
          buckets, the wide bucket tables)
  data    drawn from the model, or uniform over the symbols with c > 0 (every symbol as often:
          rare symbols of skewed models exercise both renormalisation loops), or runs of one
          symbol
  chunks  1 .. 3000 chunks, lengths 0 .. 70000 with ragged mixes (0, 1, 7, 4095, 65536, ...)
A quarter of the iterations instead draw one of:
  adaptive    the build-defined adaptive model (rc_model_create_adaptive) with random valid
              parameters, 1 .. 300 ragged chunks, against orc_encode_adaptive chunk by chunk
  stream-enc  1 .. 200 resumable streams of random (c, cum, total) triples, valid or not (the
              reference's panics and endless loops become flags at the same symbol), one
              rc_stream_encode call with finish, against orc_stream_encode: bytes, per-symbol
              counts, state and flags
  stream-dec  1 .. 200 streams, valid or garbage code, decoded under one random table (zero
              frequencies, inconsistent cum) by rc_stream_decode, against orc_stream_decode:
              symbols, state and flags
Prints a progress line per iteration and one JSON summary line; exits 1 at the first mismatch
(after printing what differed).  The oracle is the checker here, never the thing measured.

Usage (GPU box): python3 tools/parity_soak.py [seconds] [seed]
"""
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import range_coder_rust_amd as rc  # noqa: E402
from oracle import cpu  # noqa: E402


def quantise(p, total, rng):
    """Counts summing to total with every p > 0 symbol at least 1 (largest remainders)."""
    p = np.asarray(p, np.float64)
    live = p > 0
    k = int(live.sum())
    if total < k:
        total = k
    c = np.zeros(len(p), np.int64)
    c[live] = 1
    rest = total - k
    w = p[live] / p[live].sum() * rest
    fl = np.floor(w).astype(np.int64)
    c[live] += fl
    left = rest - int(fl.sum())
    if left:
        frac = w - fl
        idx = np.flatnonzero(live)[np.argsort(-frac, kind="stable")[:left]]
        c[idx] += 1
    return c.astype(np.uint32)


def draw_model(rng):
    kind = rng.choice(["uniform", "zipf", "random", "sparse"], p=[0.15, 0.35, 0.3, 0.2])
    n = 256 if kind in ("uniform", "zipf") else int(rng.choice([1, 2, 3, 17, 100, 255, 256,
                                                                  int(rng.integers(1, 257))]))
    if kind == "uniform":
        p = np.ones(n)
    elif kind == "zipf":
        s = float(rng.uniform(0.3, 2.5))
        p = 1.0 / np.arange(1, n + 1) ** s
    elif kind == "random":
        p = rng.random(n) ** 3 + 1e-3
    else:
        p = rng.random(n) ** 2
        p[rng.random(n) < 0.4] = 0.0
        if p.sum() == 0:
            p[int(rng.integers(0, n))] = 1.0
    tk = rng.choice(["pow2", "nonpow2", "small", "wide"], p=[0.4, 0.3, 0.15, 0.15])
    if tk == "pow2":
        total = 1 << int(rng.integers(8, 17))
    elif tk == "nonpow2":
        total = int(rng.integers(257, 1 << 16))
        total += total & (total - 1) == 0
    elif tk == "small":
        total = int(rng.integers(1, 256))
    else:
        total = int(rng.integers((1 << 16) + 1, 1 << 24))
    c = quantise(p, total, rng)
    total = int(c.sum())
    cum = np.concatenate([[0], np.cumsum(c.astype(np.uint64))[:-1]]).astype(np.uint32)
    return f"{kind}/{tk}", c, cum, total


def draw_lengths(rng):
    n = int(rng.choice([1, 2, 7, 64, 257, 1000, int(rng.integers(1, 3001))]))
    mode = rng.choice(["same", "ragged", "edges"])
    if mode == "same":
        L = int(rng.choice([0, 1, 15, 16, 17, 4095, 4096, 16384, 65536, int(rng.integers(0, 70001))]))
        return np.full(n, L, np.int64)
    if mode == "ragged":
        return rng.integers(0, 70001, n).astype(np.int64)
    return rng.choice([0, 1, 2, 7, 8, 9, 63, 64, 65, 4095, 4097, 65535, 65536], n).astype(np.int64)


def draw_data(rng, c, total_len):
    live = np.flatnonzero(c)
    how = rng.choice(["model", "flat", "runs"], p=[0.6, 0.3, 0.1])
    if how == "model":
        p = c.astype(np.float64) / c.sum()
        return rng.choice(len(c), total_len, p=p).astype(np.uint8), how
    if how == "flat":
        return live[rng.integers(0, len(live), total_len)].astype(np.uint8), how
    out = np.empty(total_len, np.uint8)
    pos = 0
    while pos < total_len:
        k = int(rng.integers(1, 5000))
        out[pos:pos + k] = live[int(rng.integers(0, len(live)))]
        pos += k
    return out, how


def adaptive_iteration(rng):
    n_alpha = int(rng.choice([1, 2, 17, 100, 256, int(rng.integers(1, 257))]))
    inc = int(rng.choice([1, 5, 32, 255, int(rng.integers(1, 256))]))
    period = 1 << int(rng.integers(0, 9))
    lo, hi = n_alpha + inc * period, 65535 - inc * period
    if lo > hi:
        inc, period = 32, 256
        lo, hi = n_alpha + inc * period, 65535 - inc * period
    limit = int(rng.integers(lo, hi + 1))
    n = int(rng.choice([1, 7, 64, 65, int(rng.integers(1, 301))]))
    lens = rng.choice([0, 1, 2, 63, 64, 65, 4096, int(rng.integers(0, 20001))], n).astype(np.int64)
    s_exp = float(rng.uniform(0.0, 2.0))
    w = 1.0 / np.arange(1, n_alpha + 1) ** s_exp
    data = rng.choice(n_alpha, int(lens.sum()), p=w / w.sum()).astype(np.uint8)
    sym_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    caps = np.array([rc.slot_capacity(int(L), 16) for L in lens], np.int64)
    out_off = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
    m = rc.AdaptiveModel(n_alpha, inc, limit, period)
    d_out = torch.zeros(int(out_off[-1]) + 16, dtype=torch.uint8, device="cuda")
    ol, fe = rc.encode_batch(m, torch.from_numpy(np.concatenate([data, [0]]).astype(np.uint8)).cuda(),
                             torch.from_numpy(sym_off).cuda(), d_out, torch.from_numpy(out_off).cuda())
    dec = torch.zeros(int(sym_off[-1]) + 16, dtype=torch.uint8, device="cuda")
    fd = rc.decode_batch(m, d_out, torch.from_numpy(out_off[:-1].copy()).cuda(), ol, dec,
                         torch.from_numpy(sym_off).cuda())
    torch.cuda.synchronize()
    g_out, g_len, g_fe = d_out.cpu().numpy(), ol.cpu().numpy(), fe.cpu().numpy()
    bad = []
    for k in range(n):
        f, want, L = cpu.encode_adaptive(n_alpha, inc, limit, period, data[sym_off[k]:sym_off[k + 1]])
        a = int(out_off[k])
        if f != int(g_fe[k]) or L != int(g_len[k]) or bytes(g_out[a:a + L]) != want:
            bad.append(f"adaptive chunk {k}")
            break
    if not bad and ((fd.cpu().numpy() != 0).any() or
                    not np.array_equal(dec.cpu().numpy()[: int(sym_off[-1])], data)):
        bad.append("adaptive decode")
    m.close()
    return f"adaptive n={n_alpha} inc={inc} limit={limit} period={period}", n, int(lens.sum()), \
        int(g_len.sum()), bad


def random_triples(rng, n):
    t = np.empty((n, 3), np.uint64)
    for i in range(n):
        total = int(rng.choice([256, 65536, int(rng.integers(1, 1 << 32))]))
        c = int(rng.integers(1, total + 1)) if rng.random() < 0.97 else int(rng.integers(0, 1 << 32))
        cum = int(rng.integers(0, total - min(c, total) + 1)) if rng.random() < 0.97 else \
            int(rng.integers(0, 1 << 32))
        t[i] = (c, cum, total if rng.random() < 0.995 else 0)
    return t.astype(np.uint32)


def stream_enc_iteration(rng):
    ns = int(rng.integers(1, 201))
    streams = [random_triples(rng, int(rng.choice([0, 1, 5, int(rng.integers(0, 2001))])))
               for _ in range(ns)]
    lens = np.array([len(t) for t in streams], np.int64)
    sym_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    trip = np.concatenate([t.reshape(-1) for t in streams] + [np.zeros(3, np.uint32)])
    caps = 12 * lens + 8
    out_off = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
    states = rc.stream_states(ns)
    out = torch.zeros(int(out_off[-1]) + 16, dtype=torch.uint8, device="cuda")
    nb = torch.zeros(max(int(sym_off[-1]), 1), dtype=torch.uint8, device="cuda")
    ctx = rc.default_context(0)
    ol, fl = rc.stream_encode_batch(ctx, states, torch.from_numpy(trip.view(np.int32)).cuda(),
                                    torch.from_numpy(sym_off).cuda(), out,
                                    torch.from_numpy(out_off).cuda(), nbytes=nb, finish=True)
    torch.cuda.synchronize()
    h, ol, nbh = out.cpu().numpy(), ol.cpu().numpy(), nb.cpu().numpy()
    stt = states.cpu().numpy().view(np.uint64)
    bad = []
    for k, t in enumerate(streams):
        st = cpu.Stream.fresh()
        f, b, cnt = cpu.stream_encode(st, t, finish=True)
        lo, r, d, pos, n, fs = (int(x) for x in stt[k])
        got = h[out_off[k]: out_off[k] + ol[k]].tobytes()
        tup = st.tuple()
        if got != b or nbh[sym_off[k]: sym_off[k] + len(cnt)].tolist() != cnt.tolist() or \
                (lo, r, pos, n, fs & 0xFFFFFFFF, fs >> 32) != (tup[0], tup[1], tup[3], tup[4],
                                                               tup[5], tup[6]):
            bad.append(f"stream encode {k}")
            break
    return f"stream-enc streams={ns}", ns, int(lens.sum()), int(ol.sum()), bad


def stream_dec_iteration(rng):
    na = int(rng.choice([1, 2, 40, 256, int(rng.integers(1, 257))]))
    c = np.array([int(rng.choice([0, 1, int(rng.integers(1, 900))])) for _ in range(na)], np.uint32)
    if c.sum() == 0:
        c[0] = 1
    cum = np.concatenate([[0], np.cumsum(c.astype(np.uint64))[:-1]]).astype(np.uint32)
    total = int(c.sum())
    consistent = rng.random() < 0.7
    tc, tcum, ttot = c.copy(), cum.copy(), total
    if not consistent:  # an inconsistent table, as the reference decodes it anyway
        tcum = rng.integers(0, max(total, 1) + 1, na).astype(np.uint32)
        ttot = int(rng.choice([total, int(rng.integers(0, 1 << 32))]))
    ns = int(rng.integers(1, 201))
    codes = []
    live = np.flatnonzero(c)
    for k in range(ns):
        if rng.random() < 0.5:
            syms = live[rng.integers(0, len(live), int(rng.integers(0, 600)))].astype(np.uint8)
            codes.append(cpu.encode(c, cum, total, syms)[1])
        else:
            codes.append(rng.integers(0, 256, int(rng.integers(0, 120))).astype(np.uint8).tobytes())
    m = int(rng.integers(0, 700))
    clen = np.array([len(x) for x in codes], np.int64)
    coff = np.concatenate([[0], np.cumsum(clen)[:-1]]).astype(np.int64)
    blob = np.frombuffer(b"".join(codes) + b"\0" * 16, np.uint8)
    states = rc.stream_states(ns)
    sym_off = (np.arange(ns + 1) * m).astype(np.int64)
    syms = torch.zeros(ns * m + 16, dtype=torch.uint8, device="cuda")
    ctx = rc.default_context(0)
    rc.stream_decode_batch(ctx, torch.from_numpy(tc.view(np.int32)).cuda(),
                           torch.from_numpy(tcum.view(np.int32)).cuda(), ttot, states,
                           torch.from_numpy(blob.copy()).cuda(), torch.from_numpy(coff).cuda(),
                           torch.from_numpy(clen).cuda(), syms, torch.from_numpy(sym_off).cuda())
    torch.cuda.synchronize()
    stt = states.cpu().numpy().view(np.uint64)
    h = syms.cpu().numpy()
    bad = []
    for k, code in enumerate(codes):
        st = cpu.Stream.fresh()
        f, s = cpu.stream_decode(st, tc, tcum, ttot, code, m)
        lo, r, d, pos, n, fs = (int(x) for x in stt[k])
        if h[k * m: k * m + n].tolist() != s.tolist() or \
                (lo, r, d, pos, n, fs & 0xFFFFFFFF) != st.tuple()[:6]:
            bad.append(f"stream decode {k}")
            break
    return (f"stream-dec streams={ns} n_alpha={na} {'consistent' if consistent else 'inconsistent'}",
            ns, ns * m, int(clen.sum()), bad)


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20260518
    rng = np.random.default_rng(seed)
    rc.default_context(0)
    t_end = time.time() + budget
    it = chunks = syms_total = bytes_total = 0
    kinds = {}
    while time.time() < t_end:
        other = rng.random()
        if other < 0.25:
            fn = (adaptive_iteration if other < 0.1 else
                  stream_enc_iteration if other < 0.175 else stream_dec_iteration)
            name, n, nsym, nbytes, bad = fn(rng)
            it += 1
            chunks += n
            syms_total += nsym
            bytes_total += nbytes
            key = name.split()[0]
            kinds[key] = kinds.get(key, 0) + 1
            print(f"iter {it}: {name} -> {'ok' if not bad else 'MISMATCH ' + ', '.join(bad)}",
                  flush=True)
            if bad:
                print(json.dumps({"mismatch": bad, "iteration": it, "seed": seed, "draw": name}))
                return 1
            continue
        name, c, cum, total = draw_model(rng)
        lens = draw_lengths(rng)
        data, how = draw_data(rng, c, int(lens.sum()))
        n = len(lens)
        sym_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        live = c[c > 0]
        bits = math.log2(total / int(live.min())) if total > 1 else 0.0
        caps = np.array([rc.slot_capacity(int(L), bits + 0.5, slack=1.05) for L in lens], np.int64)
        out_off = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
        m = rc.StaticModel(c, cum, total)
        d_syms = torch.from_numpy(np.concatenate([data, np.zeros(1, np.uint8)])).cuda()
        d_out = torch.zeros(int(out_off[-1]) + 16, dtype=torch.uint8, device="cuda")
        out_len, fe = rc.encode_batch(m, d_syms, torch.from_numpy(sym_off).cuda(), d_out,
                                      torch.from_numpy(out_off).cuda())
        dec = torch.zeros(int(sym_off[-1]) + 16, dtype=torch.uint8, device="cuda")
        fd = rc.decode_batch(m, d_out, torch.from_numpy(out_off[:-1].copy()).cuda(), out_len, dec,
                             torch.from_numpy(sym_off).cuda())
        torch.cuda.synchronize()
        g_out, g_len = d_out.cpu().numpy(), out_len.cpu().numpy().astype(np.uint64)
        g_fe, g_fd = fe.cpu().numpy(), fd.cpu().numpy()
        g_dec = dec.cpu().numpy()[: int(sym_off[-1])]
        o_out, o_len, o_fe = cpu.encode_batch(c, cum, total, data, sym_off, out_off, threads=16)
        bad = []
        if not np.array_equal(g_len, o_len.astype(np.uint64)):
            bad.append("encode lengths")
        if not np.array_equal(g_fe.astype(np.uint32), o_fe.astype(np.uint32)):
            bad.append("encode flags")
        if not bad:
            for k in range(n):
                a, L = int(out_off[k]), int(g_len[k])
                if not np.array_equal(g_out[a:a + L], o_out[a:a + L]):
                    bad.append(f"encode bytes of chunk {k}")
                    break
        if not bad and (g_fd != 0).any():
            bad.append("decode flags")
        if not bad and not np.array_equal(g_dec, data):
            bad.append("decode output")
        m.close()
        it += 1
        chunks += n
        syms_total += int(lens.sum())
        bytes_total += int(g_len.sum())
        key = f"{name}/{how}"
        kinds[key] = kinds.get(key, 0) + 1
        print(f"iter {it}: {name} n_alpha={len(c)} total={total} data={how} chunks={n} "
              f"symbols={int(lens.sum())} -> {'ok' if not bad else 'MISMATCH ' + ', '.join(bad)}",
              flush=True)
        if bad:
            print(json.dumps({"mismatch": bad, "iteration": it, "seed": seed, "model": name,
                              "total": total, "n_alpha": len(c), "chunks": n}))
            return 1
        del d_syms, d_out, dec
    print(json.dumps({"seed": seed, "seconds": budget, "iterations": it, "chunks": chunks,
                      "symbols": syms_total, "code_bytes": bytes_total, "mismatches": 0,
                      "draws": dict(sorted(kinds.items()))}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
