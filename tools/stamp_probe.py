"""Per-wave timelines of the static coders from in-kernel stamps.

    python tools/stamp_probe.py build                 # CPU: variants/librc_amd_stamp*.so
    RC_LIB_PATH=variants/librc_amd_stamp.so \\
      python tools/stamp_probe.py run OUT --chunks 65536 131072 ... [--config uniform|zipf]
    python tools/stamp_probe.py report OUT/stamps_<cfg>.json

A -DRC_STAMP build has lane 0 of every wave of k_encode_static / k_decode_static record, at
entry and exit, the device-wide 100 MHz clock (s_memrealtime) and the shader clock (s_memtime),
plus HW_ID / XCC_ID (rc_common.h, RC_STAMP_*).  From them, per launch:
  * span: first entry to last exit (100 MHz ticks), against the HIP-event time of the launch;
  * per wave: cycles per symbol = (c1 - c0) / symbols of its chunk, and how many waves shared
    its SIMD on average over its lifetime (from the entry/exit intervals of the waves with the
    same XCC / SE / CU / SIMD);
  * the timeline: waves resident per SIMD at 200 points of the span, and the share of the span
    spent with fewer resident waves than the launch's peak (the tail of the last round).
The stamps cost two scalar clock reads per wave at entry and exit and five vector stores by
lane 0 at exit: nothing inside the symbol loops.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {"stamp": ["-DRC_STAMP"],
            # the same code with 16 KiB more LDS per decoder workgroup: 40 KiB -> 4 workgroups
            # (4 waves per SIMD) instead of 5 for the 24-KiB direct-table decoder
            "stamp_pad4": ["-DRC_STAMP", "-DRC_DEC_LDS_PAD=16384"]}
ONLY = ("rc_decode_pow2.hip", "rc_decode_magic.hip", "rc_encode.hip")
REC = np.dtype([("rt0", "<u8"), ("rt1", "<u8"), ("c0", "<u8"), ("c1", "<u8"),
                ("hwid", "<u4"), ("xcc", "<u4"), ("nsym", "<u4"), ("valid", "<u4")])


def build():
    import __graft_entry__ as g
    for tag, flags in VARIANTS.items():
        g.build_variant(os.path.join(ROOT, "variants", f"librc_amd_{tag}.so"), flags, only=ONLY)


def read(L, tu, n_waves):
    buf = np.zeros(n_waves, dtype=REC)
    fn = getattr(L, "rc_stamp_read_" + tu)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    got = fn(buf.ctypes.data, n_waves)
    assert got == n_waves, f"rc_stamp_read_{tu}: {got}"
    return buf


def run(out, chunks, cfg, L_bytes=65536):
    import torch
    import bench
    import range_coder_rust_amd as rc
    from range_coder_rust_amd import _native, synth
    lib = _native.load()
    for tu in ("enc", "dec_pow2"):
        assert hasattr(lib, "rc_stamp_read_" + tu), "not a -DRC_STAMP build (set RC_LIB_PATH)"
    ctx = rc.default_context(0)
    dev = torch.device("cuda", 0)
    nmax = max(chunks)
    bufs = bench.Leg.alloc(torch, dev, nmax, L_bytes)
    os.makedirs(out, exist_ok=True)
    res = {"config": cfg, "lib": os.environ.get("RC_LIB_PATH", ""), "launches": {}}
    for n in chunks:
        leg = bench.Leg(torch, rc, synth, ctx, cfg, n, L_bytes, 0, bufs)
        nw = (n + 63) // 64
        for kind in ("encode", "decode"):
            f = leg.encode if kind == "encode" else leg.decode
            tu = "enc" if kind == "encode" else "dec_pow2"
            f()  # warm (and the decoder's input)
            torch.cuda.synchronize()
            read(lib, tu, nw)  # clears
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            st = read(lib, tu, nw)
            key = f"{kind}_{n}"
            np.save(os.path.join(out, f"stamps_{cfg}_{key}.npy"), st)
            s = summarize(st, ms)
            res["launches"][key] = s
            print(key, json.dumps(s), flush=True)
        ok = int(leg.fenc.abs().sum()) == 0 and int(leg.fdec.abs().sum()) == 0 and \
            bench.equal_chunked(torch, leg.dec[: n * L_bytes], leg.syms[: n * L_bytes])
        res["launches"][f"ok_{n}"] = bool(ok)
        del leg
    with open(os.path.join(out, f"stamps_{cfg}.json"), "w") as fo:
        json.dump(res, fo, indent=1)


def simd_key(st):
    # HW_ID (gfx9): wave [3:0], SIMD [5:4], pipe [7:6], CU [11:8], SH [12], SE [15:13]
    return (st["xcc"].astype(np.uint64) << 32) | ((st["hwid"].astype(np.uint64) >> 4) & 0xFFF)


def summarize(st, ms, points=200):
    v = st[st["valid"] == 1]
    assert len(v), "no stamps"
    t0, t1 = int(v["rt0"].min()), int(v["rt1"].max())
    span_ms = (t1 - t0) / 1e5
    cyc = (v["c1"] - v["c0"]).astype(np.float64)
    dur = (v["rt1"] - v["rt0"]).astype(np.float64)
    clk = cyc / (dur / 1e8) / 1e9  # GHz per wave
    cps = cyc / np.maximum(v["nsym"], 1)  # shader cycles per symbol of one wave
    # resident waves per SIMD over each wave's lifetime (the wave itself included)
    keys = simd_key(v)
    share = np.zeros(len(v))
    order = np.argsort(keys, kind="stable")
    ks = keys[order]
    bounds = np.flatnonzero(np.diff(ks)) + 1
    for grp in np.split(order, bounds):
        a, b = v["rt0"][grp].astype(np.int64), v["rt1"][grp].astype(np.int64)
        for i, g in enumerate(grp):
            ov = np.clip(np.minimum(b, b[i]) - np.maximum(a, a[i]), 0, None)
            share[g] = ov.sum() / max(b[i] - a[i], 1)
    n_simd = len(bounds) + 1
    # timeline: waves resident (whole device, per SIMD) at `points` instants
    ts = np.linspace(t0, t1, points + 2)[1:-1]
    res_per_simd = np.array([((v["rt0"] <= t) & (v["rt1"] > t)).sum() for t in ts]) / n_simd
    peak = res_per_simd.max()
    tail = float((res_per_simd < 0.9 * peak).mean())
    by_w = {}
    for w in np.unique(np.round(share)):
        m = np.round(share) == w
        by_w[str(int(w))] = dict(waves=int(m.sum()), cycles_per_symbol=round(float(np.median(cps[m])), 1))
    return dict(
        waves=int(len(v)), simds=int(n_simd), hip_ms=round(ms, 3), span_ms=round(span_ms, 3),
        clock_ghz_median=round(float(np.median(clk)), 3),
        wave_ms_median=round(float(np.median(dur)) / 1e5, 3),
        wave_ms_min=round(float(dur.min()) / 1e5, 3), wave_ms_max=round(float(dur.max()) / 1e5, 3),
        cycles_per_symbol_median=round(float(np.median(cps)), 1),
        resident_share_mean=round(float(share.mean()), 2),
        by_resident=by_w,
        resident_per_simd_peak=round(float(peak), 2),
        tail_fraction_below_90pct_peak=round(tail, 3),
        timeline_per_simd=[round(float(x), 2) for x in res_per_simd[:: max(1, points // 40)]])


def report(path):
    d = json.load(open(path))
    for k, s in d["launches"].items():
        if not isinstance(s, dict):
            print(k, s)
            continue
        print(f"{k:16s} waves {s['waves']:6d} hip {s['hip_ms']:8.3f} ms span {s['span_ms']:8.3f} "
              f"wave {s['wave_ms_median']:7.3f} ms  cyc/sym {s['cycles_per_symbol_median']:6.1f} "
              f"shared {s['resident_share_mean']:4.2f} tail {s['tail_fraction_below_90pct_peak']:.3f} "
              f"clk {s['clock_ghz_median']}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "report"])
    ap.add_argument("path", nargs="?")
    ap.add_argument("--chunks", type=int, nargs="+",
                    default=[65536, 131072, 262144, 524288, 1048576])
    ap.add_argument("--config", default="uniform", choices=["uniform", "zipf"])
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    elif a.cmd == "run":
        run(a.path, a.chunks, a.config)
    else:
        report(a.path)
