"""What binds the static kernels: summarise tools/pmc_bound.sh's passes.

Usage: python3 tools/pmc_bound.py gpurun_out/bound_<TAG> [--json out.json]

Per kernel (one launch each of the uniform/direct-table and Zipf/bucket configurations):
  clock_ghz        GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md, DVFS)
  cycles           GRBM_GUI_ACTIVE / 8: shader cycles of one XCD over the launch
  waves_per_simd   SQ_WAVE_CYCLES x 4 / (1024 SIMDs x cycles): mean resident waves per SIMD
  valu_busy        SQ_ACTIVE_INST_VALU x 4 / (1024 x cycles): the share of SIMD cycles spent
                   executing VALU instructions (SQ_* count quad-cycles, summed over waves)
  active/wait_inst/wait_any   SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY as shares of
                   SQ_WAVE_CYCLES (issuing, issue-stalled on a dependency or pipe, parked on
                   s_waitcnt / barrier)
  cyc_per_valu     SIMD cycles per VALU instruction: 1024 x cycles / SQ_INSTS_VALU
  valu_cyc_each    SQ_ACTIVE_INST_VALU x 4 / SQ_INSTS_VALU: cycles a VALU instruction keeps
                   its wave active
The counter passes run slower than plain runs (profiled clocks read lower, guide item 2), so
rates come from each pass's own GRBM_GUI_ACTIVE and the trace pass's kernel time is reported
beside them.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def short(name):
    n = name.replace("void ", "")
    return n.split("(")[0]


def counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = short(r["Kernel_Name"])
            if not k.startswith(("k_encode_static", "k_decode_static")):
                continue
            acc[(k, fn, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(dict)
    for (k, _, _), c in acc.items():
        for name, v in c.items():
            if name == "GRBM_GUI_ACTIVE":
                out[k].setdefault("_grbm", []).append(v)
            else:
                out[k][name] = v
    return out


def trace_ms(d):
    res = defaultdict(list)
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = short(r["Kernel_Name"])
            if k.startswith(("k_encode_static", "k_decode_static")):
                res[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return {k: sum(v) / len(v) for k, v in res.items()}


def summarise(root):
    out = {}
    for cfg in ("uniform", "zipf", "shard"):
        d = os.path.join(root, cfg)
        if not os.path.isdir(d):
            continue
        ms = trace_ms(os.path.join(d, "trace"))
        for k, c in counters(d).items():
            grbm = c.pop("_grbm")
            cyc = sum(grbm) / len(grbm) / XCDS  # per-XCD shader cycles over the launch
            s = {"trace_ms": round(ms.get(k, float("nan")), 3), "cycles": cyc}
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                s["waves_per_simd"] = round(wc * 4 / (SIMDS * cyc), 3)
                for name, key in (("SQ_ACTIVE_INST_ANY", "active"),
                                  ("SQ_WAIT_INST_ANY", "wait_inst"), ("SQ_WAIT_ANY", "wait_any"),
                                  ("SQ_WAIT_INST_LDS", "wait_inst_lds")):
                    if name in c:
                        s[key] = round(c[name] / wc, 4)
            if "SQ_ACTIVE_INST_VALU" in c:
                s["valu_busy"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc), 4)
                s["valu_cyc_each"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / c["SQ_INSTS_VALU"], 3)
            if "SQ_INSTS_VALU" in c:
                s["cyc_per_valu"] = round(SIMDS * cyc / c["SQ_INSTS_VALU"], 3)
            if "SQ_ACTIVE_INST_LDS" in c:
                s["lds_busy"] = round(c["SQ_ACTIVE_INST_LDS"] * 4 / (SIMDS * cyc), 4)
            if "SQ_ACTIVE_INST_SCA" in c:
                s["salu_busy"] = round(c["SQ_ACTIVE_INST_SCA"] * 4 / (SIMDS * cyc), 4)
            s["counters"] = {n: v for n, v in sorted(c.items())}
            out[f"{cfg}:{k}"] = s
    return out


def main():
    root = sys.argv[1]
    res = summarise(root)
    for k, s in res.items():
        print(k)
        for n, v in s.items():
            if n != "counters":
                print(f"   {n:16s} {v}")
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
