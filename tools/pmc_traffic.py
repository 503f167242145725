"""Turn a tools/profile.sh run into the committed profile evidence.

    python tools/pmc_traffic.py gpurun_out/prof_r01 --tag r01

Writes profiles/<tag>/kernel_stats.csv (the rocprofv3 --stats summary of the default bench
command), profiles/<tag>/bench.json (the bench line of that same run), profiles/<tag>/pmc.json
(per-launch counters of the encode/decode kernels) and merges the headline key into
profiles/traffic.json, which bench.py reads for roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE, both in KiB: on gfx950 FETCH_SIZE tallies
128-B fabric reads at 64 B (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact.
"""
import argparse
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"encode": "k_encode_static", "decode": "k_decode_static"}


def counters(d):
    """{dom: {counter: mean value per dispatch}} over the encode/decode dispatches under d."""
    acc = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                for dom, kn in KERNELS.items():
                    if kn in r["Kernel_Name"]:
                        a = acc.setdefault(dom, {}).setdefault(r["Counter_Name"], {})
                        a[r["Dispatch_Id"]] = a.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {dom: {c: sum(v.values()) / len(v) for c, v in cs.items()} for dom, cs in acc.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("run", help="gpurun_out/prof_<tag> directory")
    p.add_argument("--tag", required=True)
    p.add_argument("--config", default="uniform")
    p.add_argument("--chunks", type=int, default=1 << 20)
    p.add_argument("--chunk-bytes", type=int, default=65536)
    a = p.parse_args()
    out = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(a.run, "trace", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(out, "kernel_stats.csv"))
    with open(os.path.join(a.run, "bench.json")) as f:
        line = [l for l in f if l.startswith("{")][-1]
    with open(os.path.join(out, "bench.json"), "w") as f:
        f.write(line)
    bench = json.loads(line)

    pmc = {}
    for sub in ("fetch", "write", "sq"):
        for dom, cs in counters(os.path.join(a.run, sub)).items():
            pmc.setdefault(dom, {}).update(cs)
    n_sym = a.chunks * a.chunk_bytes
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for dom, cs in pmc.items():
        hbm = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
        cs["hbm_bytes_per_launch"] = hbm
        cs["hbm_bytes_per_symbol"] = hbm / n_sym
        if "SQ_INSTS_VALU" in cs:
            cs["valu_per_wave_symbol"] = cs["SQ_INSTS_VALU"] / (n_sym / 64)
        traffic[f"{a.config}:{a.chunks}:{a.chunk_bytes}:{dom}"] = {
            "hbm_bytes_per_launch": int(hbm), "fetch_kib": cs["FETCH_SIZE"],
            "write_kib": cs["WRITE_SIZE"], "round": a.tag,
            "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE reads half)"}
    with open(os.path.join(out, "pmc.json"), "w") as f:
        json.dump(pmc, f, indent=1, sort_keys=True)
    with open(tpath, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for dom, cs in pmc.items():
        print(f"{dom}: {cs['hbm_bytes_per_symbol']:.3f} HBM B/sym "
              f"({cs['hbm_bytes_per_launch'] / 1e9:.2f} GB/launch)")
    print("bench:", bench["value"], bench["unit"], "roofline", bench["roofline"])


if __name__ == "__main__":
    main()
