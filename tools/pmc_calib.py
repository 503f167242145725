"""Summarise a tools/pmc_calib run (FETCH_SIZE / WRITE_SIZE / kernel-trace passes):

    gpurun -- 'rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/f ... -- ./tools/pmc_calib && ...'
    python tools/pmc_calib.py gpurun_out/calib --tag r01

Writes profiles/<tag>/pmc_calib.json: for each per-lane burst shape, the true bytes per counted
byte (true = n_chunks x 64 KiB per launch) and the achieved rate.
"""
import argparse
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = (1 << 18) * 65536


def rows(pattern):
    for fn in glob.glob(pattern):
        with open(fn) as f:
            yield from csv.DictReader(f)


def shape(name):
    b = int(name.split("<")[1].split(",")[0])
    return f"{'write' if 'true' in name else 'read'} {16 * b} B/lane"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("run")
    p.add_argument("--tag", required=True)
    a = p.parse_args()
    res = {}
    for sub, ctr, kind in (("f", "FETCH_SIZE", "read"), ("w", "WRITE_SIZE", "write")):
        for r in rows(os.path.join(a.run, sub, "*counter_collection.csv")):
            if "k_calib" in r["Kernel_Name"] and shape(r["Kernel_Name"]).startswith(kind):
                res.setdefault(shape(r["Kernel_Name"]), {})[f"true_bytes_per_{ctr}_byte"] = round(
                    BYTES / (float(r["Counter_Value"]) * 1024), 4)
    for r in rows(os.path.join(a.run, "t", "*kernel_stats.csv")):
        if "k_calib" in r["Name"]:
            res.setdefault(shape(r["Name"]), {})["TB_s"] = round(BYTES / float(r["AverageNs"]) / 1e3, 3)
    out = os.path.join(ROOT, "profiles", a.tag, "pmc_calib.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"bytes_per_launch": BYTES, "shapes": res}, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
