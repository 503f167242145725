"""Summarise tools/traffic_ab.sh: per build, kernel rates and read bytes per launch.

Usage: python3 tools/traffic_ab.py gpurun_out/traffic_<TAG>
Read bytes = 32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B (the by-size request sum that
profiles/r02/pmc_calib.json calibrated against known byte counts)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ALG = {"uniform": 2 ** 36, "zipf": 2 ** 36}


def main(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        lib = os.path.basename(d)
        res = {}
        try:
            b = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
            z = b["extras"].get("zipf1.2", {})
            res["uniform"] = {"encode_gsym_s": b["encode_gsym_s"], "decode_gsym_s": b["decode_gsym_s"]}
            res["zipf"] = {"encode_gsym_s": z.get("encode_gsym_s"), "decode_gsym_s": z.get("decode_gsym_s")}
        except Exception as e:  # noqa: BLE001
            res["bench_error"] = str(e)
        acc = defaultdict(lambda: defaultdict(float))
        for fn in glob.glob(os.path.join(d, "rd", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(fn)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if k.startswith(("k_encode_static", "k_decode_static")):
                    acc[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        kern = []
        for (k, disp), c in sorted(acc.items(), key=lambda kv: int(kv[0][1])):
            rd = 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + \
                128 * c["TCC_EA0_RDREQ_128B_sum"]
            kern.append({"kernel": k, "dispatch": int(disp), "read_gb": round(rd / 1e9, 2)})
        res["reads"] = kern
        out[lib] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
