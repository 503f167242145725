"""Summarise counter_collection.csv files: mean per dispatch of each counter, per kernel."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        if not k.startswith("k_"):
            continue
        acc[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, d in acc.items():
    per = defaultdict(list)
    for (disp, name), v in d.items():
        per[name].append(sum(v))
    print(k)
    for name in sorted(per):
        print(f"  {name:28s} {sum(per[name]) / len(per[name]):.4g}")
