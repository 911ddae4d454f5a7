"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/) per kernel: mean counters per call."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:36]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for k in acc.values() for c in k})
print("| kernel | " + " | ".join(cols) + " |")
print("|---" * (len(cols) + 1) + "|")
for k, d in sorted(acc.items()):
    if not k.startswith("ss::"):
        continue
    vals = []
    for c in cols:
        v = d.get(c)
        vals.append(f"{sum(v) / len(v):.3g}" if v else "")
    print(f"| {k} | " + " | ".join(vals) + " |")
