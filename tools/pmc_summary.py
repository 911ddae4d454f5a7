"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/) per kernel: mean counters per call.

    python tools/pmc_summary.py <root> [--by-grid]

--by-grid: one row per (kernel, grid size), so two launches of one kernel with
different grids (e.g. the N>1 worker merge over N x Pd buckets and the server
merge over its Pd x m server buckets, both k_bd_reduce) are told apart."""
import collections
import csv
import glob
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
by_grid = "--by-grid" in sys.argv
root = args[0] if args else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:36]
        if by_grid:
            name += f" [grid {int(r['Grid_Size']) // max(1, int(r['Workgroup_Size']))}]"
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
