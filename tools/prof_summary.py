"""Markdown summary of a rocprofv3 --kernel-trace --stats run.

python tools/prof_summary.py <dir with run_kernel_stats.csv / run_kernel_trace.csv> [timeline rows]
Prints the per-kernel table (ss:: kernels + anything over 1%) and the last
N kernels of the trace as a per-queue timeline (steady state)."""
import csv
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
print("| kernel | calls | avg us | min us | % of kernel time |")
print("|---|---|---|---|---|")
for r in rows:
    name = r["Name"].split("(")[0].replace("void ", "")
    pct = float(r["Percentage"])
    if not name.startswith("ss::") and pct < 1.0:
        continue
    print(f"| {name[:48]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
          f"{float(r['MinNs']) / 1e3:.1f} | {pct:.1f} |")
if n:
    tr = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    tr = [r for r in tr if "ss::" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"]][-n:]
    t0 = int(tr[0]["Start_Timestamp"])
    print("\n```\nqueue   start_us   end_us   dur_us  kernel")
    for r in tr:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        print(f"q{r['Queue_Id']:>2}  {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {nm}")
    print("```")
