"""Print the last N kernels of a rocprofv3 kernel trace as a per-stream timeline."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "run_kernel_trace.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    print(f"q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} {s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f}  {name}"
          f"  grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}")
