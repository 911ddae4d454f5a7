#!/usr/bin/env python3
"""Per-stream timeline of the last steps of a rocprofv3 kernel trace.

    python tools/ktimeline.py gpurun_out/prof/run_kernel_trace.csv [last_us]

Prints, for the final `last_us` microseconds of the run, every dispatch as
(start offset, duration, queue, grid, name), so the kernels of one step can
be told apart by stream and the overlap read off directly."""
import csv
import sys


def main(path, last_us=3000.0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    end = max(int(r["End_Timestamp"]) for r in rows)
    t0 = end - last_us * 1e3
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0:
            continue
        name = r["Kernel_Name"].replace("void ", "").split("(")[0][:48]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']:>2} "
              f"grid={r['Grid_Size_X']:>9}x{r['Grid_Size_Y']:<3} {name}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 3000.0)
