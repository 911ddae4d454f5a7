#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, per step.

    python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv [steps]
    python tools/kstats.py gpurun_out/prof/run_results.db [steps]
"""
import csv
import sys


def _rows(path):
    """kernel_stats.csv rows, or the same aggregated from a rocprofv3 rocpd
    database (``run_results.db``, the default output format)."""
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3

    c = sqlite3.connect(path)
    q = "select name, count(*), sum(duration), avg(duration) from kernels group by name"
    return [{"Name": n, "Calls": str(k), "TotalDurationNs": str(t), "AverageNs": str(a)}
            for n, k, t, a in c.execute(q)]


def main(path, steps=None):
    rows = _rows(path)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':64s} {'calls':>6} {'avg us':>8} {'total ms':>9} {'%':>5}"
          + (f" {'us/step':>8}" if steps else ""))
    for r in rows[:40]:
        t = float(r["TotalDurationNs"])
        line = (f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
                f"{t / 1e6:9.2f} {100 * t / tot:5.1f}")
        if steps:
            line += f" {t / 1e3 / steps:8.1f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
