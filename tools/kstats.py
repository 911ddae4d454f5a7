#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, per step.

    python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv [steps]
    python tools/kstats.py gpurun_out/prof/run_results.db [steps]

steps: the steps the run executed (bench --steps + --warmup, + the
calibration's on N>1 paths); kernels with fewer launches are set-up work.
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
    """With ``steps`` (the steps the profiled run executed, warmup included):
    kernels launched at least once per step are the step's work (us/step
    column); kernels with fewer launches (table prefill / fill, probe
    histograms, start-up copies, the pull-ahead calibration's extras) are
    listed apart with their totals only, so a set-up launch never reads as
    per-step time."""
    rows = _rows(path)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    step_rows = [r for r in rows if not steps or int(r["Calls"]) >= steps]
    other = [r for r in rows if steps and int(r["Calls"]) < steps]
    tot = sum(float(r["TotalDurationNs"]) for r in step_rows)
    print(f"{'kernel':64s} {'calls':>6} {'avg us':>8} {'total ms':>9} {'%':>5}"
          + (f" {'us/step':>8}" if steps else ""))
    for r in step_rows[:40]:
        t = float(r["TotalDurationNs"])
        line = (f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
                f"{t / 1e6:9.2f} {100 * t / tot:5.1f}")
        if steps:
            line += f" {t / 1e3 / steps:8.1f}"
        print(line)
    if steps:
        print(f"{'per-step total':64s} {'':>6} {'':>8} {tot / 1e6:9.2f} {'':>5} "
              f"{tot / 1e3 / steps:8.1f}")
    if other:
        print(f"\nset-up / occasional kernels (fewer than {steps} launches; not per-step work):")
        for r in other[:20]:
            t = float(r["TotalDurationNs"])
            print(f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
                  f"{t / 1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
