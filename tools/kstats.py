#!/usr/bin/env python3
"""Summarise rocprofv3 kernel timings: top kernels by total time, per step.

    python tools/kstats.py <prof dir | run_kernel_trace.csv> --range timed --steps K
    python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv [steps]     (counts)
    python tools/kstats.py gpurun_out/prof/run_results.db [steps]           (counts)

Phase attribution (preferred): profile with ``--kernel-trace --marker-trace
--output-format csv``.  bench.py wraps its timed loop in a roctx range named
``timed`` (utils/tracing.py); a kernel belongs to the timed steps iff its
device start lies inside that range (the bench synchronises the device on
both sides of it, so start-up litmus, calibration, set-up and the final
checks all fall outside).  ``--steps`` is the bench's --steps.

Count attribution (older runs without markers): kernels launched at least
``steps`` times are the step's work; fewer launches are set-up work.
"""
import argparse
import csv
import os
import sys
from collections import defaultdict


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


def _find(path, suffix):
    if os.path.isdir(path):
        for root, _, files in os.walk(path):
            for f in sorted(files):
                if f.endswith(suffix):
                    return os.path.join(root, f)
        return None
    d = os.path.dirname(path)
    base = os.path.basename(path)
    cand = os.path.join(d, base.replace("kernel_trace.csv", suffix))
    return cand if os.path.exists(cand) else _find(d, suffix)


def marker_ranges(marker_csv, name):
    """(start, end) ns of every roctx range called ``name`` in a rocprofv3
    marker_api_trace.csv (the range's message is in one of its text
    columns, depending on the rocprofv3 version)."""
    out = []
    for r in csv.DictReader(open(marker_csv)):
        if name in (r.get("Function"), r.get("Message"), r.get("Operation"), r.get("Name")):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out)


def phase_rows(trace_csv, ranges):
    """Per kernel (calls, total ns) over the dispatches whose start lies in
    one of ``ranges``, and the same outside them."""
    inside = defaultdict(lambda: [0, 0])
    outside = defaultdict(lambda: [0, 0])
    for r in csv.DictReader(open(trace_csv)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        hit = any(a <= s <= b for a, b in ranges)
        acc = (inside if hit else outside)[r["Kernel_Name"]]
        acc[0] += 1
        acc[1] += e - s
    conv = lambda d: [{"Name": k, "Calls": str(c), "TotalDurationNs": str(t),  # noqa: E731
                       "AverageNs": str(t / max(1, c))} for k, (c, t) in d.items()]
    return conv(inside), conv(outside)


def _print(rows, steps, title=None, limit=40):
    rows = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if title:
        print(title)
    print(f"{'kernel':64s} {'calls':>6} {'avg us':>8} {'total ms':>9} {'%':>5}"
          + (f" {'us/step':>8}" if steps else ""))
    for r in rows[:limit]:
        t = float(r["TotalDurationNs"])
        line = (f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
                f"{t / 1e6:9.2f} {100 * t / max(tot, 1):5.1f}")
        if steps:
            line += f" {t / 1e3 / steps:8.1f}"
        print(line)
    if steps:
        print(f"{'per-step total':64s} {'':>6} {'':>8} {tot / 1e6:9.2f} {'':>5} "
              f"{tot / 1e3 / steps:8.1f}")


def main(path, steps=None, rng=None):
    if rng:
        trace = path if path.endswith("kernel_trace.csv") else _find(path, "kernel_trace.csv")
        marker = _find(path, "marker_api_trace.csv")
        if not trace or not marker:
            sys.exit(f"kstats: --range needs run_kernel_trace.csv and run_marker_api_trace.csv "
                     f"(rocprofv3 --kernel-trace --marker-trace -f csv) under {path}")
        ranges = marker_ranges(marker, rng)
        if not ranges:
            sys.exit(f"kstats: no roctx range {rng!r} in {marker}")
        ins, outs = phase_rows(trace, ranges)
        _print(ins, steps, f"kernels inside the roctx range {rng!r} ({len(ranges)} range(s), "
                           f"{steps} steps):")
        print()
        _print(outs, None, "outside it (start-up, litmus, calibration, set-up, checks; "
                           "totals only):", limit=20)
        return
    rows = _rows(path)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    step_rows = [r for r in rows if not steps or int(r["Calls"]) >= steps]
    other = [r for r in rows if steps and int(r["Calls"]) < steps]
    _print(step_rows, steps)
    if other:
        print(f"\nset-up / occasional kernels (fewer than {steps} launches; not per-step work):")
        for r in other[:20]:
            t = float(r["TotalDurationNs"])
            print(f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f} "
                  f"{t / 1e6:9.2f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("steps_pos", nargs="?", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--range", default=None, help="roctx range name (e.g. timed)")
    a = ap.parse_args()
    main(a.path, a.steps if a.steps is not None else a.steps_pos, a.range)
