#!/usr/bin/env python3
"""How much of a straggler's delay do the other ranks absorb, per staleness?

Runs the bench configuration as N xGMI rank processes on ONE GPU
(tools/prof_world.py --no-prof) while rank 1's host loop sleeps `delay` ms in
every step (SS_FAULT=delay:1:<ms>), for staleness 0 (synchronous rounds), 1
and 2 (rounds pulled 1 / 2 ahead: SS_PULL_AHEAD=1 SS_STALENESS=k), and
reports ms per step of the whole job (max over ranks, as bench.py times it).

    python tools/straggler.py --world 4 --delays 0,2,5,10 --staleness 0,1,2 \
        --out gpurun_out/straggler -- --batch 65536 --steps 30 --warmup 6

The reference's workers never wait for each other (SwiftWorker.h:88-113;
the server applies each push as it arrives, server/init.h:115-132); here
rounds are collective, and this table is what a slow rank costs.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--delays", default="0,2,5,10", help="ms per step on rank 1")
    ap.add_argument("--staleness", default="0,1,2")
    ap.add_argument("--kind", default="delay", choices=["delay", "gpudelay"],
                    help="delay: rank 1's host loop sleeps; gpudelay: a kernel keeps its GPU "
                         "busy (a slow device)")
    ap.add_argument("--p", type=float, default=1.0, help="fraction of steps delayed (jitter)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "straggler"))
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    args = [x for x in a.bench_args if x != "--"]
    os.makedirs(a.out, exist_ok=True)
    rows = []
    for k in [int(x) for x in a.staleness.split(",")]:
        for d in [float(x) for x in a.delays.split(",")]:
            env = dict(os.environ, SS_STALENESS=str(k), SS_PULL_AHEAD="1" if k else "0")
            if d > 0:
                env["SS_FAULT"] = f"{a.kind}:rank=1:ms={d:g}" + (f":p={a.p:g}" if a.p < 1 else "")
            out = os.path.join(a.out, f"k{k}_d{d:g}")
            cmd = [sys.executable, os.path.join(ROOT, "tools", "prof_world.py"), "--world",
                   str(a.world), "--no-prof", "--out", out, "--timeout", str(a.timeout), "--",
                   "--transport", "xgmi", "--cal-steps", "0"] + args
            t0 = time.time()
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                               timeout=a.timeout + 60)
            js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not js:
                print(f"staleness {k} delay {d:g}: failed rc={r.returncode}\n{r.stdout[-2000:]}",
                      file=sys.stderr)
                return 1
            j = json.loads(js[-1])
            row = {"kind": a.kind, "p": a.p, "staleness": k, "delay_ms": d, "ms_per_step": j["ms_per_step"],
                   "pull_ahead": j["config"].get("pull_ahead"), "loss_last":
                   j["config"]["loss_last"], "wall_s": round(time.time() - t0, 1)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    base = {r["staleness"]: r["ms_per_step"] for r in rows if r["delay_ms"] == 0}
    with open(os.path.join(a.out, f"straggler_{a.kind}_p{a.p:g}.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    print(f"\n| staleness | delay (ms/step on rank 1) | ms/step | added vs no delay | "
          f"delay absorbed |")
    print("|---|---|---|---|---|")
    for r in rows:
        add = r["ms_per_step"] - base.get(r["staleness"], r["ms_per_step"])
        ab = 1.0 - add / (r["delay_ms"] * a.p) if r["delay_ms"] > 0 else float("nan")
        print(f"| {r['staleness']} | {r['delay_ms']:g} | {r['ms_per_step']:.3f} | {add:+.3f} | "
              f"{ab:.0%} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
