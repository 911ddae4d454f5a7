#!/usr/bin/env python3
"""Kernel profile of an N-rank bench.py job with every rank on ONE GPU.

Spawns N rank processes (child processes, never exec) of ``bench.py`` with
the torch.distributed env set by hand, all on device 0 (SS_BENCH_DEVICE), each
wrapped in its own ``rocprofv3 --kernel-trace --stats`` (output
``<out>/rank<r>/run_kernel_stats.csv``).  The ranks time-share the GPU, so
kernel durations carry the other ranks' contention; what the profile shows is
the per-rank kernel work at the N-rank shapes (server buckets for N sources,
sub-bucket splits, per-destination segments) — the work an N-GPU job's rank
does — which a 1-rank run through the N>1 path cannot show.

    python tools/prof_world.py --world 8 --out gpurun_out/profw8 -- --steps 10 --warmup 3 \
        --transport xgmi --batch 131072
    python tools/prof_world.py --world 4 --no-prof --launch -- \
        --config configs/word2vec_1m_4x4.conf --steps 64 --warmup 16   # the config launcher
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "profw"))
    ap.add_argument("--timeout", type=float, default=400.0)
    ap.add_argument("--no-prof", action="store_true", help="run the ranks without rocprofv3")
    ap.add_argument("--pmc", default="",
                    help="counter pass instead of the kernel stats: rocprofv3 --pmc <counters> "
                         "(space-separated, one pass; <= 8 SQ / 4 TCC / 4 TCP per pass)")
    ap.add_argument("--prof-ranks", default="all",
                    help="ranks run under rocprofv3 (comma list or 'all'); the others run bare")
    ap.add_argument("--script", default="",
                    help="run this python script (repo-relative) per rank instead of bench.py")
    ap.add_argument("--launch", action="store_true",
                    help="run python -m swiftsnails_amd.launch (config jobs) instead of bench.py")
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    if not 1 <= a.world <= 12:
        raise SystemExit("prof_world: 1..12 ranks on one GPU")
    args = [x for x in a.bench_args if x != "--"]
    port = free_port()
    procs = []
    for r in range(a.world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.world),
                   LOCAL_WORLD_SIZE=str(a.world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SS_BENCH_DEVICE="0", SS_DEVICE="0", TMPDIR="/tmp")
        bench = (["python3", "-m", "swiftsnails_amd.launch"] + args if a.launch else
                 ["python3", os.path.join(ROOT, a.script)] + args if a.script else
                 ["python3", os.path.join(ROOT, "bench.py"), "--gpus", str(a.world)] + args)
        profiled = a.prof_ranks == "all" or str(r) in a.prof_ranks.split(",")
        if a.no_prof or not profiled:
            cmd = bench
        else:
            d = os.path.join(a.out, f"rank{r}")
            os.makedirs(d, exist_ok=True)
            what = (["--pmc"] + a.pmc.split() + ["--kernel-trace"] if a.pmc else
                    ["--kernel-trace", "--stats"])
            cmd = ["rocprofv3"] + what + ["--output-format", "csv", "-d", d, "-o", "run",
                                          "--"] + bench
        os.makedirs(a.out, exist_ok=True)
        log = open(os.path.join(a.out, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT,
                                       cwd=ROOT, start_new_session=True), log))
    t0, rc = time.time(), 0
    for p, log in procs:
        left = max(1.0, a.timeout - (time.time() - t0))
        try:
            c = p.wait(timeout=left)
        except subprocess.TimeoutExpired:
            c = 124
            for q, _ in procs:  # the job is wedged: end every rank's process group
                try:
                    os.killpg(q.pid, 9)
                except ProcessLookupError:
                    pass
        log.close()
        rc = rc or c
    with open(os.path.join(a.out, "rank0.log")) as f:
        for line in f:
            if line.startswith("{"):
                print(line.strip())
    print(f"prof_world: world {a.world} rc={rc} ({time.time() - t0:.0f} s)")
    return rc


if __name__ == "__main__":
    sys.exit(main())
