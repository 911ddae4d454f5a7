#!/usr/bin/env python3
"""Long run of the headline configuration (bench.py's table, engine and
worker): per-window ms/step while the region table fills, then the table's
probe-length histogram and per-region occupancy (the fullest region is what
would fill first: keys probe only inside their own region).

    python tools/long_run.py --steps 2000 --window 100 > long.json
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--window", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--load", type=float, default=0.5)
    a = ap.parse_args()
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = CtrSynth(batch_size=a.batch, num_fields=39, num_features=a.features, tail_frac=0.1)
    table = make_lr_table(a.features, 1, optimizer=Optimizer("adagrad", lr=0.05), load=a.load,
                          device=dev, init=lr_init("uniform", 0.01))
    eng = PSEngine(table, None, max_keys=a.batch * 39, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    assert eng.claim and eng.fast1
    for _ in range(a.warmup):
        w.step()
    torch.cuda.synchronize()
    windows = []
    for k in range(a.steps // a.window):
        t0 = time.perf_counter()
        for _ in range(a.window):
            w.step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        n = table.size()
        windows.append({"steps_done": (k + 1) * a.window, "ms_per_step": round(1e3 * el / a.window, 4),
                        "table_keys": n, "load": round(n / table.capacity, 4),
                        "loss": round(w.mean_loss(), 5)})
        print(json.dumps(windows[-1]), file=sys.stderr, flush=True)
    eng.check()
    ms = [x["ms_per_step"] for x in windows]
    out = {"config": {"batch": a.batch, "features": a.features, "load": a.load,
                      "capacity": table.capacity, "rbits": table.rbits},
           "windows": windows,
           "drift_last_vs_first": round(ms[-1] / ms[0] - 1.0, 4) if ms else None,
           "ms_min": min(ms), "ms_max": max(ms),
           "table": table.stats(), "probe_hist": table.probe_histogram(32).tolist(),
           "regions": table.region_occupancy()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
