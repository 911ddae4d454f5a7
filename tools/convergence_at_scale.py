#!/usr/bin/env python3
"""Held-out quality of the bench configuration after training (1 GPU).

Trains the headline model exactly as bench.py does (1B-feature sparse LR,
batch 262144 x 39, AdaGrad, fused merge + update) and reports, every
`--every` steps, held-out AUC / log-loss of the learned model next to the AUC
of the generator's planted weights (the Bayes-optimal ceiling) — evidence that
the fast path trains the model, not just moves bytes.

    python tools/convergence_at_scale.py [--steps 600] [--every 100] [--batch 262144]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--eval-batches", type=int, default=4)
    a = ap.parse_args()
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = CtrSynth(batch_size=a.batch, num_fields=39, num_features=a.features, tail_frac=0.1)
    table = make_lr_table(a.features, 1, optimizer=Optimizer("adagrad", lr=a.lr), load=0.5,
                          device=dev)
    eng = PSEngine(table, None, max_keys=a.batch * 39, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    t0 = time.perf_counter()
    for i in range(1, a.steps + 1):
        w.step()
        if i % a.every == 0 or i == a.steps:
            torch.cuda.synchronize()
            ev = w.evaluate(a.eval_batches)
            row = {"step": i, "train_samples": i * a.batch,
                   "train_loss": round(w.mean_loss(), 5)}
            row.update({k: (round(v, 5) if isinstance(v, float) else v) for k, v in ev.items()})
            row.update({"table_keys": table.size(),
                        "seconds": round(time.perf_counter() - t0, 2)})
            print(json.dumps(row), flush=True)
    table.check()


if __name__ == "__main__":
    main()
