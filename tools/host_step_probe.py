#!/usr/bin/env python3
"""Is the bench step host-bound or blocked on the device?  Times each
worker.step() call on the host WITHOUT synchronising, then the final drain:
if every call returns in ~the host's own launch time the GPU runs a queue
of work ahead; if calls take ~the GPU step time, something in the step
blocks the host on the device (and the route stream cannot run ahead)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = int(os.environ.get("B", "262144"))
    data = CtrSynth(batch_size=B, num_fields=39, num_features=1_000_000_000)
    table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.05), load=0.5,
                          device=dev, init=lr_init("uniform", 0.01))
    eng = PSEngine(table, None, max_keys=B * 39, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    for _ in range(10):
        w.step()
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(30):
        a = time.perf_counter()
        w.step()
        ts.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("host us per step call:", [round(1e6 * x) for x in ts])
    print(f"issue {1e3 * (t1 - t0):.2f} ms for 30 steps, drain {1e3 * (t2 - t1):.2f} ms, "
          f"total {1e3 * (t2 - t0) / 30:.3f} ms/step")


if __name__ == "__main__":
    main()
