#!/usr/bin/env python3
"""Time the collective read-only lookup (PSEngine.lookup) of an N-rank job:
the device path over the xGMI round (the reserved slot past the ring) against
the host-staged gloo path it replaced, after training the bench model a few
steps.  Run one process per rank (tools/prof_world.py --script), e.g. 4 ranks
on one GPU:

    python tools/prof_world.py --world 4 --no-prof --script tools/lookup_bench.py \\
        -- --keys 2500000 --steps 6

Rank 0 prints one JSON line: ms per lookup for each path, keys per rank, the
tables' total size before / after (unchanged: nothing is inserted), and
whether both paths returned the same rows."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=2_500_000, help="lookup keys per rank")
    ap.add_argument("--steps", type=int, default=6, help="training steps before the lookups")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dev_idx = int(os.environ.get("SS_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.select import build_engine
    from swiftsnails_amd.parallel.transport import default_gloo_ifname

    default_gloo_ifname()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = dist.distributed_c10d._get_default_store()
    data = CtrSynth(batch_size=a.batch, num_fields=39, num_features=a.features)
    table = make_lr_table(a.features, world, optimizer=Optimizer("adagrad", lr=0.05), load=0.5,
                          device=dev, init=lr_init("uniform", 0.01))
    max_keys = max(a.batch * 39, a.keys)

    def make(tr, ct, pt):
        return PSEngine(table, tr, max_keys=max_keys, dim=1, device=dev, count_transport=ct,
                        pull_transport=pt)

    eng, _, plane = build_engine("xgmi", rank, world, dev, store, make,
                                 log=lambda m: print(m, file=sys.stderr))
    w = SparseLRWorker(eng, data, rank=rank, world=world)
    for _ in range(a.steps):
        w.step()
    torch.cuda.synchronize()
    eng.check()

    def total_size():
        t = torch.tensor([table.size()], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())

    size0 = total_size()
    # keys: half trained (this rank's recent batches), half never seen
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    kt = torch.empty(a.batch * 39, dtype=torch.int64, device=dev)
    lab = torch.empty(a.batch, dtype=torch.float32, device=dev)
    data.generate(0, rank, world, kt, lab)
    seen = kt[torch.randint(0, kt.numel(), (a.keys // 2,), generator=g).to(dev)]
    fresh = torch.randint(1 << 41, 1 << 42, (a.keys - a.keys // 2,), generator=g,
                          dtype=torch.int64).to(dev)
    keys = torch.cat([seen, fresh])
    res = {}
    rows = {}
    slot = eng.lookup_slot
    for path in ("device", "gloo"):
        eng.lookup_slot = slot if path == "device" else None
        rows[path] = eng.lookup(keys)  # warm
        torch.cuda.synchronize()
        times = []
        for _ in range(a.reps):
            dist.barrier()
            t0 = time.perf_counter()
            eng.lookup(keys)
            torch.cuda.synchronize()
            dist.barrier()
            times.append(time.perf_counter() - t0)
        t = torch.tensor([min(times)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res[path] = round(1e3 * float(t.item()), 3)
    eng.lookup_slot = slot
    same = torch.equal(rows["device"].cpu(), rows["gloo"].cpu())
    ok = torch.tensor([1 if same else 0], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    size1 = total_size()
    if rank == 0:
        print(json.dumps({"world": world, "keys_per_rank": a.keys, "devices": plane.devices,
                          "ms_device": res["device"], "ms_gloo": res["gloo"],
                          "speedup": round(res["gloo"] / res["device"], 2),
                          "same_rows": bool(ok.item()), "table_size_before": size0,
                          "table_size_after": size1, "unchanged": size0 == size1,
                          "fresh_keys_read_zero": bool((rows["device"][a.keys // 2:] == 0)
                                                       .all().item())}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
