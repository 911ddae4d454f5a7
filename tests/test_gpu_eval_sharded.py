"""Sharded evaluation and N>1 training quality (xGMI ranks on one GPU).

Sparse LR trained on the same samples at world 1, 2 and 4 — per-rank batch
B / N, so every round covers exactly world 1's batch (the generator gives
rank r of N the samples [(step*N + r) * B/N, ...)) — then evaluated on the
same held-out samples through the collective read-only pull
(PSEngine.lookup: every shard answers, nothing is inserted).  The servers'
merged push (one AdaGrad step on the sum of the workers' gradients per key)
makes a round at world N the same update as world 1's step, so the held-out
AUC must agree within 0.005."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo

pytestmark = pytest.mark.gpu

B, F, FEATS, STEPS = 8192, 13, 200_000, 30


def _train_eval(rank, world, dev, transport):
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.parallel.engine import PSEngine

    data = CtrSynth(batch_size=B // world, num_fields=F, num_features=FEATS, tail_frac=0.05)
    table = make_lr_table(FEATS, world, device=dev)
    eng = PSEngine(table, transport, max_keys=(B // world) * F, dim=1, device=dev)
    w = SparseLRWorker(eng, data, rank=rank, world=world)
    for _ in range(STEPS):
        w.step()
    torch.cuda.synchronize()
    eng.check()
    before = table.size()
    ev = w.evaluate(batches=2)
    assert table.size() == before  # read-only: nothing inserted
    return ev, before


def _rank(rank, world, init, q):
    os.environ["SS_PULL_AHEAD"] = "0"
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.parallel.transport import TorchDistTransport
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        tr = XgmiTransport(rank, world, dev, dist.distributed_c10d._get_default_store(),
                           aux=TorchDistTransport(), timeout_s=60)
        ev, n = _train_eval(rank, world, dev, tr)
        q.put((rank, ev, n))
    finally:
        dist.destroy_process_group()


def _world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_rank, args=(r, world, init, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    evs = [ev for _, ev, _ in res]
    for ev in evs[1:]:  # every rank reports the same global metrics
        assert ev == evs[0]
    return evs[0], sum(n for _, _, n in res)


def test_sharded_eval_matches_world1():
    from swiftsnails_amd.parallel.transport import LoopbackTransport

    dev = torch.device("cuda", 0)
    ref, n1 = _train_eval(0, 1, dev, LoopbackTransport())
    assert ref["auc"] > 0.6 and ref["samples"] == 2 * B
    for world in (2, 4):
        ev, n = _world(world)
        assert ev["samples"] == 2 * B
        assert n == n1  # the same keys trained, each on exactly one shard
        assert abs(ev["auc"] - ref["auc"]) < 0.005, (world, ev, ref)
        assert abs(ev["auc_truth"] - ref["auc_truth"]) < 1e-9
