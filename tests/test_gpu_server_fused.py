"""The fused N>1 server pull of scalar rows (server.hip k_srv_pull1: dedup of
the received keys + table lookup-or-insert + response rows in one kernel)
against the three-kernel form (SS_SRV_FUSED=0) and, at world 1, against the
one-GPU fast path: sparse LR over the xGMI mailboxes with synchronous rounds
trains the same model step for step (float summation order aside)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo

pytestmark = pytest.mark.gpu


def _rank(rank, world, init, fused, transport, q):
    os.environ["SS_SRV_FUSED"] = fused
    os.environ["SS_PULL_AHEAD"] = "0"
    if world > 1:
        init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
        from swiftsnails_amd.ops.optim import Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import LoopbackTransport, TorchDistTransport
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if transport == "fast":
            tr = LoopbackTransport()
        else:
            store = dist.distributed_c10d._get_default_store() if world > 1 else None
            tr = XgmiTransport(rank, world, dev, store,
                               aux=TorchDistTransport() if world > 1 else None, timeout_s=60)
        data = CtrSynth(batch_size=4096, num_fields=13, num_features=300_000, tail_frac=0.2)
        table = make_lr_table(data.num_features, world, Optimizer("adagrad", lr=0.1), device=dev)
        eng = PSEngine(table, tr, max_keys=4096 * 13, dim=1, device=dev)
        w = SparseLRWorker(eng, data, rank=rank, world=world)
        losses = [float(w.step().sum().item()) for _ in range(12)]
        torch.cuda.synchronize()
        eng.check()
        q.put((rank, losses, table.to_dict(with_state=True), dict(eng.metrics.counters)))
    finally:
        if world > 1:
            dist.destroy_process_group()


def _job(world, fused, transport="xgmi"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_rank, args=(r, world, init, fused, transport, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return {r: (l, t, m) for r, l, t, m in res}


def _same(a, b, rtol):
    for r in a:
        np.testing.assert_allclose(a[r][0], b[r][0], rtol=rtol)
        ta, tb = a[r][1], b[r][1]
        assert ta.keys() == tb.keys()
        ks = list(ta.keys())
        np.testing.assert_allclose(np.stack([ta[k] for k in ks]), np.stack([tb[k] for k in ks]),
                                   rtol=1e-4, atol=1e-6)


def test_fused_server_pull_world1_matches_unfused_and_fast_path():
    fused, split, fast = _job(1, "1"), _job(1, "0"), _job(1, "1", "fast")
    _same(fused, split, 1e-5)
    _same(fused, fast, 1e-4)
    m = fused[0][2]
    assert 0 < m["server_unique"] == m["unique_recv"]  # one source: nothing to merge


def test_fused_server_pull_world3_matches_unfused():
    fused, split = _job(3, "1"), _job(3, "0")
    _same(fused, split, 1e-5)
    for r in fused:  # three sources: the servers merged duplicates across them
        m = fused[r][2]
        assert 0 < m["server_unique"] < m["unique_recv"]
