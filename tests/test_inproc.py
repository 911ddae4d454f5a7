"""In-process multi-rank transport (parallel/inproc.py): N rank threads, one
device, collective semantics — checked against the same single-table oracle
as the multi-process gloo tests (tests/test_engine_cpu.py)."""
import numpy as np
import pytest
import torch

from test_engine_cpu import DIM, ROUNDS, _grads_for, _keys_for, _oracle


def _engine_rank(rank, groups, servers, workers, opt_kind, device):
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    if device.type == "cuda":
        from swiftsnails_amd.ops.table import HbmTable

        torch.cuda.set_device(device)
        table_cls = lambda: HbmTable(DIM, 4096, Optimizer(opt_kind, lr=0.1),  # noqa: E731
                                     InitConfig("uniform", 0.2, 0.01), device=device)
    else:
        from swiftsnails_amd.ops.host_table import HostTable

        table_cls = lambda: HostTable(DIM, 4, Optimizer(opt_kind, lr=0.1),  # noqa: E731
                                      InitConfig("uniform", 0.2, 0.01))
    tr, ct = (g.transports(device)[rank] for g in groups)
    try:
        ctx = torch.cuda.stream(torch.cuda.Stream(device)) if device.type == "cuda" else None
        if ctx is not None:
            ctx.__enter__()
        table = table_cls() if rank in servers else None
        eng = PSEngine(table, tr, max_keys=300, dim=DIM, frag_num=64, server_ranks=servers,
                       device=device, count_transport=ct)
        pulled = {}
        for rnd in range(ROUNDS):
            k = _keys_for(rank, rnd) if rank in workers else np.zeros(0, np.int64)
            r = eng.pull(torch.from_numpy(k).to(device))
            pulled[(rank, rnd)] = eng.gather(r, len(k)).cpu().numpy().copy()
            if len(k):
                eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)).to(device))
            eng.push(r)
        if device.type == "cuda":
            torch.cuda.synchronize()
            eng.check()
        return pulled, (table.to_dict(with_state=True) if table is not None else {})
    except BaseException:
        for g in groups:
            g.abort()
        raise


def _check_against_oracle(res, world, workers, opt):
    merged, pulled = {}, {}
    for pl, st in res:
        assert not (set(st) & set(merged)), "a key lives on two shards"
        merged.update(st)
        pulled.update(pl)
    ref_state, ref_pulled = _oracle(world, workers, opt)
    assert set(merged) == set(ref_state)
    for k in ref_state:
        np.testing.assert_allclose(merged[k], ref_state[k], rtol=3e-5, atol=3e-6)
    for key, v in ref_pulled.items():
        np.testing.assert_allclose(pulled[key], v, rtol=3e-5, atol=3e-6)


@pytest.mark.parametrize("world,servers,workers,opt", [
    (2, [0, 1], [0, 1], "adagrad"),
    (4, [0, 1], [2, 3], "ftrl"),      # split roles: 2 servers + 2 workers
    (8, list(range(8)), list(range(8)), "adagrad"),
])
def test_inproc_engine_cpu(world, servers, workers, opt):
    from swiftsnails_amd.parallel.inproc import InprocGroup, run_ranks

    groups = (InprocGroup(world, timeout=120), InprocGroup(world, timeout=120))
    res = run_ranks(world, _engine_rank, groups, servers, workers, opt, torch.device("cpu"),
                    timeout=300)
    _check_against_oracle(res, world, workers, opt)


def test_inproc_allreduce_barrier_and_failure_cpu():
    from swiftsnails_amd.parallel.inproc import InprocGroup, run_ranks

    g = InprocGroup(3, timeout=60)

    def body(rank):
        t = torch.tensor([float(rank + 1), 10.0 * rank])
        g.transports()[rank].allreduce_(t, "sum")
        m = torch.tensor([float(rank)])
        g.transports()[rank].allreduce_(m, "max")
        g.transports()[rank].barrier()
        return t.tolist(), m.item()

    out = run_ranks(3, body)
    assert all(o == ([6.0, 30.0], 2.0) for o in out)

    # a rank that fails aborts the group: the others do not hang
    g2 = InprocGroup(3, timeout=60)

    def bad(rank):
        try:
            if rank == 1:
                raise ValueError("rank 1 failed")
            g2.transports()[rank].barrier()
        except BaseException:
            g2.abort()
            raise

    with pytest.raises(ValueError, match="rank 1 failed"):
        run_ranks(3, bad, timeout=60)


@pytest.mark.gpu
@pytest.mark.parametrize("world,servers,workers,opt", [
    (4, [0, 1, 2, 3], [0, 1, 2, 3], "adagrad"),
    (4, [0, 1], [2, 3], "sgd"),
])
def test_inproc_engine_gpu(world, servers, workers, opt):
    from swiftsnails_amd.parallel.inproc import InprocGroup, run_ranks

    groups = (InprocGroup(world, timeout=120), InprocGroup(world, timeout=120))
    res = run_ranks(world, _engine_rank, groups, servers, workers, opt,
                    torch.device("cuda", 0), timeout=300)
    _check_against_oracle(res, world, workers, opt)


def _rehearse(args):
    import importlib.util
    import json
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("rehearse_world",
                                                  os.path.join(root, "tools", "rehearse_world.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = mod.main(args)
    out = json.loads([l for l in buf.getvalue().splitlines() if l.startswith("{")][-1])
    return rc, out


@pytest.mark.gpu
@pytest.mark.parametrize("model,world,servers,workers", [
    ("sparse_lr", 8, "all", "all"),  # the bench layout, small batch
    ("word2vec", 4, "0-1", "2-3"),   # split servers + workers
    ("word2vec", 4, "all", "all"),   # BASELINE config 3: 4 colocated ranks
    ("fm", 4, "all", "all"),
])
def test_rehearse_world_gpu(model, world, servers, workers, monkeypatch):
    """N rank threads on one GPU through the N>1 engine path (pull-ahead for
    FM / word2vec, synchronous rounds for sparse LR): no dedup overflow, every
    checked key on the shard the router names, loss goes down on every
    worker."""
    extra = (["--batch", "2048", "--vocab", "20000", "--dim", "64"] if model == "word2vec"
             else ["--batch", "4096", "--fields", "13", "--features", "2000000"])
    rc, out = _rehearse(["--world", str(world), "--model", model, "--servers", servers,
                         "--workers", workers, "--steps", "24", "--warmup", "2",
                         "--log-every", "4", "--timeout", "100"] + extra)
    assert rc == 0, out
    assert out["misrouted"] == 0
    ranks = out["ranks"]
    assert sum(r.get("keys_checked", 0) for r in ranks) > 0
    for r in ranks:
        assert r["pull_ahead"] == (model != "sparse_lr")
        if r["worker"]:
            l = r["losses"]
            assert np.isfinite(l).all() and l[-1] < l[0], (r["rank"], l)
        if r["server"]:
            assert r["table_keys"] > 0
        else:
            assert "table_keys" not in r
