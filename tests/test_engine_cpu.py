"""Collective round engine on CPU: world 1 + multi-process gloo (world 2/3,
colocated and split server/worker roles), checked against a single-table
oracle that merges each round's gradients over ALL workers per key and
applies one update per distinct key (the servers' cross-source merge).
"""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo

DIM = 3
ROUNDS = 4


def _keys_for(rank, rnd):
    rng = np.random.default_rng(1000 * rank + rnd)
    return rng.integers(0, 400, size=257, dtype=np.int64)  # overlapping, duplicated


def _grads_for(keys, rank, rnd):
    k = keys.astype(np.float32)
    return np.stack([np.sin(k + rnd), np.cos(k * 0.5 + rank), np.full_like(k, 0.1 * (rank + 1))],
                    1).astype(np.float32)


def _oracle(world, workers, opt_kind):
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    t = HostTable(DIM, 4, Optimizer(opt_kind, lr=0.1), InitConfig("uniform", 0.2, 0.01))
    pulled = {}
    for rnd in range(ROUNDS):
        for r in workers:
            k = _keys_for(r, rnd)
            pulled[(r, rnd)] = t.pull_keys(k).numpy()
        # one merged gradient per distinct key over every worker's push
        ks = [_keys_for(r, rnd) for r in workers]
        gs = [_grads_for(k, r, rnd) for k, r in zip(ks, workers)]
        k = np.concatenate(ks)
        u, inv = np.unique(k, return_inverse=True)
        m = np.zeros((len(u), DIM), np.float64)
        np.add.at(m, inv, np.concatenate(gs).astype(np.float64))
        t.push_keys(u, m.astype(np.float32))
        t.next_round()
    return t.to_dict(with_state=True), pulled


def _run_rank(rank, world, init, servers, workers, opt_kind, q):
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.ops.host_table import HostTable
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        table = (HostTable(DIM, 4, Optimizer(opt_kind, lr=0.1), InitConfig("uniform", 0.2, 0.01))
                 if rank in servers else None)
        eng = PSEngine(table, TorchDistTransport(), max_keys=300, dim=DIM, frag_num=64,
                       server_ranks=servers, device="cpu")
        pulled = {}
        for rnd in range(ROUNDS):
            if rank in workers:
                k = _keys_for(rank, rnd)
            else:
                k = np.zeros(0, np.int64)
            kt = torch.from_numpy(k)
            r = eng.pull(kt)
            vals = eng.gather(r).numpy().copy()
            pulled[(rank, rnd)] = vals
            if len(k):
                eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)))
            eng.push(r)
        state = table.to_dict(with_state=True) if table is not None else {}
        q.put((rank, pulled, state))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,servers,workers,opt", [
    (2, [0, 1], [0, 1], "adagrad"),
    (3, [0, 1, 2], [0, 1, 2], "sgd"),
    (3, [0], [1, 2], "adagrad"),      # split: 1 server + 2 workers
    (3, [1, 2], [0], "ftrl"),         # split: 2 servers + 1 worker
    (4, [0, 1], [2, 3], "adam"),      # split: 2 servers + 2 workers (BASELINE config 3 shape)
    (8, list(range(8)), list(range(8)), "adagrad"),  # the 8-rank colocated layout of the bench
])
def test_engine_multiprocess_gloo(world, servers, workers, opt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_rank, args=(r, world, init, servers, workers, opt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    merged, pulled = {}, {}
    for rank, pl, st in res:
        assert not (set(st) & set(merged)), "a key lives on two shards"
        merged.update(st)
        pulled.update(pl)
    ref_state, ref_pulled = _oracle(world, workers, opt)
    assert set(merged) == set(ref_state)
    for k in ref_state:
        np.testing.assert_allclose(merged[k], ref_state[k], rtol=2e-5, atol=2e-6)
    for key, v in ref_pulled.items():
        np.testing.assert_allclose(pulled[key], v, rtol=2e-5, atol=2e-6)


def test_engine_world1_cpu_push_keys_and_pull_dense():
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    t = HostTable(2, 2, Optimizer("sgd", lr=1.0), InitConfig("zero"))
    eng = PSEngine(t, None, max_keys=100, dim=2, device="cpu")
    k = torch.tensor([5, 7, 5, 9, 7, 5])
    eng.push_keys(k, torch.ones(6, 2))
    v = eng.pull_dense(k).numpy()[:, 0]
    np.testing.assert_allclose(v, [-3, -2, -3, -1, -2, -3])


def test_engine_phase_tracing_cpu():
    """trace: 1 — the engine's route / pull / push phases land in the tracer
    (roctx ranges + host time; device time on GPU)."""
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.utils.tracing import Tracer

    t = HostTable(2, 2, Optimizer("sgd", lr=1.0), InitConfig("zero"))
    eng = PSEngine(t, None, max_keys=100, dim=2, device="cpu")
    eng.pull_dense(torch.tensor([1, 2, 3]))  # tracer off: nothing recorded, no error
    eng.tracer = Tracer(enabled=True, roctx=False)
    k = torch.tensor([5, 7, 5])
    for _ in range(3):
        rnd = eng.pull(k)
        eng.push(rnd)
    s = eng.tracer.summary()
    assert s["calls"]["route"] == 3 and s["calls"]["pull"] == 3 and s["calls"]["push"] == 3
    assert all(s["host_s"][k] >= 0 for k in ("route", "pull", "push"))


def test_effective_ndest_counts_receiving_servers():
    """Bucketed dedup sizing: buckets per destination come from
    the servers that actually receive keys, not the world size."""
    from swiftsnails_amd.ops.dedup import effective_ndest
    from swiftsnails_amd.parallel.router import HashFrag

    assert effective_ndest(HashFrag(8, 1024).rank_map(), 8) == 8
    assert effective_ndest(HashFrag(1, 1024).rank_map([2]), 4) == 1
    assert effective_ndest(HashFrag(3, 1024).rank_map([0, 1, 2]), 6) == 3  # 342/341/341
    assert effective_ndest(HashFrag(3, 4).rank_map(), 3) == 2  # one node owns half
    assert effective_ndest(np.zeros(1, np.int32), 4) == 1


def test_rounds_done_under_graph_replays():
    """A replay of a depth-step graph applies all its rounds at the period's
    first step: backups are labelled with what the device has applied."""
    from swiftsnails_amd.models.base import PipelinedWorker

    w = PipelinedWorker.__new__(PipelinedWorker)
    w._graphs, w.step_idx = None, 7
    assert w.rounds_done() == 7
    w._graphs, w._gbase, w._gper = [object()], 10, 4
    got = []
    for k in range(10, 19):
        w.step_idx = k
        got.append(w.rounds_done())
    assert got == [10, 14, 14, 14, 14, 18, 18, 18, 18]


def _run_uneven_rank(rank, world, init, quotas, every, q):
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.ops.host_table import HostTable
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        table = HostTable(DIM, 4, Optimizer("adagrad", lr=0.1), InitConfig("uniform", 0.2, 0.01))
        eng = PSEngine(table, TorchDistTransport(), max_keys=300, dim=DIM, frag_num=64,
                       device="cpu")
        rnd = 0
        while True:
            if rnd % every == 0 and eng.all_done(rnd >= quotas[rank]):
                break
            k = _keys_for(rank, rnd) if rnd < quotas[rank] else np.zeros(0, np.int64)
            r = eng.pull(torch.from_numpy(k))
            if len(k):
                eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)))
            eng.push(r)
            rnd += 1
        q.put((rank, rnd, table.to_dict(with_state=True)))
    finally:
        dist.destroy_process_group()


def test_uneven_shards_collective_termination():
    """Three workers with shards of 3, 7 and 2 rounds (SwiftWorker's own
    pace): a finished worker keeps serving empty rounds; every 4 rounds the
    ranks agree whether all are done (PSEngine.all_done); all stop at the
    same round, and the tables match the oracle in which each round merges
    only the workers that still had data."""
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    world, quotas, every = 3, [3, 7, 2], 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_uneven_rank, args=(r, world, init, quotas, every, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    stops = {rnd for _, rnd, _ in res}
    assert stops == {8}  # the first multiple of 4 at which all 7 rounds are done
    merged = {}
    for _, _, st in res:
        merged.update(st)
    t = HostTable(DIM, 4, Optimizer("adagrad", lr=0.1), InitConfig("uniform", 0.2, 0.01))
    for rnd in range(8):
        live = [r for r in range(world) if rnd < quotas[r]]
        if not live:
            t.next_round()
            continue
        ks = [_keys_for(r, rnd) for r in live]
        gs = [_grads_for(k, r, rnd) for k, r in zip(ks, live)]
        for k in ks:
            t.pull_keys(k)
        u, inv = np.unique(np.concatenate(ks), return_inverse=True)
        m = np.zeros((len(u), DIM), np.float64)
        np.add.at(m, inv, np.concatenate(gs).astype(np.float64))
        t.push_keys(u, m.astype(np.float32))
        t.next_round()
    ref = t.to_dict(with_state=True)
    assert set(merged) == set(ref)
    for k in ref:
        np.testing.assert_allclose(merged[k], ref[k], rtol=2e-5, atol=2e-6)


def _init_rows(keys):
    """user initialiser: w_j = key/1000 + j, AdaGrad state 0.5"""
    k = keys.to(torch.float64)
    w = torch.stack([k / 1000 + j for j in range(DIM)], 1)
    return torch.cat([w, torch.full((len(keys), DIM), 0.5, dtype=torch.float64)], 1).float()


def _pull_vals(keys, rows):
    """user pull transform: parameters scaled by 1/sqrt(state)"""
    return rows[:, :DIM] / rows[:, DIM:].sqrt()


def _run_access_rank(rank, world, init, q):
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.ops.host_table import HostTable
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        table = HostTable(DIM, 4, Optimizer("adagrad", lr=0.1), InitConfig("zero"))
        table.set_init_method(_init_rows)
        table.set_pull_method(_pull_vals)
        eng = PSEngine(table, TorchDistTransport(), max_keys=300, dim=DIM, frag_num=64,
                       device="cpu")
        out = []
        for rnd in range(3):
            k = _keys_for(rank, rnd)
            r = eng.pull(torch.from_numpy(k))
            out.append((k, eng.gather(r).numpy().copy()))
            eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)))
            eng.push(r)
        q.put((rank, out, table.to_dict(with_state=True)))
    finally:
        dist.destroy_process_group()


def test_user_init_and_pull_methods_world2():
    """User access methods (the reference's PullAccessMethod::init_param and
    get_pull_value as tensor code) on the servers of a 2-rank job: every key
    is created with the user's rows, every pull returns the user's transform
    of the stored row, and the merged AdaGrad updates apply to those rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_access_rank, args=(r, 2, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = collect(q, procs, 2, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    state = {}
    for _, _, st in res:
        state.update(st)
    check_access_results(res, state)


def access_oracle(world=2, rounds=3):
    """rows after `rounds` merged AdaGrad rounds (lr 0.1) of every rank's
    keys from the user initialiser, and what each (rank, round) pulled"""
    rows, pulled = {}, {}
    for rnd in range(rounds):
        for r in range(world):
            k = _keys_for(r, rnd)
            for x in k.tolist():
                if x not in rows:
                    rows[x] = _init_rows(torch.tensor([x])).numpy()[0].astype(np.float64)
            pulled[(r, rnd)] = np.stack(
                [rows[x][:DIM] / np.sqrt(rows[x][DIM:]) for x in k.tolist()])
        acc = {}
        for r in range(world):
            k = _keys_for(r, rnd)
            for x, g in zip(k.tolist(), _grads_for(k, r, rnd).astype(np.float64)):
                acc[x] = acc.get(x, 0) + g
        for x, g in acc.items():
            rows[x][DIM:] += g * g
            rows[x][:DIM] -= 0.1 * g / np.sqrt(rows[x][DIM:] + 1e-8)
    return rows, pulled


def check_access_results(res, state, world=2):
    rows, pulled_ref = access_oracle(world)
    for rank, out, _ in res:
        for rnd, (k, vals) in enumerate(out):
            np.testing.assert_allclose(vals, pulled_ref[(rank, rnd)], rtol=1e-4, atol=1e-5)
    assert set(state) == set(rows)
    for x, row in rows.items():
        np.testing.assert_allclose(state[x], row, rtol=1e-4, atol=1e-5)


def test_compiled_const_init():
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    t = HostTable(2, 2, Optimizer("adagrad"), InitConfig("const", scale=0.25, state_init=0.1))
    v = t.pull_keys(np.array([3, 9], dtype=np.int64)).numpy()
    np.testing.assert_allclose(v, 0.25)
    np.testing.assert_allclose(t.to_dict(with_state=True)[3], [0.25, 0.25, 0.1, 0.1])
