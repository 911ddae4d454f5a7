"""Pull-ahead (bounded staleness) pipeline switched on and off mid-run
(PipelinedWorker.set_pull_ahead / drain), on the CPU engine with gloo ranks.

The CPU engine runs every collective in host order, so the pulled-ahead
schedule is exact: round j+L is pulled before round j is pushed.  The test
records the global order of pull / push events and replays it on a single
HostTable oracle: pulled rows must match the oracle under that schedule, and
the final state must equal the synchronous oracle's (gradients here do not
depend on the pulled rows, the init is key-seeded, and pushes stay in round
order — switching modes must not lose, repeat or reorder an update)."""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo
from test_engine_cpu import DIM, _grads_for, _keys_for

STEPS = 16
# (step at which to switch, mode): sync 0-2, ahead 3-7, off (drains L), ahead 11-13, off
SWITCH = {3: True, 8: False, 11: True, 14: False}


def _oracle_schedule(workers, events):
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    t = HostTable(DIM, 4, Optimizer("adagrad", lr=0.1), InitConfig("uniform", 0.2, 0.01))
    pulled = {}
    for kind, rnd in events:
        if kind == "pull":
            for r in workers:
                pulled[(r, rnd)] = t.pull_keys(_keys_for(r, rnd)).numpy()
            continue
        ks = [_keys_for(r, rnd) for r in workers]
        gs = [_grads_for(k, r, rnd) for k, r in zip(ks, workers)]
        u, inv = np.unique(np.concatenate(ks), return_inverse=True)
        m = np.zeros((len(u), DIM), np.float64)
        np.add.at(m, inv, np.concatenate(gs).astype(np.float64))
        t.push_keys(u, m.astype(np.float32))
        t.next_round()
    return t.to_dict(with_state=True), pulled


def _run_rank(rank, world, init, staleness, q):
    import os

    os.environ["SS_STALENESS"] = str(staleness)
    os.environ["SS_PULL_AHEAD"] = "auto"
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.models.base import PipelinedWorker
        from swiftsnails_amd.ops.host_table import HostTable
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        table = HostTable(DIM, 4, Optimizer("adagrad", lr=0.1), InitConfig("uniform", 0.2, 0.01))
        eng = PSEngine(table, TorchDistTransport(), max_keys=300, dim=DIM, frag_num=64,
                       device="cpu", depth=4)
        assert not eng.pull_ahead and eng.lookahead == staleness
        events, pulled, slot_step = [], {}, {}

        class W(PipelinedWorker):
            def _produce(self, step, slot, stream):
                slot_step[slot] = step
                return torch.from_numpy(_keys_for(rank, step))

            def _compute(self, rnd, slot, st):
                step = slot_step[slot]
                pulled[(rank, step)] = eng.gather(rnd).numpy().copy()
                k = _keys_for(rank, step)
                eng.accumulate(rnd, torch.from_numpy(_grads_for(k, rank, step)))

            def samples_per_step(self):
                return 257

        pull_stage, push = eng._pull_stage, eng.push

        def pull_logged(r, uv, st, ahead):
            events.append(("pull", slot_step[r.slot]))
            return pull_stage(r, uv, st, ahead)

        def push_logged(rnd, grads=None):
            events.append(("push", slot_step[rnd.slot]))
            return push(rnd, grads)

        eng._pull_stage, eng.push = pull_logged, push_logged
        w = W(eng, rank=rank, world=world)
        modes = []
        for i in range(STEPS):
            if i in SWITCH:
                w.set_pull_ahead(SWITCH[i])
            modes.append(bool(eng.pull_ahead))
            w.step()
        w.drain()
        q.put((rank, events, pulled, table.to_dict(with_state=True), modes, w.step_idx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("staleness", [1, 2])
def test_pull_ahead_switches_mid_run_gloo(staleness):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_rank, args=(r, world, init, staleness, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    evs = {r: e for r, e, *_ in res}
    assert evs[0] == evs[1], "ranks issued different collective orders"
    events = evs[0]
    steps = res[0][5]
    assert steps >= STEPS
    pushes = [j for k, j in events if k == "push"]
    assert pushes == list(range(steps)), pushes      # every round pushed once, in order
    pulls = [j for k, j in events if k == "pull"]
    assert sorted(pulls) == list(range(steps))       # every round pulled once
    # the schedule really pulled ahead: some round was pulled `staleness`
    # pushes before its own push, never more
    lag = {j: sum(1 for k, i in events[:events.index(("pull", j))] if k == "push")
           for j in pulls}
    assert max(j - lag[j] for j in pulls) == staleness
    assert min(j - lag[j] for j in pulls) == 0       # ... and some synchronously
    state, pulled = {}, {}
    for _, _, pl, st, modes, _ in res:
        assert not (set(st) & set(state))
        state.update(st)
        pulled.update(pl)
    ref_state, ref_pulled = _oracle_schedule([0, 1], events)
    sync_state, _ = _oracle_schedule([0, 1], [(k, j) for j in range(steps)
                                              for k in ("pull", "push")])
    assert set(state) == set(ref_state) == set(sync_state)
    for k in ref_state:
        np.testing.assert_allclose(state[k], ref_state[k], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(state[k], sync_state[k], rtol=2e-5, atol=2e-6)
    assert set(pulled) == set(ref_pulled)
    for key, v in ref_pulled.items():
        np.testing.assert_allclose(pulled[key], v, rtol=2e-5, atol=2e-6)


def test_graph_declined_with_more_than_four_ranks_per_gpu(monkeypatch):
    """enable_graph() keeps eager rounds when more than 4 ranks of an xGMI
    job share one GPU (replays ran every round at ~21 ms there,
    profiles/raw/r6_config3_split_roles.txt); SS_GRAPH=force overrides; ranks
    on devices of their own are not affected."""
    from types import SimpleNamespace

    from swiftsnails_amd.models.base import PipelinedWorker

    def worker(world, devices):
        eng = SimpleNamespace(gpu=True, fast1=False, xg=SimpleNamespace(devices=devices),
                              world=world, table=None, shared_device=devices < world)
        w = object.__new__(PipelinedWorker)
        w.engine, w.quota = eng, None
        w.data = SimpleNamespace(graph_capturable=True)
        w._graphs = ["captured"]  # past the guard, enable_graph returns True here
        return w

    monkeypatch.delenv("SS_GRAPH", raising=False)
    assert not worker(8, 1).enable_graph()
    assert not worker(5, 1).enable_graph()
    assert worker(4, 1).enable_graph()
    assert worker(8, 8).enable_graph()
    assert worker(8, 2).enable_graph()  # 4 ranks per device
    monkeypatch.setenv("SS_GRAPH", "force")
    assert worker(8, 1).enable_graph()
