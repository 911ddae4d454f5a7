"""PipelinedWorker.calibrate_exchange (bench.py's SS_XCHG=auto) on the CPU
engine over gloo, world 2: two candidate workers whose engines share one
table are timed in alternating windows; every rank must reach the same
choice (the timings are maxed over ranks), the table must end up with every
round of both workers applied (the windows quiesce between workers), and
SS_CAL_XCHG must force either outcome.  The candidates here are two
unique-key engines standing in for the GPU's unique / record pair (the
record exchange needs the xGMI mailboxes; its GPU form is
tests/test_gpu_xgmi_tiers.py::test_bench_world2_exchange_calibration)."""
import multiprocessing as mp

import numpy as np
import pytest
import torch
import torch.distributed as dist

from tests._mp import collect, file_init, init_gloo

DIM = 2


def _keys_for(rank: int, step: int) -> np.ndarray:
    rng = np.random.default_rng(1000 * step + rank)
    return rng.integers(0, 500, size=200).astype(np.int64)


def _run_rank(rank, world, init, pick, q):
    import os

    if pick:
        os.environ["SS_CAL_XCHG"] = pick
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.models.base import PipelinedWorker
        from swiftsnails_amd.ops.host_table import HostTable
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        table = HostTable(DIM, 4, Optimizer("sgd", lr=0.1), InitConfig("zero"))
        pushed = []

        def make(name):
            eng = PSEngine(table, TorchDistTransport(), max_keys=256, dim=DIM, frag_num=64,
                           device="cpu", depth=4)
            steps = {}

            class W(PipelinedWorker):
                def _produce(self, step, slot, stream):
                    steps[slot] = step
                    return torch.from_numpy(_keys_for(rank, step))

                def _compute(self, rnd, slot, st):
                    k = _keys_for(rank, steps[slot])
                    eng.accumulate(rnd, torch.ones((k.size, DIM), dtype=torch.float32))
                    pushed.append((name, steps[slot]))

                def samples_per_step(self):
                    return 200

            return W(eng, rank=rank, world=world)

        cands = {"unique": make("unique"), "records": make("records")}
        best, rep = PipelinedWorker.calibrate_exchange(cands, "unique", steps=2, windows=2)
        q.put((rank, best, rep, pushed, table.to_dict(with_state=False)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pick", ["", "records", "unique"])
def test_calibrate_exchange_gloo(pick):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_rank, args=(r, world, init, pick, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    bests = {r: b for r, b, *_ in res}
    assert bests[0] == bests[1], "ranks chose different exchanges"
    if pick:
        assert bests[0] == pick
    for _, best, rep, pushed, _ in res:
        assert rep["exchange"] == best and rep["default"] == "unique"
        assert len(rep["unique_ms"]) == len(rep["records_ms"]) == 2
        # 2 windows x (2 settle + 2 timed) steps per candidate, in window order
        assert [n for n, _ in pushed] == (["unique"] * 4 + ["records"] * 4) * 2
        assert [s for n, s in pushed if n == "unique"] == list(range(8))
    # every round of both candidates landed in the shared table: with SGD
    # (lr 0.1, all-ones gradients) a key's row is -0.1 x its occurrences
    counts = {}
    for r in range(world):
        for cand in range(2):
            for s in range(8):
                for k in _keys_for(r, s):
                    counts[int(k)] = counts.get(int(k), 0) + 1
    rows = {}
    for *_, tab in res:
        assert not (set(tab) & set(rows))  # disjoint shards
        rows.update(tab)
    assert set(rows) == set(counts)
    for k, c in counts.items():
        np.testing.assert_allclose(rows[k], np.full(DIM, -0.1 * c, np.float32), rtol=1e-5)
