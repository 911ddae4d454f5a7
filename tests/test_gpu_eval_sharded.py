"""Sharded evaluation and N>1 training quality (xGMI ranks on one GPU).

Sparse LR trained on the same samples at world 1, 2 and 4 — per-rank batch
B / N, so every round covers exactly world 1's batch (the generator gives
rank r of N the samples [(step*N + r) * B/N, ...)) — then evaluated on the
same held-out samples through the collective read-only pull
(PSEngine.lookup: every shard answers, nothing is inserted).  The servers'
merged push (one AdaGrad step on the sum of the workers' gradients per key)
makes a round at world N the same update as world 1's step, so with
synchronous rounds the held-out AUC must agree within 0.005.  With
pulled-ahead rounds (bounded staleness 1 or 2: what the start-up calibration
may pick on a multi-GPU node) a round misses up to that many rounds' updates;
the held-out AUC must stay within 0.01 of world 1.  At N > 1 the evaluation's
read-only pull runs on the device (the xGMI round on the slot past the ring,
PSEngine._lookup_xgmi), and it leaves every table's size unchanged."""
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
    eng = PSEngine(table, transport, max_keys=(B // world) * F, dim=1, device=dev,
                   exchange=os.environ.get("SS_TEST_XCHG", "unique"))
    assert eng.records == (world > 1 and os.environ.get("SS_TEST_XCHG") == "records")
    w = SparseLRWorker(eng, data, rank=rank, world=world)
    for _ in range(STEPS):
        w.step()
    torch.cuda.synchronize()
    eng.check()
    before = table.size()
    ev = w.evaluate(batches=2)
    assert table.size() == before  # read-only: nothing inserted
    if world > 1:  # the device lookup ran, not the gloo fallback
        assert eng.metrics.counters.get("lookup_keys", 0) == 2 * (B // world) * F
    ev["pull_ahead"] = bool(eng.pull_ahead)
    # the shard's rows, and the rounds whose keys were pulled (inserted): the
    # trained steps plus the rounds pulled ahead past the last one
    keys, rows = _export(table)
    return ev, before, keys, rows, w.step_idx + len(w._pulled)


def _export(table):
    ks, rs = [], []
    for k, r in table.export():
        ks.append(k.numpy())
        rs.append(r.numpy())
    keys = np.concatenate(ks) if ks else np.zeros(0, np.int64)
    rows = np.concatenate(rs) if rs else np.zeros((0, 2), np.float32)
    return keys, rows


def _keys_of_rounds(world, rounds):
    """Every distinct key the ranks of a world-``world`` job pull in rounds
    0 .. rounds-1 (regenerated with the same device generator)."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth

    dev = torch.device("cuda", 0)
    data = CtrSynth(batch_size=B // world, num_fields=F, num_features=FEATS, tail_frac=0.05)
    k = torch.empty((B // world) * F, dtype=torch.int64, device=dev)
    y = torch.empty(B // world, dtype=torch.float32, device=dev)
    out = []
    for s in range(rounds):
        for r in range(world):
            data.generate(s, r, world, k, y)
            out.append(torch.unique(k))
    return torch.unique(torch.cat(out)).cpu().numpy()


def _rank(rank, world, init, q, env):
    os.environ.update(env)
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.parallel.transport import TorchDistTransport
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        tr = XgmiTransport(rank, world, dev, dist.distributed_c10d._get_default_store(),
                           aux=TorchDistTransport(), timeout_s=60)
        ev, n, keys, rows, pulled = _train_eval(rank, world, dev, tr)
        q.put((rank, ev, n, keys, rows, pulled))
    finally:
        dist.destroy_process_group()


def _world(world, env):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_rank, args=(r, world, init, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    evs = [x[1] for x in res]
    for ev in evs[1:]:  # every rank reports the same global metrics
        assert ev == evs[0]
    pulled = {x[5] for x in res}
    assert len(pulled) == 1, pulled  # every rank pulled the same rounds
    shards = [(x[3], x[4]) for x in sorted(res, key=lambda x: x[0])]
    return evs[0], sum(x[2] for x in res), shards, pulled.pop()


_REF = {}


def _ref():
    """World 1 (the one-GPU path, synchronous), trained once per session."""
    from swiftsnails_amd.parallel.transport import LoopbackTransport

    if not _REF:
        old = os.environ.get("SS_PULL_AHEAD")
        os.environ["SS_PULL_AHEAD"] = "0"
        try:
            _REF["ref"] = _train_eval(0, 1, torch.device("cuda", 0), LoopbackTransport())
        finally:
            if old is None:
                del os.environ["SS_PULL_AHEAD"]
            else:
                os.environ["SS_PULL_AHEAD"] = old
    return _REF["ref"]


@pytest.mark.parametrize("mode,env,bound", [
    ("sync", {"SS_PULL_AHEAD": "0"}, 0.005),
    ("staleness1", {"SS_PULL_AHEAD": "1", "SS_STALENESS": "1"}, 0.01),
    ("staleness2", {"SS_PULL_AHEAD": "1", "SS_STALENESS": "2"}, 0.01),
    # the record exchange (every occurrence shipped, servers dedup + merge)
    ("sync", {"SS_PULL_AHEAD": "0", "SS_TEST_XCHG": "records"}, 0.005),
    ("staleness2", {"SS_PULL_AHEAD": "1", "SS_STALENESS": "2", "SS_TEST_XCHG": "records"},
     0.01),
    # grouped records: 3 server sub-buckets forced at this small shape, so
    # every source bucket's records are grouped by them after the scatter
    # (bdedup.hip k_rec_group) and the servers read exact ranges
    ("sync", {"SS_PULL_AHEAD": "0", "SS_TEST_XCHG": "records", "SS_REC_GROUP": "1",
              "SS_SRV_SUB": "3"}, 0.005),
])
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_eval_matches_world1(world, mode, env, bound):
    ref, n1, *ref_rows, _ = _ref()
    assert ref["auc"] > 0.6 and ref["samples"] == 2 * B
    ev, n, shards, pulled = _world(world, env)
    assert ev["samples"] == 2 * B
    assert ev["pull_ahead"] == (mode != "sync")
    # every exported key is unique within its shard and across shards (a
    # duplicate claim — two pulls claiming slots for one new key before a
    # commit — would store it twice), and the shards together hold exactly the
    # distinct keys of the rounds pulled: the trained steps, plus with
    # pulled-ahead rounds the ones pulled past the last step
    keys = np.concatenate([k for k, _ in shards])
    rows = np.concatenate([r for _, r in shards])
    assert len(np.unique(keys)) == len(keys) == n
    want = _keys_of_rounds(world, pulled)
    assert pulled == STEPS if mode == "sync" else pulled > STEPS
    assert np.array_equal(np.sort(keys), want)
    if mode == "sync":
        # synchronous world N is the same update as world 1 (one AdaGrad step
        # per key on the sum of every source's gradient): the rows agree up
        # to float summation order
        assert n == n1
        rk, rr = ref_rows
        oa, ob = np.argsort(rk), np.argsort(keys)
        assert np.array_equal(rk[oa], keys[ob])
        a, b = rr[oa], rows[ob]
        np.testing.assert_allclose(b[:, 1], a[:, 1], rtol=1e-4, atol=1e-7)  # AdaGrad sums
        # a weight whose summed gradient is ~0 can take its first AdaGrad
        # step (+-lr) with either sign depending on the summation order
        assert np.isclose(b[:, 0], a[:, 0], rtol=1e-4, atol=1e-6).mean() >= 0.9995
        np.testing.assert_allclose(b[:, 0], a[:, 0], rtol=0, atol=2 * 0.05 * STEPS)
    assert abs(ev["auc"] - ref["auc"]) < bound, (world, mode, ev, ref)
    assert abs(ev["auc_truth"] - ref["auc_truth"]) < 1e-9
