"""An independent fp32 oracle for the headline training path.

``bench.py`` trains sparse LR through the one-GPU engine's fastest path:
region tables, region-aligned dedup buckets, new keys' slots claimed in LDS
(no CAS), 4-byte slot indices, the occurrence fill fused into the claimed
pull, and the gradient merge with the AdaGrad update fused into it, storing
whole 16-byte ``[w | h | key]`` slots.  Every other test of that path
compares it with another path of this repository (claimed vs CAS, fused vs
separate apply); a bug they share would pass them all.  Here the reference is
plain PyTorch fp32 with nothing from the engine:

    z_s = sum_f w[key_sf]              (binary features)
    g_s = sigmoid(z_s) - y_s,          loss_s = softplus-form log loss
    G_k = sum of g_s over the occurrences of key k
    h_k += G_k^2,  w_k -= lr * G_k / sqrt(h_k + eps)

with new keys initialised by ``init_reference`` (the host mirror of the
key-seeded uniform init) and the keys / labels from the same synthetic
generator.  The engine's per-step losses and every key's final (w, h) must
match.  At world 2 and 4 (xGMI ranks on one GPU, synchronous rounds) a round
is one AdaGrad step per key on the sum of every rank's gradients — the world-1
update of the union batch — so the same oracle applies to the merged shards
(reference semantics: lookup-or-init then in-place apply,
/root/reference/src/core/parameter/sparsetable.h:142-149,181-192).
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo

pytestmark = pytest.mark.gpu

F, FEATS, STEPS, LR, SCALE = 39, 100_000_000, 10, 0.05, 0.01


class TorchLROracle:
    """Sparse LR + AdaGrad over a sorted key set, fp32, pure PyTorch."""

    def __init__(self, dev, init, lr=LR, eps=1e-8):
        self.dev, self.init, self.lr, self.eps = dev, init, lr, eps
        self.keys = torch.empty(0, dtype=torch.int64, device=dev)
        self.w = torch.empty(0, dtype=torch.float32, device=dev)
        self.h = torch.empty(0, dtype=torch.float32, device=dev)

    def _insert(self, u):
        """Positions of the sorted unique keys ``u`` in the key set, new keys
        inserted with their initial (w, h)."""
        from swiftsnails_amd.ops.optim import init_reference

        n = self.keys.numel()
        pos = torch.searchsorted(self.keys, u)
        hit = pos < n
        hit[hit.clone()] = self.keys[pos[hit]] == u[hit]
        new = u[~hit]
        if new.numel():
            r = init_reference(self.init, new.cpu().numpy(), 1, 2)
            keys = torch.cat([self.keys, new])
            w = torch.cat([self.w, torch.from_numpy(r[:, 0]).to(self.dev)])
            h = torch.cat([self.h, torch.from_numpy(r[:, 1]).to(self.dev)])
            order = torch.argsort(keys)
            self.keys, self.w, self.h = keys[order], w[order], h[order]
            pos = torch.searchsorted(self.keys, u)
        return pos

    def step(self, keys, labels):
        """One synchronous round over ``keys`` [B*F] / ``labels`` [B];
        returns the per-sample losses."""
        B = labels.numel()
        u, inv = torch.unique(keys, return_inverse=True)
        pos = self._insert(u)
        wu = self.w[pos]
        z = wu[inv].view(B, -1).sum(1)
        y = labels.float()
        g = torch.sigmoid(z) - y
        loss = torch.clamp(z, min=0) + torch.log1p(torch.exp(-z.abs())) - y * z
        G = torch.zeros_like(wu).index_add_(0, inv, g.repeat_interleave(keys.numel() // B))
        h = self.h[pos] + G * G
        self.h[pos] = h
        self.w[pos] = wu - self.lr * G / torch.sqrt(h + self.eps)
        return loss


def _batches(B, world, steps, dev):
    """(keys, labels) of every rank and step from the synthetic generator."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth

    data = CtrSynth(batch_size=B, num_fields=F, num_features=FEATS, tail_frac=0.1)
    out = []
    for s in range(steps):
        ks, ys = [], []
        for r in range(world):
            k = torch.empty(B * F, dtype=torch.int64, device=dev)
            y = torch.empty(B, dtype=torch.float32, device=dev)
            data.generate(s, r, world, k, y)
            ks.append(k)
            ys.append(y)
        out.append((ks, ys))
    return out


def _oracle(B, world, dev):
    """Per step, per rank mean losses and the final (keys, w, h) (sorted)."""
    from swiftsnails_amd.models.sparse_lr import lr_init

    orc = TorchLROracle(dev, lr_init("uniform", SCALE))
    losses = []
    for ks, ys in _batches(B, world, STEPS, dev):
        loss = orc.step(torch.cat(ks), torch.cat(ys))
        losses.append([float(x) for x in loss.view(world, B).mean(1).cpu()])
    return np.array(losses), orc.keys.cpu().numpy(), orc.w.cpu().numpy(), orc.h.cpu().numpy()


def _export(table):
    ks, rs = [], []
    for k, r in table.export():
        ks.append(k.numpy())
        rs.append(r.numpy())
    return np.concatenate(ks), np.concatenate(rs)


def _bench_path_worker(B, world, rank, dev, transport=None):
    """The bench.py configuration at a test shape: same table, engine and
    worker construction (bench.py main)."""
    from swiftsnails_amd.models.sparse_lr import (CtrSynth, SparseLRWorker, lr_init,
                                                  make_lr_table)
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    data = CtrSynth(batch_size=B, num_fields=F, num_features=FEATS, tail_frac=0.1)
    table = make_lr_table(FEATS, world, optimizer=Optimizer("adagrad", lr=LR), load=0.5,
                          device=dev, init=lr_init("uniform", SCALE))
    eng = PSEngine(table, transport, max_keys=B * F, dim=1, device=dev)
    w = SparseLRWorker(eng, data, rank=rank, world=world)
    return w, table, eng


def _compare(keys, rows, okeys, ow, oh):
    order = np.argsort(keys)
    keys, rows = keys[order], rows[order]
    assert len(np.unique(keys)) == len(keys)  # one slot per key
    assert np.array_equal(keys, okeys), (len(keys), len(okeys))
    # AdaGrad sums: sums of squared per-round gradients.  A key's gradient is
    # a sum of (p - y) terms of both signs: where they nearly cancel, its
    # float summation order moves it relatively more (seen: 1 in 10^4 sums
    # off by up to 6e-4 relative), so nearly every sum tight, all close
    hc = np.isclose(rows[:, 1], oh, rtol=1e-4, atol=1e-7)
    assert hc.mean() >= 0.999, hc.mean()
    np.testing.assert_allclose(rows[:, 1], oh, rtol=3e-3, atol=1e-6)
    # weights: a key whose summed gradient is ~0 may take its first AdaGrad
    # step (+-lr) with either sign depending on the summation order, so
    # nearly every weight tight and every weight within that excursion
    close = np.isclose(rows[:, 0], ow, rtol=1e-4, atol=1e-6)
    assert close.mean() >= 0.9995, (close.mean(), np.abs(rows[:, 0] - ow).max())
    np.testing.assert_allclose(rows[:, 0], ow, rtol=0, atol=2 * LR * STEPS)


def test_bench_path_matches_fp32_oracle_world1(monkeypatch):
    """10 steps of the bench path at 65536 x 39 over 1e8 features (region
    tables with 2^16 regions, ~90 regions per dedup bucket) against the
    PyTorch fp32 oracle: every step's loss and every key's (w, h)."""
    for k in ("SS_CLAIM", "SS_SLOT32", "SS_TABLE_REGIONS", "SS_ENGINE_GENERAL", "SS_DEDUP"):
        monkeypatch.delenv(k, raising=False)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = 65536
    w, table, eng = _bench_path_worker(B, 1, 0, dev)
    # the headline path is what runs (not a fallback)
    assert eng.fast1 and eng.slot32 and eng.claim and eng.claim_rounds
    assert eng.claim_occ is w.occ and w.bucketed
    assert table.rbits == 16 and all(d.rbits == table.rbits for d in eng.dedupers)
    losses = []
    for _ in range(STEPS):
        w.step()
        losses.append(w.mean_loss())
    torch.cuda.synchronize()
    eng.check()
    ol, okeys, ow, oh = _oracle(B, 1, dev)
    np.testing.assert_allclose(losses, ol[:, 0], rtol=1e-4)
    assert losses[-1] < losses[0]
    keys, rows = _export(table)
    _compare(keys, rows, okeys, ow, oh)


def _xgmi_rank(rank, world, B, init, q):
    os.environ["SS_PULL_AHEAD"] = "0"
    os.environ["SS_XGMI_TIMEOUT"] = "60"
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.parallel.transport import TorchDistTransport
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        tr = XgmiTransport(rank, world, dev, dist.distributed_c10d._get_default_store(),
                           aux=TorchDistTransport(), timeout_s=60)
        w, table, eng = _bench_path_worker(B, world, rank, dev, tr)
        lay = eng.layout_info()
        losses = []
        for _ in range(STEPS):
            w.step()
            losses.append(w.mean_loss())
        torch.cuda.synchronize()
        eng.check()
        keys, rows = _export(table)
        q.put((rank, losses, keys, rows, lay, bool(eng.pull_ahead)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_path_matches_fp32_oracle_xgmi(world):
    """The N>1 bench path (xGMI mailboxes, server merge of every source's
    keys, claimed server inserts, the fused server merge + AdaGrad) at world
    2 and 4 against the same oracle over the union of the ranks' batches:
    each rank's per-step loss and the merged shards' (w, h)."""
    B = 16384
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_xgmi_rank, args=(r, world, B, init, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    for _, _, _, _, lay, ahead in res:
        assert lay["claim"] and lay["srv_rbits"] > 0 and not ahead
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ol, okeys, ow, oh = _oracle(B, world, dev)
    for rank, losses, *_ in res:
        np.testing.assert_allclose(losses, ol[:, rank], rtol=1e-4)
    keys = np.concatenate([x[2] for x in res])
    rows = np.concatenate([x[3] for x in res])
    _compare(keys, rows, okeys, ow, oh)
