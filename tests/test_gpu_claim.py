"""Region tables and claimed pulls (ss_device.h ProbeSeq, table.hip
k_pull_claim_bk / k_commit_claims, bdedup.hip region buckets and the
16-byte [w | h | key] merge store), against the CAS-insert path and host
references.  Run on MI355X: -m gpu."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

_GOLD = np.uint64(0x9E3779B97F4A7C15)


@pytest.fixture(scope="module")
def dev():
    from swiftsnails_amd._native import hip

    hip()  # loud failure if the extension is missing on a GPU box
    return torch.device("cuda", 0)


def _region_of(keys: np.ndarray, rbits: int) -> np.ndarray:
    from swiftsnails_amd.utils.hashing import fmix64

    k = keys.view(np.uint64) if keys.dtype == np.int64 else keys
    return (fmix64(k ^ _GOLD) >> np.uint64(64 - rbits)).astype(np.int64)


def _keys(n, seed=0, hi=1 << 40):
    rng = np.random.default_rng(seed)
    return np.unique(rng.integers(0, hi, size=n, dtype=np.int64))


def _rows_close(a, b):
    """Rows trained through different bucket layouts (region vs hash
    buckets) sum each key's gradient in a different float order: all but a
    handful of coordinates agree to 1e-4, every one to 1e-2."""
    close = np.isclose(a, b, rtol=1e-4, atol=1e-6)
    assert close.mean() > 0.9999, close.mean()
    np.testing.assert_allclose(a, b, rtol=1e-2, atol=1e-4)


def _lr_table(dev, cap=1 << 22, init="uniform", lr=0.1):
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable

    ic = InitConfig("uniform", 0.02, 0.1, seed=5) if init == "uniform" else \
        InitConfig("zero", state_init=0.1)
    return HbmTable(1, cap, optimizer=Optimizer("adagrad", lr=lr), init=ic, device=dev)


def test_region_table_layout_and_cas_probing(dev):
    """Scalar LR shards are split into 2^rbits regions (capacity rounded up to
    whole regions); CAS inserts, lookups and the export keep every key inside
    the region of its hash's top bits; the probe histogram still counts all."""
    t = _lr_table(dev, cap=3_000_000)
    assert t.rbits == 11 and t.capacity % (1 << t.rbits) == 0 and t.capacity >= 3_000_000
    assert t.dt.rbits == t.rbits and t.dt.rlen == t.capacity >> t.rbits
    k = _keys(200_000, 1)
    kt = torch.from_numpy(k).to(dev)
    v, s = t.pull(kt, unique=True)
    v2, s2 = t.pull(kt, insert=False)
    torch.cuda.synchronize()
    t.check()
    assert torch.equal(s, s2) and torch.equal(v, v2) and t.size() == len(k)
    sn = s.cpu().numpy()
    assert (sn >= 0).all() and len(np.unique(sn)) == len(k)
    np.testing.assert_array_equal(sn // t.dt.rlen, _region_of(k, t.rbits))
    assert int(t.probe_histogram(16).sum()) == len(k)
    d = t.to_dict()
    assert set(d) == set(int(x) for x in k.view(np.uint64))
    # tables that keep one region: other layouts, or SS_TABLE_REGIONS=0
    from swiftsnails_amd.ops.table import HbmTable

    assert HbmTable(3, 1 << 22, device=dev).rbits == 0
    assert _lr_table(dev, cap=1 << 12).rbits == 0


@pytest.mark.parametrize("init", ["uniform", "zero"])
def test_claim_pull_then_commit(dev, init):
    """The claimed pull returns the initial (w, h) of new keys and the stored
    row of old ones, writes nothing to the table, and every new key's slot is
    distinct, empty and inside its region; the commit then stores exactly
    those keys and rows (a CAS lookup finds them where the claim put them)."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.ops.optim import init_reference

    t = _lr_table(dev, init=init)
    old = _keys(30_000, 2)
    t.pull(torch.from_numpy(old).to(dev), unique=True)  # CAS-inserted, initial rows
    torch.cuda.synchronize()
    size0 = t.size()
    new = _keys(60_000, 3, hi=1 << 50)
    occ = np.concatenate([old[:20_000], new, new[:5000], old[:3000]])  # duplicates too
    np.random.default_rng(4).shuffle(occ)
    dd = Deduper(len(occ), device=dev)
    dd.rbits = t.rbits
    res = dd(torch.from_numpy(occ).to(dev))
    assert res.rbits == t.rbits  # region buckets at this call size
    bk, bs, un, ub, P = dd.bucket_view(len(occ))
    ucap = len(occ)
    slots = torch.full((ucap,), -7, dtype=torch.int32, device=dev)
    out = torch.zeros(ucap, device=dev)
    snap = torch.zeros((ucap, 2), device=dev)
    before = t.storage.clone()
    h = hip()
    h.pull_claim_bk(t.dt, bk, bs, un, ub, P, slots.data_ptr(), out.data_ptr(), snap.data_ptr(),
                    t._init_native, t.size_ctr.data_ptr(), t.err.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    t.check()
    assert torch.equal(before, t.storage)  # nothing written by the pull
    n = int(res.ucount[0].item())
    # unique keys in unique-id order: bucket b's keys at ubase[b] + l
    bkeys = dd.bkeys.cpu().numpy()
    ubase = dd.scratch.cpu().numpy()
    _, o_bs, o_un, o_ub = h.bd_offsets(len(occ), 1, 1)
    bstart = ubase[o_bs:o_bs + P + 1]
    unum, ub0 = ubase[o_un:o_un + P], ubase[o_ub:o_ub + P]
    uk = np.empty(n, dtype=np.int64)
    for b in range(P):
        uk[ub0[b]:ub0[b] + unum[b]] = bkeys[bstart[b]:bstart[b] + unum[b]]
    assert set(uk.tolist()) == set(np.unique(occ).tolist())
    sl = slots.cpu().numpy()[:n].astype(np.int64)
    assert (sl >= 0).all() and len(np.unique(sl)) == n
    np.testing.assert_array_equal(sl // t.dt.rlen, _region_of(uk, t.rbits))
    is_new = ~np.isin(uk, old)
    assert t.size() - size0 == int(is_new.sum())
    ref = init_reference(t.init_cfg, uk, 1, 2)
    np.testing.assert_array_equal(snap.cpu().numpy()[:n], ref[:, :2])  # old keys: initial rows
    np.testing.assert_array_equal(out.cpu().numpy()[:n], ref[:, 0])
    # the old keys' slots are where the CAS path put them
    s_old = t.pull(torch.from_numpy(uk[~is_new]).to(dev), insert=False)[1]
    np.testing.assert_array_equal(s_old.cpu().numpy(), sl[~is_new])
    keys_view = t.keys_view().cpu().numpy()
    assert (keys_view[sl[is_new]] == -1).all()  # claimed slots still EMPTY
    # the fused occurrence fill (the LR forward's one-gather mode): the same
    # pull again (it wrote nothing) with occ[p] = w(luid[p]) and no uvals
    occ_t = torch.full((len(occ),), -5.0, device=dev)
    snap2 = torch.zeros_like(snap)
    ctr2 = torch.zeros_like(t.size_ctr)  # its insert count goes elsewhere
    slots2 = torch.empty_like(slots)  # which lane wins an empty slot may differ per launch
    h.pull_claim_bk(t.dt, bk, bs, un, ub, P, slots2.data_ptr(), 0, snap2.data_ptr(),
                    t._init_native, ctr2.data_ptr(), t.err.data_ptr(),
                    torch.cuda.current_stream().cuda_stream, dd.luid.data_ptr(), occ_t.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(snap2, snap) and int(ctr2.sum()) == int(is_new.sum())
    luid = dd.luid.cpu().numpy().view(np.uint32)
    on = out.cpu().numpy()
    want = np.zeros(len(occ), dtype=np.float32)
    for b in range(P):
        p0, p1 = bstart[b], bstart[b + 1]
        want[p0:p1] = on[ub0[b] + luid[p0:p1].astype(np.int64)]
    np.testing.assert_array_equal(occ_t.cpu().numpy(), want)
    h.commit_claims(t.dt, bk, bs, un, ub, P, slots.data_ptr(), snap.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
    vals, s2 = t.pull(torch.from_numpy(uk).to(dev), insert=False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(s2.cpu().numpy(), sl)
    np.testing.assert_array_equal(vals.cpu().numpy()[:, 0], ref[:, 0])
    d = t.to_dict(with_state=True)
    assert len(d) == len(old) + int(is_new.sum())
    np.testing.assert_array_equal(d[int(uk[0])], ref[0, :2])


@pytest.mark.parametrize("init", ["uniform", "zero"])
def test_sparse_lr_claimed_matches_cas(dev, monkeypatch, init):
    """Sparse LR on the one-GPU path trains the same model with claimed pulls
    (LDS claims + 16-byte [w | h | key] merge stores) as with CAS inserts,
    step for step: same losses, same keys, same rows and AdaGrad state."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    out = {}
    for claim in ("1", "0"):
        monkeypatch.setenv("SS_CLAIM", claim)
        data = CtrSynth(batch_size=4096, num_fields=13, num_features=2_000_000, tail_frac=0.3)
        table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev,
                              capacity=1 << 22, init=lr_init(init, 0.01))
        assert table.rbits == 12
        eng = PSEngine(table, None, max_keys=4096 * 13, dim=1, device=dev)
        assert eng.claim == (claim == "1")
        w = SparseLRWorker(eng, data)
        losses, used = [], 0
        for _ in range(10):
            losses.append(float(w.step().sum().item()))
            used += eng._deferred_slot is not None
        torch.cuda.synchronize()
        eng.check()
        assert (used > 0) == (claim == "1") and not eng._claimed
        out[claim] = (losses, table.to_dict(with_state=True), table.size())
    (l1, t1, n1), (l0, t0, n0) = out["1"], out["0"]
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    assert n1 == n0 == len(t0) and t1.keys() == t0.keys()
    ks = list(t1.keys())
    _rows_close(np.stack([t1[k] for k in ks]), np.stack([t0[k] for k in ks]))


def test_interleaved_claimed_pulls(dev, monkeypatch):
    """pull A, pull B, push A, push B over overlapping NEW keys: B's pull
    first commits A's claims (else both would claim slots for the shared
    keys), and B's stale snapshot re-reads its rows — the same table as with
    CAS inserts."""
    from swiftsnails_amd.parallel.engine import PSEngine

    ka = torch.arange(1, 30001, dtype=torch.int64, device=dev) * 7919
    kb = torch.arange(15001, 45001, dtype=torch.int64, device=dev) * 7919
    res = {}
    for claim in ("1", "0"):
        monkeypatch.setenv("SS_CLAIM", claim)
        t = _lr_table(dev, lr=0.5)
        eng = PSEngine(t, None, max_keys=32768, dim=1, device=dev)
        eng.claim_rounds = True
        ra = eng.pull(ka)
        rb = eng.pull(kb)
        assert ra.slot32 and not ra.deferred  # A committed by B's pull
        assert rb.deferred == (claim == "1")
        eng.accumulate(ra, torch.ones(len(ka), 1, device=dev))
        eng.push(ra)
        eng.accumulate(rb, torch.full((len(kb), 1), 2.0, device=dev))
        eng.push(rb)
        rc = eng.pull(kb)
        assert rc.deferred == (claim == "1")
        eng.accumulate(rc, torch.ones(len(kb), 1, device=dev))
        eng.push(rc)  # not fused: committed, then the apply
        torch.cuda.synchronize()
        t.check()
        assert t.size() == 45000
        res[claim] = t.to_dict(with_state=True)
    assert res["1"].keys() == res["0"].keys()
    for k in res["0"]:
        np.testing.assert_array_equal(res["1"][k], res["0"][k])
    np.testing.assert_allclose(res["1"][20000 * 7919][1], 6.1, rtol=1e-6)


def test_sparse_lr_xgmi_path_claimed_matches_cas(dev, monkeypatch):
    """The N>1 engine path (a size-1 xGMI mailbox arena: keys + bucket runs
    in, the server's merge of the sources' keys, rows back, gradients, the
    server's fused merge) with claimed server pulls — the senders' buckets
    and the server's sub-buckets follow the shard's regions — trains the
    same model as with CAS inserts."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    out = {}
    for claim in ("1", "0"):
        monkeypatch.setenv("SS_CLAIM", claim)
        data = CtrSynth(batch_size=4096, num_fields=13, num_features=2_000_000, tail_frac=0.3)
        table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev,
                              capacity=1 << 22, init=lr_init("uniform", 0.01))
        tr = XgmiTransport(0, 1, dev, None, timeout_s=30)
        eng = PSEngine(table, tr, max_keys=4096 * 13, dim=1, device=dev)
        assert not eng.fast1 and eng.xg is not None
        assert eng.claim == (claim == "1") and eng.srv_rbits == (12 if claim == "1" else 0)
        w = SparseLRWorker(eng, data)
        losses, used = [], 0
        for _ in range(10):
            losses.append(float(w.step().sum().item()))
            used += eng._deferred_slot is not None
        torch.cuda.synchronize()
        eng.check()
        assert (used > 0) == (claim == "1")
        out[claim] = (losses, table.to_dict(with_state=True))
        tr.close()
    (l1, t1), (l0, t0) = out["1"], out["0"]
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    assert t1.keys() == t0.keys()
    ks = list(t1.keys())
    _rows_close(np.stack([t1[k] for k in ks]), np.stack([t0[k] for k in ks]))


def test_region_full_fails_loudly_without_silent_loss(dev, monkeypatch):
    """A region table driven towards full through the bench path (claimed
    pulls, region-aligned buckets, the fused [w | h | key] merge store): a
    key whose region has no empty slot left sets the sticky error, and the
    engine's check raises a region-full error at that step.  Until then no
    row is lost: after every step that passed its check the table holds
    exactly the distinct keys pulled so far.  The first region fills only
    near full load (keys probe only their own 1024-slot region)."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.table import TableFullError
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    # 1664 keys per call: <= 16 buckets, so each bucket gets >= 4 of the 64
    # regions (the region-bucket rule of launch_bd_dedup) and pulls claim
    B, F = 128, 13
    data = CtrSynth(batch_size=B, num_fields=F, num_features=50_000_000, tail_frac=1.0)
    table = make_lr_table(data.num_features, 1, load=0.5, device=dev, capacity=1 << 16,
                          init=lr_init("uniform", 0.01))
    assert table.rbits == 6 and table.capacity == 1 << 16  # 64 regions of 1024 slots
    eng = PSEngine(table, None, max_keys=B * F, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    assert eng.claim and all(d.rbits == table.rbits for d in eng.dedupers)
    k = torch.empty(B * F, dtype=torch.int64, device=dev)
    y = torch.empty(B, dtype=torch.float32, device=dev)
    seen = torch.empty(0, dtype=torch.int64, device=dev)
    err = None
    for step in range(100):
        w.step()
        torch.cuda.synchronize()
        assert eng._deferred_slot is not None  # the pull claimed (bench path)
        try:
            eng.check()
        except TableFullError as e:
            err = e
            break
        data.generate(step, 0, 1, k, y)
        seen = torch.unique(torch.cat([seen, k]))
        assert table.size() == seen.numel(), step  # no silent row loss
        keys = torch.cat([kk for kk, _ in table.export(to_host=False)])
        assert keys.numel() == seen.numel() and torch.equal(torch.sort(keys)[0], seen)
    assert err is not None, "the table never filled"
    assert "region" in str(err), str(err)
    # near full: the last clean step left the table above 85 % load
    assert seen.numel() >= 0.85 * table.capacity, seen.numel() / table.capacity


def test_region_buckets_fit_the_dedup_table_all_distinct(dev):
    """Region buckets hold whole regions, floor or ceil of R / Pd of them:
    with R / Pd just above 4 some buckets get 5 regions, 1.25x the target
    occurrences (~4480 at the one-rank 3584).  All-distinct keys would then
    overflow the dedup's 4096-slot LDS table — a run-ending error the hash
    buckets (~2 % size spread) never hit.  The dedup takes region buckets
    only when the fullest bucket fits with every key distinct, so this call
    falls back to hash buckets and dedups cleanly; the bench shape (R / Pd
    ~23) keeps its region buckets."""
    from swiftsnails_amd.ops.dedup import Deduper

    # 2^13 regions, ~1905 buckets of the 3584 target: R / Pd ~ 4.3
    n = 3584 * 1905
    k = torch.from_numpy(_keys(int(n * 1.05), 11)[:n]).to(dev)
    assert k.numel() == n
    d = Deduper(n, nranks=1, device=dev, mode="bucket")
    d.rbits = 13
    r = d(k)
    torch.cuda.synchronize()
    d.check()  # no overflow
    assert r.rbits == 0  # the layout declined region buckets
    assert int(r.ucount[0]) == n
    # the bench's call shape keeps them: 10.2M keys over 2^16 regions
    n2 = 262144 * 39
    k2 = torch.randint(0, 1 << 30, (n2,), dtype=torch.int64, device=dev)
    d2 = Deduper(n2, nranks=1, device=dev, mode="bucket")
    d2.rbits = 16
    r2 = d2(k2)
    torch.cuda.synchronize()
    d2.check()
    assert r2.rbits == 16
