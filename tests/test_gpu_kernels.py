"""HIP kernel numerics vs fp32 host references (run on MI355X: -m gpu)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from swiftsnails_amd._native import hip

    hip()  # loud failure if the extension is missing on a GPU box
    return torch.device("cuda", 0)


def _keys(n, seed=0, hi=1 << 40):
    rng = np.random.default_rng(seed)
    return rng.integers(0, hi, size=n, dtype=np.int64)


def test_table_pull_inits_and_is_stable(dev):
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, init_reference
    from swiftsnails_amd.ops.table import HbmTable

    init = InitConfig("uniform", scale=0.25, state_init=0.1, seed=7)
    t = HbmTable(8, 4096, optimizer=Optimizer("adagrad"), init=init, device=dev)
    k = np.unique(_keys(1000, 1))
    kt = torch.from_numpy(k).to(dev)
    v1, s1 = t.pull(kt)
    v2, s2 = t.pull(kt)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == len(k)
    ref = init_reference(init, k, 8, t.width)
    np.testing.assert_array_equal(v1.cpu().numpy(), ref[:, :8])
    np.testing.assert_array_equal(v2.cpu().numpy(), v1.cpu().numpy())
    assert torch.equal(s1, s2)
    d = t.to_dict(with_state=True)
    row = d[int(k[3])]
    np.testing.assert_allclose(row[8:], 0.1)


@pytest.mark.parametrize("G", [1, 4, 16, 64])
def test_probe_duplicates_same_slot(dev, G):
    from swiftsnails_amd.ops.table import HbmTable

    t = HbmTable(4, 1 << 12, device=dev, lane_group=G)
    base = _keys(300, 2)
    k = np.concatenate([base, base[::-1], base[:50]])
    kt = torch.from_numpy(k).to(dev)
    v, s = t.pull(kt, unique=False)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == len(np.unique(base))
    sn = s.cpu().numpy()
    for key in np.unique(base)[:50]:
        idx = np.nonzero(k == key)[0]
        assert len(set(sn[idx].tolist())) == 1


@pytest.mark.parametrize("G,dim", [(1, 1), (4, 8), (16, 16), (64, 33)])
def test_pull_duplicates_see_initialised_rows(dev, G, dim):
    """Non-unique fused pull (the N>1 server side gets a key from several
    workers): every occurrence of a key created in this launch must read the
    initial row, never the 0xFF fill of the empty slot."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, init_reference
    from swiftsnails_amd.ops.table import HbmTable

    init = InitConfig("uniform", scale=0.5, seed=11)
    t = HbmTable(dim, 1 << 15, optimizer=Optimizer("adagrad"), init=init, device=dev,
                 lane_group=G)
    base = np.unique(_keys(4000, 5))
    rng = np.random.default_rng(3)
    # every key 1-8 times, shuffled: duplicates land in the same wavefront
    k = np.repeat(base, rng.integers(1, 9, size=len(base)))
    rng.shuffle(k)
    old = base[:500]  # a third of the keys exist before the launch
    t.pull(torch.from_numpy(old).to(dev), unique=True)
    v, s = t.pull(torch.from_numpy(k).to(dev), unique=False)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == len(base)
    ref = init_reference(init, k, dim, t.width)[:, :dim]
    np.testing.assert_array_equal(v.cpu().numpy(), ref)
    sn = s.cpu().numpy()
    first = {}
    for key, sl in zip(k.tolist(), sn.tolist()):
        assert first.setdefault(key, sl) == sl


@pytest.mark.parametrize("cap", [1 << 14, 4200])
@pytest.mark.parametrize("dim", [9, 32, 64, 128])
@pytest.mark.parametrize("init_kind", ["uniform", "zero"])
def test_pull_wide_rows_from_buckets(dev, dim, init_kind, cap):
    """Bucketed unique pull of wide fp32 rows (k_pull_rows_bk: 8 lanes per
    key, 16-byte row vectors; the rows start 16-byte aligned in the slot) and
    of FM's narrow rows (dim 9, k_pull_narrow_bk: key + parameters read by
    the probe's own 16-byte loads): new keys read their initial row, existing
    keys their stored row, slots agree with a probe, and partial last lane
    groups of a bucket are inert.  Capacity 4200 for 3001 keys: long probe
    runs (keys away from their home slot, where the row read beside the
    first key load must be repeated)."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, init_reference
    from swiftsnails_amd.ops.table import HbmTable

    init = InitConfig(init_kind, scale=0.5, seed=7)
    t = HbmTable(dim, cap, optimizer=Optimizer("adagrad", lr=0.2), init=init, device=dev)
    assert t.stride % 16 == 0 and (t.row_off % 16 == 0 or 8 + 4 * dim <= 64)
    k = np.unique(_keys(3001, 9))
    kt = torch.from_numpy(k).to(dev)
    old = kt[::3].contiguous()
    t.pull(old, unique=True)
    g = torch.randn((old.numel(), dim), device=dev)
    t.push(old, g)  # the existing rows differ from their initial value
    torch.cuda.synchronize()
    before = t.to_dict(with_state=True)
    # buckets of uneven sizes (1 .. 70 keys: partial 8-lane groups and rounds)
    sizes, n = [], len(k)
    rng = np.random.default_rng(5)
    while sum(sizes) < n:
        sizes.append(int(min(rng.integers(1, 71), n - sum(sizes))))
    bstart = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    bs = torch.from_numpy(bstart).to(dev)
    un = torch.from_numpy(np.asarray(sizes, np.int32)).to(dev)
    out = torch.full((n, dim), float("nan"), device=dev)
    slots = torch.empty(n, dtype=torch.int64, device=dev)
    t.pull_buckets((kt.data_ptr(), bs.data_ptr(), un.data_ptr(), bs.data_ptr(), len(sizes)),
                   out, slots)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == n
    ref = init_reference(init, k, dim, t.width)[:, :dim]
    for i in range(0, n, 3):
        ref[i] = before[int(k.view(np.uint64)[i])][:dim]
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(slots.cpu().numpy(), t.lookup_slots(kt).cpu().numpy())


@pytest.mark.parametrize("kind", ["sgd", "adagrad", "ftrl", "adam"])
@pytest.mark.parametrize("dim", [1, 5, 8, 9, 33, 32, 128])
def test_apply_matches_reference(dev, kind, dim):
    """K5 per optimizer vs the NumPy reference; dims 5-9 with state take the
    LDS-staged 8-byte-chunk form (k_apply_st), 32 / 128 the 16-byte-vector
    form (k_apply_rows), 1 and 33 the others."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, apply_reference
    from swiftsnails_amd.ops.table import HbmTable

    opt = Optimizer(kind, lr=0.1, l1=0.01, l2=0.001, grad_scale=0.5, clip=5.0)
    opt.step = 1
    t = HbmTable(dim, 4096, optimizer=opt, init=InitConfig("uniform", 0.5, 0.05), device=dev)
    k = np.unique(_keys(700, 3))
    kt = torch.from_numpy(k).to(dev)
    t.pull(kt)
    before = t.to_dict(with_state=True)
    rows0 = np.stack([before[int(x)] for x in k.view(np.uint64)])
    g = np.random.default_rng(4).standard_normal((len(k), dim)).astype(np.float32)
    t.push(kt, torch.from_numpy(g).to(dev))
    torch.cuda.synchronize()
    after = t.to_dict(with_state=True)
    rows1 = np.stack([after[int(x)] for x in k.view(np.uint64)])
    ref = apply_reference(opt, rows0, g, dim)
    np.testing.assert_allclose(rows1, ref, rtol=2e-5, atol=2e-6)


def test_export_assign_resize_roundtrip(dev):
    from swiftsnails_amd.ops.optim import InitConfig
    from swiftsnails_amd.ops.table import HbmTable

    t = HbmTable(3, 1000, init=InitConfig("normal", 0.1), device=dev)
    k = np.unique(_keys(600, 5))
    t.pull(torch.from_numpy(k).to(dev))
    d0 = t.to_dict(with_state=True)
    t.resize(5000)
    assert t.capacity == 5000 and t.size() == len(k)
    d1 = t.to_dict(with_state=True)
    assert d0.keys() == d1.keys()
    for kk in d0:
        np.testing.assert_array_equal(d0[kk], d1[kk])


def test_table_full_raises(dev):
    from swiftsnails_amd.ops.table import HbmTable, TableFullError

    t = HbmTable(1, 64, device=dev)
    t.pull(torch.from_numpy(_keys(100, 6)).to(dev))
    torch.cuda.synchronize()
    with pytest.raises(TableFullError):
        t.check()


@pytest.mark.parametrize("servers", [[0], [0, 2]])
def test_bucket_dedup_split_roles_unique_heavy(dev, servers):
    """split roles (1 or 2 servers in 4 ranks) with all-unique
    keys.  Buckets were sized for 4 destinations, so each receiving
    destination's buckets got 4x (2x) the occurrences and overflowed the
    4096-slot LDS table, dropping keys silently; now sized by the effective
    destination count, no overflow and every key gets its id."""
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.parallel.router import HashFrag

    n, nranks = 1 << 21, 4
    fm = HashFrag(len(servers), 1024).rank_map(servers)
    d = Deduper(n, nranks=nranks, frag_map=torch.from_numpy(fm.astype(np.int32)), device=dev,
                mode="bucket")
    assert d.ndest == len(servers)
    k = np.random.default_rng(5).permutation(np.arange(1, n + 1, dtype=np.int64) * 7919)
    r = d(torch.from_numpy(k).to(dev))
    torch.cuda.synchronize()
    d.check()  # raises DedupOverflowError on an overflowed bucket
    uc = r.ucount.cpu().numpy()
    assert int(uc.sum()) == n and all(uc[q] == 0 for q in range(nranks) if q not in servers)
    inv = r.inv.cpu().numpy().view(np.uint32).astype(np.int64)
    np.testing.assert_array_equal(r.ukeys.cpu().numpy()[inv], k)


def test_dedup_overflow_is_raised_by_engine_check(dev):
    """The sticky overflow word reaches PSEngine.check (end of bench,
    backups, finish) instead of being dropped silently."""
    from swiftsnails_amd.ops.dedup import DedupOverflowError
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    t = HbmTable(1, 1 << 16, optimizer=Optimizer("sgd"), device=dev)
    eng = PSEngine(t, None, max_keys=1 << 12, dim=1, device=dev)
    eng.check()
    eng.dedupers[1].scratch[0] = 1  # what k_bd_dedup sets on a full LDS table
    with pytest.raises(DedupOverflowError):
        eng.check()


@pytest.mark.parametrize("mode", ["bucket", "hash"])
@pytest.mark.parametrize("nranks,n,frags", [(1, 20000, 97), (3, 20000, 97), (8, 20000, 97),
                                            (8, 20000, 128), (1, 400000, 97),
                                            (3, 400000, 1024)])
def test_dedup_route_matches_reference(dev, nranks, n, frags, mode):
    from swiftsnails_amd.ops.dedup import Deduper, dedup_reference
    from swiftsnails_amd.parallel.router import HashFrag

    rng = np.random.default_rng(nranks)
    if n <= 20000:
        k = rng.integers(0, 5000, size=n, dtype=np.int64)  # heavy duplication
    else:  # many buckets, Zipf hot keys, long tail
        k = (rng.zipf(1.2, n) * 7919 % 2_000_003).astype(np.int64)
    hf = HashFrag(nranks, frags)  # 97: modulo routing; powers of two: masked routing
    fm = hf.rank_map()
    d = Deduper(n + 5000, nranks=nranks, frag_map=torch.from_numpy(fm.astype(np.int32)), gdim=2,
                device=dev, mode=mode)
    r = d(torch.from_numpy(k).to(dev))
    torch.cuda.synchronize()
    uk_ref, uc_ref, _ = dedup_reference(k, nranks, fm, ucap=d.ucap)
    uc = r.ucount.cpu().numpy()
    np.testing.assert_array_equal(uc, uc_ref)
    uk = r.ukeys.cpu().numpy()
    for q in range(nranks):
        seg = np.sort(uk[q * d.ucap:q * d.ucap + uc[q]])
        np.testing.assert_array_equal(seg, np.sort(uk_ref[q * d.ucap:q * d.ucap + uc_ref[q]]
                                                   .view(np.int64)))
    inv = r.inv.cpu().numpy().view(np.uint32).astype(np.int64)
    np.testing.assert_array_equal(uk[inv], k)  # ukeys[inv] reproduces the batch
    g = r.ugrad.cpu().numpy()
    for q in range(nranks):
        assert not g[q * d.ucap:q * d.ucap + uc[q]].any()
    # reference routing parity: dest segment of each key == map[fmix64 % frag]
    dest = inv // d.ucap
    np.testing.assert_array_equal(dest, hf.rank_map()[hf.frag_of(k)])
    # the scratch cleans itself (no per-call memset): later calls stay exact
    for rep in range(3):
        k2 = rng.integers(0, 7000 + rep, size=15000 + rep, dtype=np.int64)
        r2 = d(torch.from_numpy(k2).to(dev))
        torch.cuda.synchronize()
        uk2 = r2.ukeys.cpu().numpy()
        inv2 = r2.inv.cpu().numpy().view(np.uint32).astype(np.int64)
        np.testing.assert_array_equal(uk2[inv2], k2)
        assert int(r2.ucount.sum().item()) == len(np.unique(k2))
    if mode == "hash":
        assert (d.skeys.cpu().numpy() == -1).all()
    else:
        d.check()
    # invalid (EMPTY) keys map to INVALID and are not counted
    k3 = k[:1000].copy()
    k3[::7] = -1
    r3 = d(torch.from_numpy(k3).to(dev))
    torch.cuda.synchronize()
    inv3 = r3.inv.cpu().numpy().view(np.uint32)
    assert (inv3[::7] == 0xFFFFFFFF).all()
    ok = k3 != -1
    np.testing.assert_array_equal(r3.ukeys.cpu().numpy()[inv3[ok].astype(np.int64)], k3[ok])
    assert int(r3.ucount.sum().item()) == len(np.unique(k3[ok]))


@pytest.mark.parametrize("nranks", [1, 4])
def test_bucket_dedup_edge_sizes_and_hot_key(dev, nranks):
    """Bucketed dedup at the sizes where its layout changes (tiny calls, one
    wave, one register tile) and a Zipf-extreme batch: one key repeated far
    past a dedup thread's register slots (the hot-bucket excess loop)."""
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.parallel.router import HashFrag

    fm = torch.from_numpy(HashFrag(nranks, 64).rank_map().astype(np.int32))
    d = Deduper(200_000, nranks=nranks, frag_map=fm, gdim=1, device=dev, mode="bucket")
    rng = np.random.default_rng(7)
    cases = [np.array([42], np.int64), np.array([5, 5], np.int64),
             rng.integers(0, 50, 63), rng.integers(0, 10**12, 64), rng.integers(0, 30, 65),
             rng.integers(0, 10**9, 4097),
             np.concatenate([np.full(150_000, 123456789, np.int64), rng.integers(0, 999, 3000)])]
    cases.append(np.concatenate([rng.integers(0, 1 << 32, 5000), [(1 << 32) + 7]]))
    for k in cases:
        k = k.astype(np.int64)
        r = d(torch.from_numpy(k).to(dev))
        torch.cuda.synchronize()
        inv = r.inv.cpu().numpy().view(np.uint32).astype(np.int64)
        np.testing.assert_array_equal(r.ukeys.cpu().numpy()[inv], k)
        assert int(r.ucount.sum().item()) == len(np.unique(k))
        # scratch word 3: this call's record width (0: 8-byte records, every
        # key fits 32 bits; the next call decides afresh)
        if os.environ.get("SS_BD_REC") is None:
            assert int(d.scratch[3].item()) == int(bool((k >> 32).any()))
    d.check()


@pytest.mark.parametrize("nranks", [1, 3])
@pytest.mark.parametrize("singles", [False, True])
def test_bucket_reduce_lr_matches_atomic_path(dev, nranks, singles):
    """Bucketed dedup's LDS reduction == per-occurrence atomics (also with
    the dedup's singleton flags: keys seen once are stored, not added)."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.parallel.router import HashFrag

    h = hip()
    B, F = 20000, 13
    n = B * F
    rng = np.random.default_rng(5 + nranks)
    keys = (rng.zipf(1.3, n) % 300000).astype(np.int64)
    keys[::101] = -1  # a few invalid occurrences
    fm = HashFrag(nranks, 64).rank_map()
    d = Deduper(n, nranks=nranks, frag_map=torch.from_numpy(fm.astype(np.int32)), gdim=1,
                device=dev, mode="bucket")
    if singles:
        d.track_singletons()
    r = d(torch.from_numpy(keys).to(dev))
    st = torch.cuda.current_stream().cuda_stream
    U = nranks * d.ucap
    if singles:  # the flags match the key multiplicities
        kv = keys[keys != -1]
        uk, cnt = np.unique(kv, return_counts=True)
        once = dict(zip(uk.tolist(), (cnt == 1).tolist()))
        uc0 = r.ucount.cpu().numpy()
        us, ukd = d.usingle.cpu().numpy(), r.ukeys.cpu().numpy()
        for q in range(nranks):
            for i in range(q * d.ucap, q * d.ucap + int(uc0[q]), 97):
                assert bool(us[i]) == once[int(ukd[i])]
    uvals = torch.randn(U, device=dev) * 0.1
    y = torch.from_numpy((rng.random(B) < 0.3).astype(np.float32)).to(dev)
    g_at = torch.zeros(U, device=dev)
    l_at = torch.zeros(256 * 32, device=dev)
    h.lr_fwd_bwd(r.inv.data_ptr(), 0, y.data_ptr(), B, F, uvals.data_ptr(), g_at.data_ptr(),
                 l_at.data_ptr(), 0, st)
    gs = torch.empty(B, device=dev)
    l_b = torch.zeros(256 * 32, device=dev)
    g_b = torch.full((U,), float("nan"), device=dev)  # reduce must write every unique row
    h.lr_fwd_g(r.inv.data_ptr(), 0, y.data_ptr(), B, F, uvals.data_ptr(), gs.data_ptr(), 1,
               l_b.data_ptr(), 0, st)
    d.reduce(n, gs, F, g_b)
    # the same forward through the BdIndex (no inverse index) gives the same gradients
    gs2 = torch.empty(B, device=dev)
    h.lr_fwd_g(0, 0, y.data_ptr(), B, F, uvals.data_ptr(), gs2.data_ptr(), 1, 0, 0, st,
               d.index_ptrs(n))
    # ... and through per-bucket occurrence-position parameters (k_bd_fill_occ:
    # one gather per occurrence); invalid occurrences read 0
    occ = torch.full((n,), float("nan"), device=dev)
    d.fill_occ(n, uvals, occ)
    gs3 = torch.empty(B, device=dev)
    l_c = torch.zeros(256 * 32, device=dev)
    h.lr_fwd_g(0, 0, y.data_ptr(), B, F, uvals.data_ptr(), gs3.data_ptr(), 1, l_c.data_ptr(),
               0, st, d.index_ptrs(n), occ=occ.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(gs, gs2)
    assert torch.equal(gs, gs3)
    np.testing.assert_allclose(l_c.sum().item(), l_b.sum().item(), rtol=1e-6)
    # occ holds each occurrence's row at its bucket position
    pos_of = d.pos_of[:n].cpu().numpy().astype(np.int64)
    inv = r.inv.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    ok = inv != 0xFFFFFFFF
    on = occ.cpu().numpy()
    np.testing.assert_array_equal(on[pos_of[ok]], uvals.cpu().numpy()[inv[ok]])
    d.check()
    uc = r.ucount.cpu().numpy()
    for q in range(nranks):
        a, b = q * d.ucap, q * d.ucap + uc[q]
        np.testing.assert_allclose(g_b[a:b].cpu().numpy(), g_at[a:b].cpu().numpy(), rtol=1e-4,
                                   atol=1e-4)
    np.testing.assert_allclose(l_b.sum().item(), l_at.sum().item(), rtol=1e-5)


@pytest.mark.parametrize("F", [39, 7, 64, 100])  # lane-group layout (<=64) and LDS fallback
def test_lr_fwd_bwd_matches_torch(dev, F):
    from swiftsnails_amd._native import hip

    B, U = 3000, 5000
    rng = np.random.default_rng(9)
    inv = rng.integers(0, U, size=B * F).astype(np.int32)
    x = rng.standard_normal(B * F).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    w = (rng.standard_normal(U) * 0.1).astype(np.float32)
    tinv, tx, ty, tw = (torch.from_numpy(a).to(dev) for a in (inv, x, y, w))
    g = torch.zeros(U, device=dev)
    loss = torch.zeros(256 * 32, device=dev)
    pred = torch.empty(B, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    hip().lr_fwd_bwd(tinv.data_ptr(), tx.data_ptr(), ty.data_ptr(), B, F, tw.data_ptr(),
                     g.data_ptr(), loss.data_ptr(), pred.data_ptr(), st)
    torch.cuda.synchronize()
    # fp32 torch reference
    W = torch.from_numpy(w).double()
    z = (W[torch.from_numpy(inv).long()] * torch.from_numpy(x).double()).view(B, F).sum(1)
    p = torch.sigmoid(z)
    Y = torch.from_numpy(y).double()
    ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(z, Y, reduction="sum")
    gs = (p - Y).repeat_interleave(F) * torch.from_numpy(x).double()
    ref_g = torch.zeros(U, dtype=torch.float64).index_add_(0, torch.from_numpy(inv).long(), gs)
    np.testing.assert_allclose(pred.cpu().numpy(), p.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.sum().item(), ref_loss.item(), rtol=1e-4)
    np.testing.assert_allclose(g.cpu().numpy(), ref_g.numpy(), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("F", [39, 13, 100])
@pytest.mark.parametrize("with_x", [False, True])
def test_lr_fwd_one_gather_matches_torch(dev, F, with_x):
    """The bucketed forward's one-gather mode (occ[pos_of[j]], per-sample
    gradient p - y): several sample groups per workgroup with their gathers
    in flight together (k_lr_fwd_occ).  B is not a multiple of a workgroup's
    samples, and some occurrences have no position (invalid keys: 0)."""
    from swiftsnails_amd._native import hip

    B, M = 3001, 40000
    rng = np.random.default_rng(17 + F)
    pos = rng.integers(0, M, size=B * F).astype(np.int64)
    pos[::97] = 0xFFFFFFFF
    x = rng.standard_normal(B * F).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    occ = (rng.standard_normal(M) * 0.2).astype(np.float32)
    tpos = torch.from_numpy(pos.astype(np.uint32).view(np.int32)).to(dev)
    tx, ty, tocc = (torch.from_numpy(a).to(dev) for a in (x, y, occ))
    gs = torch.full((B,), float("nan"), device=dev)
    loss = torch.zeros(256 * 32, device=dev)
    pred = torch.empty(B, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    hip().lr_fwd_g(0, tx.data_ptr() if with_x else 0, ty.data_ptr(), B, F, 0, gs.data_ptr(), 1,
                   loss.data_ptr(), pred.data_ptr(), st, [tpos.data_ptr(), 0, 0, 0],
                   occ=tocc.data_ptr())
    torch.cuda.synchronize()
    valid = pos != 0xFFFFFFFF
    w = np.where(valid, occ[np.where(valid, pos, 0)], 0.0).astype(np.float64)
    xv = x.astype(np.float64) if with_x else np.ones(B * F)
    z = torch.from_numpy((w * xv).reshape(B, F).sum(1))
    p = torch.sigmoid(z)
    Y = torch.from_numpy(y).double()
    ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(z, Y, reduction="sum")
    np.testing.assert_allclose(pred.cpu().numpy(), p.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gs.cpu().numpy(), (p - Y).numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.sum().item(), ref_loss.item(), rtol=1e-4)


@pytest.mark.parametrize("nranks", [1, 3])
def test_segreduce_lr_matches_atomic_path(dev, nranks):
    """Atomic-free bin-partition reduction == per-occurrence atomics (and torch)."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.parallel.router import HashFrag

    h = hip()
    B, F = 20000, 13
    n = B * F
    rng = np.random.default_rng(21 + nranks)
    keys = (rng.zipf(1.3, n) % 300000).astype(np.int64)  # heavy duplication + long tail
    fm = HashFrag(nranks, 64).rank_map()
    d = Deduper(n, nranks=nranks, frag_map=torch.from_numpy(fm.astype(np.int32)), gdim=1,
                device=dev, mode="hash")
    r = d(torch.from_numpy(keys).to(dev))
    st = torch.cuda.current_stream().cuda_stream
    U = nranks * d.ucap
    uvals = (torch.randn(U, device=dev) * 0.1)
    y = torch.from_numpy((rng.random(B) < 0.3).astype(np.float32)).to(dev)
    # atomic reference path
    g_at = torch.zeros(U, device=dev)
    l_at = torch.zeros(256 * 32, device=dev)
    h.lr_fwd_bwd(r.inv.data_ptr(), 0, y.data_ptr(), B, F, uvals.data_ptr(), g_at.data_ptr(),
                 l_at.data_ptr(), 0, st)
    # segmented path
    nbins, nch = h.sr_nbins(n), h.sr_nchunks(n)
    hist = torch.empty(h.sr_hist_words(n), dtype=torch.int32, device=dev)
    plan = torch.empty(n, dtype=torch.int64, device=dev)  # (occurrence j, cu low bits)
    gocc = torch.empty(n, device=dev)
    items = torch.empty(4 * h.sr_max_items(n), dtype=torch.int32, device=dev)
    nitems = torch.zeros(1, dtype=torch.int32, device=dev)
    g_sr = torch.zeros(U, device=dev)  # dedup zeroes the round's rows
    l_sr = torch.zeros(256 * 32, device=dev)
    h.sr_plan(r.inv.data_ptr(), n, r.ucount.data_ptr(), nranks, d.ucap, hist.data_ptr(), nbins,
              plan.data_ptr(), items.data_ptr(), nitems.data_ptr(), st)
    h.lr_fwd_g(r.inv.data_ptr(), 0, y.data_ptr(), B, F, uvals.data_ptr(), gocc.data_ptr(), 0,
               l_sr.data_ptr(), 0, st)
    h.sr_reduce(plan.data_ptr(), gocc.data_ptr(), items.data_ptr(), nitems.data_ptr(), n,
                r.ucount.data_ptr(), nranks, d.ucap, g_sr.data_ptr(), st)
    torch.cuda.synchronize()
    uc = r.ucount.cpu().numpy()
    assert int(hist[-1].item()) == n  # every valid occurrence placed exactly once
    ps = np.sort(plan.cpu().numpy().view(np.uint32).reshape(n, 2)[:, 0])
    np.testing.assert_array_equal(ps, np.arange(n, dtype=np.uint32))
    for q in range(nranks):
        a, b = q * d.ucap, q * d.ucap + uc[q]
        np.testing.assert_allclose(g_sr[a:b].cpu().numpy(), g_at[a:b].cpu().numpy(), rtol=1e-4,
                                   atol=1e-4)
    np.testing.assert_allclose(l_sr.sum().item(), l_at.sum().item(), rtol=1e-5)


def test_gen_ctr_ranges(dev):
    from swiftsnails_amd.models.sparse_lr import CtrSynth

    d = CtrSynth(batch_size=4096, num_fields=39, num_features=10_000_000)
    keys = torch.empty(4096 * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(4096, device=dev)
    d.generate(0, 0, 1, keys, labels)
    torch.cuda.synchronize()
    k = keys.cpu().numpy().reshape(4096, 39)
    V = d.vocab_per_field
    f = k // V
    assert (f == np.arange(39)[None, :]).all()
    lab = labels.cpu().numpy()
    assert set(np.unique(lab)) <= {0.0, 1.0} and 0.05 < lab.mean() < 0.95
    k2 = torch.empty_like(keys)
    d.generate(0, 0, 1, k2, labels)
    assert torch.equal(keys, k2)  # deterministic


@pytest.mark.parametrize("F", [39, 100])  # lane-group kernel and the LDS fallback
def test_gen_ctr_matches_numpy_generator(dev, F):
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.ctr_data import gen_ctr_np

    B, V = 2000, 1_000_003
    keys = torch.empty(B * F, dtype=torch.int64, device=dev)
    labels = torch.empty(B, device=dev)
    hip().gen_ctr(7, 12345, B, F, V, 0.1, 1.0, -1.0, keys.data_ptr(), labels.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rk, rl = gen_ctr_np(7, 12345, B, F, V, 0.1, 1.0, -1.0)
    # ids use fp64 exp on both sides: allow a rare last-ulp floor difference
    assert (keys.cpu().numpy() == rk).mean() > 0.9999
    assert (labels.cpu().numpy() == rl).mean() > 0.995  # sums differ in float order only


def test_sparse_lr_trains_world1(dev):
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    data = CtrSynth(batch_size=8192, num_fields=16, num_features=200_000, tail_frac=0.0)
    table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev)
    eng = PSEngine(table, None, max_keys=8192 * 16, dim=1, device=dev)
    w = SparseLRWorker(eng, data)
    losses = []
    for i in range(60):
        w.step()
        losses.append(w.mean_loss())
    table.check()
    assert np.mean(losses[-5:]) < np.mean(losses[:3]) - 0.02, losses
    assert 0 < table.size() <= data.num_features


def test_engine_pull_push_keys_world1(dev):
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    t = HbmTable(4, 1 << 14, optimizer=Optimizer("sgd", lr=1.0), init=InitConfig("zero"),
                 device=dev)
    eng = PSEngine(t, None, max_keys=1000, dim=4, device=dev)
    k = torch.tensor([5, 7, 5, 9, 7, 5], dtype=torch.int64, device=dev)
    g = torch.ones(6, 4, device=dev)
    eng.push_keys(k, g)
    vals = eng.pull_dense(k)
    torch.cuda.synchronize()
    v = vals.cpu().numpy()[:, 0]
    np.testing.assert_allclose(v, [-3, -2, -3, -1, -2, -3])  # SGD lr=1, merged grads


def test_rccl_comm_world1(dev):
    from swiftsnails_amd._native import hip

    h = hip()
    c = h.RcclComm(0, 1, h.RcclComm.unique_id(), 0)
    a = torch.arange(10, dtype=torch.float32, device=dev)
    b = torch.zeros(10, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    c.alltoallv(a.data_ptr(), [4], [2], b.data_ptr(), [4], [5], 4, st)
    c.allreduce(a.data_ptr(), a.data_ptr(), 10, 0, 0, st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(b.cpu().numpy()[5:9], [2, 3, 4, 5])


@pytest.mark.parametrize("G,load", [(1, 0.9), (4, 0.5), (64, 0.95)])
def test_pull_unique_insert(dev, G, load):
    """Unique-key pull (CAS insert) under heavy collisions."""
    from swiftsnails_amd.ops.optim import InitConfig, init_reference
    from swiftsnails_amd.ops.table import HbmTable

    init = InitConfig("uniform", 1.0, 0.0, seed=11)
    n = 20000
    t = HbmTable(2, int(n / load) + 1, init=init, device=dev, lane_group=G)
    k = np.unique(_keys(n + 500, 12))[:n]
    rng = np.random.default_rng(13)
    # two overlapping rounds: half old keys, half new keys in round 2
    k1 = k[: n // 2]
    k2 = np.concatenate([k[n // 4: n // 2], k[n // 2:]])
    rng.shuffle(k2)
    v1, s1 = t.pull(torch.from_numpy(k1).to(dev), unique=True)
    v2, s2 = t.pull(torch.from_numpy(k2).to(dev), unique=True)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == n
    np.testing.assert_array_equal(v1.cpu().numpy(), init_reference(init, k1, 2, 2)[:, :2])
    np.testing.assert_array_equal(v2.cpu().numpy(), init_reference(init, k2, 2, 2)[:, :2])
    s2n = s2.cpu().numpy()
    assert (s2n >= 0).all() and len(np.unique(s2n)) == len(k2)
    d = t.to_dict()
    assert len(d) == n and set(d) == set(int(x) for x in k.view(np.uint64))


def test_probe_histogram_and_stats(dev):
    from swiftsnails_amd.ops.table import HbmTable

    t = HbmTable(1, 5000, device=dev)
    keys = torch.arange(3500, dtype=torch.int64, device=dev) * 7919 + 11
    t.pull(keys, insert=True)
    h = t.probe_histogram(16)
    assert int(h.sum()) == 3500 == t.size()
    assert h[0] > 1000  # most keys sit at their home slot at load 0.7
    st = t.stats()
    assert abs(st["load_factor"] - 3500 / t.capacity) < 1e-9
    assert 0 <= st["probe_mean"] < 5


@pytest.mark.parametrize("prefill", ["1", "0"])
def test_sparse_lr_dist_path_matches_fast_path(dev, monkeypatch, prefill):
    """One GPU through the N>1 engine path (SS_ENGINE_GENERAL=1: send
    segments, bucket runs, the server's merge of received keys, the server's
    snapshot pull and fused blind-store AdaGrad) trains the same model as the
    1-GPU fast path (pull snapshot + AdaGrad fused into the worker's merge),
    step for step, up to the float summation order."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_TABLE_PREFILL", prefill)
    monkeypatch.setenv("SS_PULL_AHEAD", "0")  # the fast path's LR schedule (no staleness)
    out = {}
    for general in ("0", "1"):
        monkeypatch.setenv("SS_ENGINE_GENERAL", general)
        data = CtrSynth(batch_size=4096, num_fields=13, num_features=300_000, tail_frac=0.2)
        table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev)
        eng = PSEngine(table, None, max_keys=4096 * 13, dim=1, device=dev)
        assert eng.fast1 == (general == "0")
        w = SparseLRWorker(eng, data)
        losses = [float(w.step().sum().item()) for _ in range(12)]
        torch.cuda.synchronize()
        eng.check()
        if general == "1":
            assert eng.srv[0].snap_valid  # blind store from the server's snapshot
            m = eng.metrics.counters
            assert 0 < m["server_unique"] == m["unique_recv"]  # one source: no cross merges
        out[general] = (losses, table.to_dict(with_state=True))
    (l1, t1), (l0, t0) = out["1"], out["0"]
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    assert t1.keys() == t0.keys()
    ks = list(t1.keys())[:20000]
    np.testing.assert_allclose(np.stack([t1[k] for k in ks]), np.stack([t0[k] for k in ks]),
                               rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("prefill", ["1", "0"])
def test_zero_init_prefilled_rows(dev, monkeypatch, prefill):
    """Zero-init tables are allocated with the initial row in every empty
    slot (insert = key CAS only); pulled rows, state and a following update
    are the same as with per-insert row writes."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable

    monkeypatch.setenv("SS_TABLE_PREFILL", prefill)
    t = HbmTable(3, 1 << 14, optimizer=Optimizer("adagrad", lr=0.5),
                 init=InitConfig("zero", state_init=0.1), device=dev)
    assert t.prefilled == (prefill == "1")
    base = np.unique(_keys(3000, 9))
    k = np.concatenate([base, base[:700]])  # duplicates in one launch
    v, s = t.pull(torch.from_numpy(k).to(dev), unique=False)
    torch.cuda.synchronize()
    t.check()
    assert t.size() == len(base)
    assert torch.count_nonzero(v).item() == 0
    d = t.to_dict(with_state=True)
    np.testing.assert_allclose(np.stack([d[int(x)] for x in base[:100]]),
                               np.tile([0, 0, 0, 0.1, 0.1, 0.1], (100, 1)), rtol=1e-6)
    g = torch.ones((len(base), 3), device=dev)
    t.push(torch.from_numpy(base).to(dev), g)
    torch.cuda.synchronize()
    d = t.to_dict(with_state=True)
    row = d[int(base[5])]
    np.testing.assert_allclose(row[3:], 1.1, rtol=1e-6)
    np.testing.assert_allclose(row[:3], -0.5 / np.sqrt(1.1), rtol=1e-4)


def test_engine_snapshot_invalidated_by_interleaved_push(dev, monkeypatch):
    """pull A, pull B, push A, push B over overlapping keys: B's snapshot is
    stale after A's push, so B must re-read its rows (no lost update)."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    ka = torch.arange(1, 3001, dtype=torch.int64, device=dev)
    kb = torch.arange(1501, 4501, dtype=torch.int64, device=dev)
    res = {}
    for snap in ("1", "0"):
        t = HbmTable(1, 1 << 16, optimizer=Optimizer("adagrad", lr=0.5),
                     init=InitConfig("uniform", 0.1, 0.1, seed=3), device=dev)
        assert t.snapshot_ok
        eng = PSEngine(t, None, max_keys=4096, dim=1, device=dev)
        eng.snapshot = snap == "1"  # "0": every apply reads its rows
        ra = eng.pull(ka)
        rb = eng.pull(kb)
        assert (ra.snap is not None) == (snap == "1")
        eng.accumulate(ra, torch.ones(len(ka), 1, device=dev))
        eng.push(ra)
        eng.accumulate(rb, torch.full((len(kb), 1), 2.0, device=dev))
        eng.push(rb)
        rc = eng.pull(kb)  # sequential pull -> push: the snapshot is used
        eng.accumulate(rc, torch.ones(len(kb), 1, device=dev))
        eng.push(rc)
        torch.cuda.synchronize()
        t.check()
        res[snap] = t.to_dict(with_state=True)
    assert res["1"].keys() == res["0"].keys()
    for k in res["0"]:
        np.testing.assert_array_equal(res["1"][k], res["0"][k])
    # keys in both A and B saw both updates: h = 0.1 + 1 + 4 + 1
    np.testing.assert_allclose(res["1"][2000][1], 6.1, rtol=1e-6)


def test_hbm_table_streaming_checkpoint(dev, tmp_path):
    """Binary checkpoint of an HBM shard streamed in small export chunks and
    loaded back in small chunks reproduces every row and optimizer state."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.utils import checkpoint as ck

    t = HbmTable(5, 1 << 16, optimizer=Optimizer("adagrad", lr=0.3),
                 init=InitConfig("uniform", 0.2, 0.1, seed=11), device=dev)
    k = torch.from_numpy(np.unique(_keys(20000, 4))).to(dev)
    t.pull(k, unique=True)
    t.push(k, torch.randn(len(k), 5, device=dev))
    torch.cuda.synchronize()

    class Chunked:
        def __init__(self, tab):
            self.tab = tab

        def __getattr__(self, a):
            return getattr(self.tab, a)

        def export(self, *a, **kw):
            return self.tab.export(chunk_slots=4096)

    p = str(tmp_path / "shard.bin")
    assert ck.save_binary(Chunked(t), p) == t.size() == len(k)
    t2 = HbmTable(5, 1 << 16, optimizer=Optimizer("adagrad", lr=0.3), init=InitConfig("zero"),
                  device=dev)
    assert ck.load_binary(t2, p, chunk=3000) == len(k)
    a, b = t.to_dict(with_state=True), t2.to_dict(with_state=True)
    assert a.keys() == b.keys()
    for key in list(a)[:2000]:
        np.testing.assert_array_equal(a[key], b[key])


def test_native_gpu_worker_pull_push(dev):
    """C++ GpuWorker (worker.h): pull returns rows in occurrence order
    (inserting missing keys), push applies the per-key SUM of duplicate keys'
    gradients once — the same table as the Python path with merged grads."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable

    def table():
        return HbmTable(4, 1 << 15, optimizer=Optimizer("adagrad", lr=0.2),
                        init=InitConfig("uniform", 0.3, 0.1, seed=9), device=dev)

    t, ref = table(), table()
    w = hip().GpuWorker(t.dt, t.size_ctr.data_ptr(), t.err.data_ptr(), t._init_native,
                        t.opt.native(), t.G, 4096)
    rng = np.random.default_rng(2)
    keys_np = rng.integers(1, 700, 3000).astype(np.int64)  # heavy duplication
    keys = torch.from_numpy(keys_np).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    vals = torch.empty(len(keys), 4, device=dev)
    h = w.pull(keys.data_ptr(), len(keys), vals.data_ptr(), st)
    h.wait()
    assert h.done()
    uk = np.unique(keys_np)
    rv, _ = ref.pull(torch.from_numpy(uk).to(dev), unique=True)
    torch.cuda.synchronize()
    row = {int(k): rv[i].cpu().numpy() for i, k in enumerate(uk)}
    np.testing.assert_array_equal(vals.cpu().numpy(), np.stack([row[int(k)] for k in keys_np]))
    assert t.size() == len(uk)
    g_np = rng.standard_normal((len(keys_np), 4)).astype(np.float32)
    w.push(keys.data_ptr(), len(keys), torch.from_numpy(g_np).to(dev).data_ptr(), st).wait()
    merged = np.zeros((len(uk), 4), np.float32)
    np.add.at(merged, np.searchsorted(uk, keys_np), g_np)
    ref.push(torch.from_numpy(uk).to(dev), torch.from_numpy(merged).to(dev))
    torch.cuda.synchronize()
    t.check()
    a, b = t.to_dict(with_state=True), ref.to_dict(with_state=True)
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_allclose(a[k], b[k], rtol=1e-5, atol=1e-6)


def test_stream_helpers_match_torch(dev):
    """utils/streams.py: the explicit-device lookups and the stream switch
    agree with torch's own view of the current stream, and restore it."""
    from swiftsnails_amd.utils.streams import current, current_raw, use_stream

    idx = dev.index or 0
    base = torch.cuda.current_stream(dev)
    assert current_raw(idx) == base.cuda_stream == current_raw()
    assert current(idx) == base
    s = torch.cuda.Stream(device=dev)
    with use_stream(s):
        assert torch.cuda.current_stream(dev) == s
        assert current_raw(idx) == s.cuda_stream
        x = torch.ones(1000, device=dev) * 2  # a torch op lands on s
    assert torch.cuda.current_stream(dev) == base
    s.synchronize()
    assert float(x.sum().item()) == 2000.0


@pytest.mark.parametrize("dim,fused", [(1, True), (3, False), (64, False), (9, True),
                                       (128, True)])
def test_server_merge_matches_reference(dev, dim, fused):
    """server.hip on the keys three sources route to one server (real
    bucketed dedups with the common N>1 layout, overlapping key sets): one
    entry per distinct key, response rows per received position, and the
    merged gradient of every distinct key — fused into the AdaGrad update
    (scalar rows: read-modify-write, no snapshot; wider rows: a lane group per
    key), else a merged row then the apply kernel.  N = 3 splits a server
    bucket in m = 2: the sources group each run by sub-bucket and send the
    offsets, the server reads exact ranges."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.router import HashFrag

    h = hip()
    N, me, n = 3, 1, 30000
    fm = torch.from_numpy(HashFrag(N, 64).rank_map().astype(np.int32))
    rng = np.random.default_rng(17)
    pool = rng.choice(1 << 40, 40000, replace=False).astype(np.int64) + 1
    ds = [Deduper(n, nranks=N, frag_map=fm, gdim=dim, device=dev) for _ in range(N)]
    for d in ds:
        d.lay_n = n
    Pd = h.bd_buckets(n, N, ds[0].ndest) // N
    m = h.srv_sub_buckets(N)
    assert m > 1
    for d in ds:
        d.split_for_servers(m)
    roff = torch.zeros(N * Pd * m, dtype=torch.int32, device=dev)
    cap = n
    rkeys = torch.full((N * cap,), -1, dtype=torch.int64, device=dev)
    meta = torch.zeros(2 * N * Pd, dtype=torch.int32, device=dev)
    recv = []
    for s, d in enumerate(ds):
        keys = torch.from_numpy(rng.choice(pool, n)).to(dev)  # duplicates within + across
        r = d(keys)
        c = int(r.ucount[me])
        rkeys[s * cap:s * cap + c] = r.ukeys[me * cap:me * cap + c]
        ub, un = d.run_tables(Pd)
        meta[s * Pd:(s + 1) * Pd] = ub[me * Pd:(me + 1) * Pd]
        meta[N * Pd + s * Pd:N * Pd + (s + 1) * Pd] = un[me * Pd:(me + 1) * Pd]
        roff[s * Pd * m:(s + 1) * Pd * m] = d.sub_table(Pd)[me * Pd * m:(me + 1) * Pd * m]
        recv.append((s * cap, c))
    P = Pd * m
    rows = N * cap
    i32 = dict(dtype=torch.int32, device=dev)
    cnt, bstart = torch.zeros(P + 1, **i32), torch.empty(P + 1, **i32)
    ubase, unum = torch.empty(P, **i32), torch.empty(P, **i32)
    pj, luid = torch.empty(rows, **i32), torch.empty(rows, **i32)
    bkeys = torch.empty(rows, dtype=torch.int64, device=dev)
    uc = torch.zeros(1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, **i32)
    st = torch.cuda.current_stream().cuda_stream
    h.srv_dedup(rkeys.data_ptr(), meta.data_ptr(), meta.data_ptr() + 4 * N * Pd, cap, N, Pd, m,
                me, cnt.data_ptr(), bstart.data_ptr(), pj.data_ptr(), luid.data_ptr(),
                bkeys.data_ptr(), ubase.data_ptr(), unum.data_ptr(), uc.data_ptr(),
                err.data_ptr(), st, roff.data_ptr())
    pos = np.concatenate([np.arange(a, a + c) for a, c in recv])
    rk = rkeys.cpu().numpy()[pos]
    distinct = np.unique(rk)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert int(uc.item()) == len(distinct) < len(pos)  # the sources overlap
    assert int(bstart[P].item()) == len(pos)
    t = HbmTable(dim, 1 << 18, optimizer=Optimizer("adagrad", lr=0.3),
                 init=InitConfig("uniform", 0.2, 0.1, seed=5), device=dev)
    svals = torch.empty((rows, dim), device=dev)
    sslots = torch.empty(rows, dtype=torch.int64, device=dev)
    t.pull_buckets((bkeys.data_ptr(), bstart.data_ptr(), unum.data_ptr(), ubase.data_ptr(), P),
                   svals, sslots)
    rvals = torch.full((rows, dim), float("nan"), device=dev)
    h.srv_fill(P, bstart.data_ptr(), ubase.data_ptr(), unum.data_ptr(), pj.data_ptr(),
               luid.data_ptr(), svals.data_ptr(), rvals.data_ptr(), dim, st)
    torch.cuda.synchronize()
    assert t.size() == len(distinct)
    before = t.to_dict(with_state=True)
    np.testing.assert_array_equal(rvals.cpu().numpy()[pos],
                                  np.stack([before[int(k)][:dim] for k in rk]))
    g = torch.randn((rows, dim), device=dev)
    gn = g.cpu().numpy()
    if fused:
        h.srv_merge(P, bstart.data_ptr(), ubase.data_ptr(), unum.data_ptr(), pj.data_ptr(),
                    luid.data_ptr(), g.data_ptr(), 0, dim, t.dt, sslots.data_ptr(), 0,
                    t.opt.native(), st)
    else:
        merged = torch.empty((rows, dim), device=dev)
        h.srv_merge(P, bstart.data_ptr(), ubase.data_ptr(), unum.data_ptr(), pj.data_ptr(),
                    luid.data_ptr(), g.data_ptr(), merged.data_ptr(), dim, st=st)
        t.push_slots(sslots, merged, segs=t.dev_segs(uc), max_n=rows)
    torch.cuda.synchronize()
    after = t.to_dict(with_state=True)
    acc = {}
    for k, p in zip(rk.tolist(), pos.tolist()):
        acc[k] = acc.get(k, 0.0) + gn[p].astype(np.float64)
    for k in list(acc)[:3000]:
        w0, h0 = before[k][:dim].astype(np.float64), before[k][dim:].astype(np.float64)
        h1 = h0 + acc[k] ** 2
        w1 = w0 - 0.3 * acc[k] / np.sqrt(h1 + 1e-8)
        np.testing.assert_allclose(after[k][dim:], h1, rtol=2e-4, atol=1e-5)
        np.testing.assert_allclose(after[k][:dim], w1, rtol=2e-4, atol=1e-5)


def test_push_method_set_after_engine_on_lr_table(dev):
    """A tensor-code update rule installed AFTER the engine was built on a
    scalar-AdaGrad (LR-shaped) table: the pull takes no snapshot, the rule
    runs, and hipGraph replay is refused (the rule syncs the host)."""
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    data = CtrSynth(batch_size=1024, num_fields=8, num_features=50_000)
    t = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev)
    eng = PSEngine(t, None, max_keys=1024 * 8, dim=1, device=dev)
    assert eng.snapshot and t.snapshot_ok
    calls = []

    def rule(rows, g):
        calls.append(rows.shape[0])
        rows[:, 0] -= 0.5 * g[:, 0]
        return rows

    t.set_push_method(rule)
    assert not t.snapshot_ok
    keys = torch.arange(1, 201, dtype=torch.int64, device=dev)
    r = eng.pull(keys)
    assert r.snap is None
    eng.accumulate(r, torch.ones(200, 1, device=dev))
    eng.push(r)
    torch.cuda.synchronize()
    assert calls == [200]
    v, _ = t.pull(keys, insert=False)
    np.testing.assert_allclose(v.cpu().numpy()[:, 0], -0.5, rtol=1e-6)
    w = SparseLRWorker(eng, data)
    assert not w.enable_graph()


def test_user_init_and_pull_methods_fast_path(dev):
    """One GPU (fast path, bucketed pull): keys are created with the user's
    rows, pulls return the user's transform, the compiled const init works,
    and a push of never-pulled keys starts from the user's rows too."""
    from test_engine_cpu import DIM, _grads_for, _init_rows, _keys_for, _pull_vals, access_oracle

    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    t = HbmTable(DIM, 8192, Optimizer("adagrad", lr=0.1), InitConfig("zero"), device=dev)
    t.set_init_method(lambda k: _init_rows(k.cpu()).to(dev))
    t.set_pull_method(_pull_vals)
    assert not t.snapshot_ok
    eng = PSEngine(t, None, max_keys=300, dim=DIM, device=dev)
    rows, pulled = access_oracle(world=1)  # one worker's stream
    for rnd in range(3):
        k = _keys_for(0, rnd)
        r = eng.pull(torch.from_numpy(k).to(dev))
        got = eng.gather(r, len(k)).cpu().numpy()
        np.testing.assert_allclose(got, pulled[(0, rnd)], rtol=1e-4, atol=1e-5)
        eng.accumulate(r, torch.from_numpy(_grads_for(k, 0, rnd)).to(dev))
        eng.push(r)
    torch.cuda.synchronize()
    st = t.to_dict(with_state=True)
    assert set(st) == set(rows)
    for x, row in rows.items():
        np.testing.assert_allclose(st[x], row, rtol=1e-4, atol=1e-5)
    # a push creates keys with the user's rows before the update
    t.push(torch.tensor([999_001], device=dev), torch.ones(1, DIM, device=dev))
    row = t.to_dict(with_state=True)[999_001]
    r0 = _init_rows(torch.tensor([999_001])).numpy()[0]
    np.testing.assert_allclose(row[DIM:], r0[DIM:] + 1, rtol=1e-5)
    # compiled constant initialiser
    c = HbmTable(2, 1024, Optimizer("sgd"), InitConfig("const", scale=0.25), device=dev)
    v, _ = c.pull(torch.tensor([5, 6], device=dev))
    np.testing.assert_allclose(v.cpu().numpy(), 0.25)


def _bf16_round(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even) -> fp32, finite inputs."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("G", [1, 4, 16, 64])
def test_compact_bf16_rows(dev, G):
    """Compact rows (row_dtype="bf16"): half the slot bytes; a pull returns
    the bf16-rounded initial row; AdaGrad pushes track an fp32 table to bf16
    precision; updates far below half an ulp still move a weight in
    expectation (stochastic rounding); checkpoint export / assign round-trip
    exactly; a tensor-code init method works on compact rows."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable

    # (dim 32 / 128: word2vec's wide rows — the vectorised apply moves 4
    # bf16 words per 8-byte access, table.hip k_apply_rows<D, true>)
    dim = {1: 1, 4: 9, 16: 32, 64: 128}[G]
    init = InitConfig("uniform", 0.5, 0.1, seed=3)
    mk = lambda dt: HbmTable(dim, 1 << 14, optimizer=Optimizer("adagrad", lr=0.05),  # noqa: E731
                             init=init, device=dev, lane_group=G, row_dtype=dt)
    t32, t16 = mk("fp32"), mk("bf16")
    # (a scalar LR row is 8 B either way inside its 16-byte [row | key] slot)
    assert t16.stride <= t32.stride and (dim == 1 or t16.nbytes < 0.75 * t32.nbytes)
    keys = torch.from_numpy(np.unique(_keys(3000, 8))[:2000]).to(dev)
    v32, s32 = t32.pull(keys, unique=True)
    v16, s16 = t16.pull(keys, unique=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(v16.cpu().numpy(), _bf16_round(v32.cpu().numpy()))
    rng = np.random.default_rng(1)
    for _ in range(20):
        g = torch.from_numpy(rng.standard_normal((keys.numel(), dim)).astype(np.float32)).to(dev)
        t32.push_slots(s32, g)
        t16.push_slots(s16, g)
    a, b = t32.pull(keys, insert=False)[0], t16.pull(keys, insert=False)[0]
    torch.cuda.synchronize()
    np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=0.03, atol=0.02)
    # checkpoint rows go out as fp32 and come back bit-exact
    d = t16.to_dict(with_state=True)
    t2 = mk("bf16")
    ks = np.array(list(d.keys()), dtype=np.uint64)
    t2.assign(torch.from_numpy(ks.view(np.int64)).to(dev),
              torch.from_numpy(np.stack([d[int(k)] for k in ks])))
    d2 = t2.to_dict(with_state=True)
    assert d2.keys() == d.keys()
    for k in list(d)[:200]:
        np.testing.assert_array_equal(d2[k], d[k])
    # 400 SGD steps of lr * g = 1e-4 on weights of 1.0 (half an ulp is
    # 2^-8 = 3.9e-3): round-to-nearest would never move them
    sgd = HbmTable(dim, 1 << 12, optimizer=Optimizer("sgd", lr=1e-4), device=dev,
                   init=InitConfig("const", 1.0), lane_group=G, row_dtype="bf16")
    k2 = keys[:512]
    _, s2 = sgd.pull(k2, unique=True)
    one = torch.ones((k2.numel(), dim), device=dev)
    for _ in range(400):
        sgd.push_slots(s2, one)
    w = sgd.pull(k2, insert=False)[0].cpu().numpy()
    assert abs(w.mean() - (1.0 - 400 * 1e-4)) < 4e-3, w.mean()
    # tensor-code initialiser on compact rows (marker row, replaced after the pull)
    t16.set_init_method(lambda k: torch.full((k.numel(), t16.width), 0.25, device=dev))
    newk = torch.from_numpy(np.unique(_keys(500, 99))[:300]).to(dev)
    v, _ = t16.pull(newk, unique=True)
    torch.cuda.synchronize()
    assert torch.all(v == 0.25)


def test_server_bucket_past_parking_area(dev):
    """A server bucket with more received keys than its LDS parking area
    (8192; a Zipf-head bucket of the record exchange, whose sources ship every
    occurrence) is deduplicated whole: the keys past the parking area find
    their local id by a second probe, no error is set, and the fill writes
    every received position's row and nothing past the bucket."""
    from swiftsnails_amd._native import hip

    h = hip()
    n, nd = 10000, 100
    rng = np.random.default_rng(5)
    keys = torch.from_numpy(rng.choice(np.arange(1, nd + 1, dtype=np.int64), n)).to(dev)
    rbase = torch.zeros(1, dtype=torch.int32, device=dev)
    rnum = torch.full((1,), n, dtype=torch.int32, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    cnt, bstart = torch.zeros(2, **i32), torch.empty(2, **i32)
    ubase, unum = torch.empty(1, **i32), torch.empty(1, **i32)
    rows = n + 64
    pj = torch.full((rows,), -7, **i32)
    luid = torch.full((rows,), -7, **i32)
    bkeys = torch.empty(rows, dtype=torch.int64, device=dev)
    uc = torch.zeros(1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, **i32)
    st = torch.cuda.current_stream().cuda_stream
    h.srv_dedup(keys.data_ptr(), rbase.data_ptr(), rnum.data_ptr(), rows, 1, 1, 1, 0,
                cnt.data_ptr(), bstart.data_ptr(), pj.data_ptr(), luid.data_ptr(),
                bkeys.data_ptr(), ubase.data_ptr(), unum.data_ptr(), uc.data_ptr(),
                err.data_ptr(), st)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    pjn, ln = pj.cpu().numpy(), luid.cpu().numpy()
    np.testing.assert_array_equal(pjn[:n], np.arange(n))
    assert (ln[:n] >= 0).all() and int(uc.item()) == len(np.unique(keys.cpu().numpy()))
    bk = bkeys.cpu().numpy()
    np.testing.assert_array_equal(bk[ln[:n]], keys.cpu().numpy()[pjn[:n]])
    assert (pjn[n:] == -7).all() and (ln[n:] == -7).all()  # nothing past the bucket
    svals = torch.arange(rows, dtype=torch.float32, device=dev) + 1.0
    out = torch.full((rows,), float("nan"), device=dev)
    h.srv_fill(1, bstart.data_ptr(), ubase.data_ptr(), unum.data_ptr(), pj.data_ptr(),
               luid.data_ptr(), svals.data_ptr(), out.data_ptr(), 1, st)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    np.testing.assert_array_equal(o[:n], ln[:n] + 1.0)  # ubase 0: row luid + 1
    assert np.isnan(o[n:]).all()
