"""Model kernels on MI355X vs fp64/fp32 host references: word2vec SGNS, FM,
plus short end-to-end training runs through the PS engine."""
import os

import numpy as np
import pytest
import torch
from _mp import in_child

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from swiftsnails_amd._native import hip

    hip()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("D,bf16", [(32, 0), (64, 0), (128, 0), (32, 1), (64, 1), (128, 1)])
def test_w2v_sgns_tile_matches_reference(dev, D, bf16):
    """fp32 tile: fp32-exact; bf16 tile (SS_W2V_MFMA=bf16): negative-sample
    GEMMs from bf16-rounded rows, checked at bf16 tolerance."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.word2vec import sgns_reference

    T, C, S = 128, 4, 64  # two tiles
    tiles = T // 64
    rng = np.random.default_rng(D)
    nrows = T + T * C + tiles * S  # every occurrence its own row: exact per-row check
    U = (rng.standard_normal((nrows, D)) * 0.3).astype(np.float32)
    inv = np.arange(nrows, dtype=np.int32)
    g = torch.zeros((nrows, D), device=dev)
    loss = torch.zeros(256 * 32, device=dev)
    tu, ti = torch.from_numpy(U).to(dev), torch.from_numpy(inv).to(dev)
    p, es = ti.data_ptr(), 4
    neg_scale = 0.7
    hip().w2v_sgns(p, p + T * es, p + T * (1 + C) * es, T, C, D, neg_scale, tu.data_ptr(),
                   g.data_ptr(), loss.data_ptr(), torch.cuda.current_stream().cuda_stream,
                   bf16)
    torch.cuda.synchronize()
    G = g.cpu().numpy()
    tot = 0.0
    # bf16 tile: rows rounded to 8 mantissa bits -> ~3 significant digits in
    # the negative-sample terms (the positive pairs and context grads are fp32)
    rt, at = (2e-4, 2e-5) if not bf16 else (3e-2, 1e-2)
    for t in range(tiles):
        V = U[t * 64:(t + 1) * 64]
        X = U[T:T + T * C].reshape(T, C, D)[t * 64:(t + 1) * 64]
        N = U[T + T * C + t * S:T + T * C + (t + 1) * S]
        l, gV, gX, gN = sgns_reference(V, X, N, neg_scale)
        tot += l
        np.testing.assert_allclose(G[t * 64:(t + 1) * 64], gV, rtol=rt, atol=at)
        np.testing.assert_allclose(G[T:T + T * C].reshape(T, C, D)[t * 64:(t + 1) * 64], gX,
                                   rtol=2e-4, atol=2e-5)
        np.testing.assert_allclose(G[T + T * C + t * S:T + T * C + (t + 1) * S], gN, rtol=rt,
                                   atol=at)
    np.testing.assert_allclose(loss.sum().item(), tot, rtol=1e-4 if not bf16 else 3e-3)


@pytest.mark.parametrize("D,W,B", [(32, 2, 128), (64, 5, 150), (128, 5, 256), (128, 15, 100)])
def test_w2v_window_tile_matches_reference(dev, D, W, B):
    """Windowed skip-gram tile (k_w2v_win_bf16) vs the fp64 reference on the
    same band of valid pairs: every run position its own row, so each row's
    gradient (summed over the tiles whose window covers it) is checked;
    random sentence tags, reduced windows and masked positions; a partial
    last tile (B = 150, 100)."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.word2vec import sgns_window_reference, window_pairs_reference

    S, T = 64, 64
    tiles = (B + T - 1) // T
    R = B + 2 * W
    rng = np.random.default_rng(D + W)
    tags = np.cumsum(rng.random(R) < 0.08)  # sentences of ~12 tokens
    bs = rng.integers(1, W + 1, R)
    meta = ((tags << 4) | bs).astype(np.int32)
    meta[rng.random(R) < 0.1] = -1
    nrows = B + R + tiles * S
    U = (rng.standard_normal((nrows, D)) * 0.3).astype(np.float32)
    inv = np.arange(nrows, dtype=np.int32)
    g = torch.zeros((nrows, D), device=dev)
    loss, pairs = torch.zeros(256 * 32, device=dev), torch.zeros(256 * 32, device=dev)
    tu, ti, tm = (torch.from_numpy(U).to(dev), torch.from_numpy(inv).to(dev),
                  torch.from_numpy(meta).to(dev))
    p = ti.data_ptr()
    npp = 5 / S
    hip().w2v_win(p, p + B * 4, p + (B + R) * 4, tm.data_ptr(), B, W, D, npp, tu.data_ptr(),
                  g.data_ptr(), loss.data_ptr(), pairs.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    G = g.cpu().numpy().astype(np.float64)
    mask = window_pairs_reference(meta, B, W)
    ref = np.zeros((nrows, D))
    tot, npairs = 0.0, 0.0
    for t in range(tiles):
        c0, c1 = t * T, min(B, t * T + T)
        q0, q1 = c0, min(R, c0 + T + 2 * W)
        l, n, gV, gU, gN = sgns_window_reference(U[c0:c1], U[B + q0:B + q1],
                                                 U[B + R + t * S:B + R + (t + 1) * S],
                                                 mask[c0:c1, q0:q1], npp)
        tot, npairs = tot + l, npairs + n
        ref[c0:c1] += gV
        ref[B + q0:B + q1] += gU
        ref[B + R + t * S:B + R + (t + 1) * S] += gN
    assert mask.sum() == npairs > 0
    assert pairs.sum().item() == npairs
    # bf16 rows (8 mantissa bits) in every GEMM, fp32 accumulation
    np.testing.assert_allclose(G, ref, rtol=3e-2, atol=1e-2)
    np.testing.assert_allclose(loss.sum().item(), tot, rtol=3e-3)
    # centers without a valid pair and masked positions get no gradient
    dead = ~mask.any(1)
    assert not G[:B][dead].any()
    assert not G[B:B + R][meta < 0].any()


@pytest.mark.parametrize("D,W,K,B", [(32, 2, 3, 70), (64, 5, 5, 128), (128, 5, 5, 200),
                                     (128, 15, 16, 40)])
def test_w2v_per_pair_negatives_match_reference(dev, D, W, K, B):
    """Classic SGNS (k_w2v_pp + k_w2v_ppctx): K negatives per positive pair,
    gradients as occurrence rows.  The center rows and the run-position rows
    (summed over the 2W centers that pair with them) as rows, every negative
    occurrence as its (gn, center) pair — its row is gn * v_center — vs the
    fp64 reference; invalid pairs and masked positions get zero gradients."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.word2vec import sgns_pp_reference, window_pairs_reference

    R = B + 2 * W
    rng = np.random.default_rng(D + W + K)
    tags = np.cumsum(rng.random(R) < 0.08)
    bs = rng.integers(1, W + 1, R)
    meta = ((tags << 4) | bs).astype(np.int32)
    meta[rng.random(R) < 0.1] = -1
    nneg = B * 2 * W * K
    nrows = B + R + nneg
    U = (rng.standard_normal((nrows, D)) * 0.3).astype(np.float32)
    inv = np.arange(nrows, dtype=np.int32)
    og = torch.full((B + R, D), float("nan"), device=dev)  # every row must be written
    gnc = torch.full((nneg, 2), float("nan"), device=dev)
    gp = torch.empty(B * 2 * W, device=dev)
    loss, pairs = torch.zeros(256 * 32, device=dev), torch.zeros(256 * 32, device=dev)
    tu, ti, tm = (torch.from_numpy(U).to(dev), torch.from_numpy(inv).to(dev),
                  torch.from_numpy(meta).to(dev))
    p = ti.data_ptr()
    hip().w2v_pp(p, p + B * 4, p + (B + R) * 4, tm.data_ptr(), B, W, K, D, tu.data_ptr(),
                 og.data_ptr(), gp.data_ptr(), loss.data_ptr(), pairs.data_ptr(),
                 torch.cuda.current_stream().cuda_stream, gnc.data_ptr())
    torch.cuda.synchronize()
    gn = gnc.cpu().numpy()
    cen = gn[:, 1].copy().view(np.uint32)
    assert np.isfinite(gn[:, 0]).all()
    live = cen != 0xFFFFFFFF
    assert (gn[~live, 0] == 0).all()
    Gneg = np.zeros((nneg, D))
    Gneg[live] = gn[live, 0:1].astype(np.float64) * U[cen[live].astype(np.int64)]
    G = np.concatenate([og.cpu().numpy().astype(np.float64), Gneg])
    assert np.isfinite(G).all()
    band = window_pairs_reference(meta, B, W)  # [B, R]
    offs = [o - W if o < W else o - W + 1 for o in range(2 * W)]
    qidx = np.arange(B)[:, None] + W + np.array(offs)[None, :]  # [B, 2W] run positions
    mask = band[np.arange(B)[:, None], qidx]
    V = U[:B]
    Uc = U[B + qidx]
    N = U[B + R:].reshape(B, 2 * W, K, D)
    l, gV, gU, gN = sgns_pp_reference(V, Uc, N, mask)
    ref = np.zeros((nrows, D))
    ref[:B] = gV
    np.add.at(ref, B + qidx.reshape(-1), gU.reshape(-1, D))
    ref[B + R:] = gN.reshape(-1, D)
    assert mask.sum() > 0 and pairs.sum().item() == mask.sum()
    np.testing.assert_allclose(G, ref, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(loss.sum().item(), l, rtol=1e-4)


def test_w2v_stream_gen_window_layout(dev):
    """Synthetic stream (k_w2v_stream_gen): centers are the run's middle
    positions, sentence tags follow the position, reduced windows in [1, W],
    and the runs of consecutive steps overlap consistently by 2W positions."""
    from swiftsnails_amd.models.word2vec import OUT_BIT, W2VSynth

    d = W2VSynth(batch_size=256, window=4, vocab=10000, sentence_len=10)
    R, B, W = d.run_len, d.batch_size, d.window
    out = []
    for step in (0, 1):
        keys = torch.empty(d.n_keys, dtype=torch.int64, device=dev)
        meta = torch.empty(R, dtype=torch.int32, device=dev)
        d.generate(step, 0, 1, keys, meta=meta)
        torch.cuda.synchronize()
        out.append((keys.cpu().numpy(), meta.cpu().numpy()))
    (k0, m0), (k1, m1) = out
    ob = 1 << OUT_BIT
    for k, m, step in ((k0, m0, 0), (k1, m1, 1)):
        run = k[B:B + R]
        assert ((run & ob) != 0).all() and ((k[:B] & ob) == 0).all()
        np.testing.assert_array_equal(k[:B], run[W:W + B] & ~ob)
        assert (((k[B + R:] & ob) != 0)).all() and ((k[B + R:] & ~ob) < d.vocab).all()
        g = step * B - W + np.arange(R)
        valid = g >= 0
        assert (m[~valid] == -1).all()
        mv = m[valid].astype(np.int64)
        np.testing.assert_array_equal(mv >> 4, g[valid] // d.sentence_len)
        assert ((mv & 15) >= 1).all() and ((mv & 15) <= W).all()
    # step 1's first 2W positions are step 0's last 2W
    np.testing.assert_array_equal(k1[B:B + 2 * W], k0[B + B:B + B + 2 * W])
    np.testing.assert_array_equal(m1[:2 * W], m0[B:B + 2 * W])


@pytest.mark.parametrize("mode", ["window", "pairs"])
def test_word2vec_modes_train(dev, mode):
    """Both batch layouts train (loss per pair falls); the window layout
    counts its pairs on the device (~B x (W + 1) minus sentence edges) and
    carries B + 2W context keys instead of 2W per center."""
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    data = W2VSynth(batch_size=2048, window=3, vocab=5000, noise=0.05, mode=mode)
    opt, init = make_w2v_table_args(64, None)
    table = HbmTable(64, 40000, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, None, max_keys=data.n_keys, dim=64, device=dev)
    w = Word2VecWorker(eng, data)
    losses = []
    for _ in range(40):
        w.step()
        losses.append(w.mean_loss())
    table.check()
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < 0.85 * np.mean(losses[:3]), losses
    if mode == "window":
        assert data.n_keys == 2048 + 2048 + 6 + 32 * 64
        assert w.samples_per_step() == 2048
        n = w.step_pairs()
        assert 0.7 * 2048 * 4 < n <= 2048 * 6, n
    else:
        assert w.step_pairs() == 2048 * 6


def test_w2v_sgns_duplicate_rows_accumulate(dev):
    """Repeated words (same unique row) must receive the SUM of their grads."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.word2vec import sgns_reference

    T, C, S, D = 64, 2, 64, 32
    rng = np.random.default_rng(5)
    nrows = 40
    U = (rng.standard_normal((nrows, D)) * 0.3).astype(np.float32)
    inv = rng.integers(0, nrows, size=T + T * C + S).astype(np.int32)
    g = torch.zeros((nrows, D), device=dev)
    ti = torch.from_numpy(inv).to(dev)
    tu = torch.from_numpy(U).to(dev)
    p = ti.data_ptr()
    hip().w2v_sgns(p, p + T * 4, p + T * (1 + C) * 4, T, C, D, 0.5, tu.data_ptr(), g.data_ptr(),
                   0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    V, X, N = U[inv[:T]], U[inv[T:T + T * C]].reshape(T, C, D), U[inv[T + T * C:]]
    _, gV, gX, gN = sgns_reference(V, X, N, 0.5)
    ref = np.zeros((nrows, D))
    np.add.at(ref, inv[:T], gV)
    np.add.at(ref, inv[T:T + T * C], gX.reshape(-1, D))
    np.add.at(ref, inv[T + T * C:], gN)
    np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=5e-4, atol=5e-5)


@pytest.mark.parametrize("dim", [2, 5, 9, 17])
def test_fm_fwd_bwd_matches_reference(dev, dim):
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.fm import fm_reference

    B, F = 1000, 13
    rng = np.random.default_rng(dim)
    U = B * F  # unique row per occurrence: exact per-row gradient check
    rows = (rng.standard_normal((U, dim)) * 0.2).astype(np.float32)
    inv = np.arange(U, dtype=np.int32)
    y = (rng.random(B) < 0.4).astype(np.float32)
    tr, ti, ty = (torch.from_numpy(a).to(dev) for a in (rows, inv, y))
    g = torch.zeros((U, dim), device=dev)
    loss = torch.zeros(256 * 32, device=dev)
    pred = torch.empty(B, device=dev)
    hip().fm_fwd_bwd(ti.data_ptr(), ty.data_ptr(), B, F, dim, tr.data_ptr(), g.data_ptr(),
                     loss.data_ptr(), pred.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    l, p, gr = fm_reference(rows.reshape(B, F, dim), y)
    np.testing.assert_allclose(pred.cpu().numpy(), p, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.sum().item(), l, rtol=1e-4)
    np.testing.assert_allclose(g.cpu().numpy().reshape(B, F, dim), gr, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("dim,nranks", [(9, 1), (5, 3), (17, 1)])
def test_fm_bucket_reduce_matches_atomic_path(dev, dim, nranks):
    """Atomic-free FM (lane-group forward + per-bucket LDS row reduction) ==
    the per-occurrence atomic kernel, with heavy key duplication."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.parallel.router import HashFrag

    h = hip()
    B, F = 6000, 20
    n = B * F
    rng = np.random.default_rng(dim + nranks)
    keys = (rng.zipf(1.3, n) % 50000).astype(np.int64)
    fm = HashFrag(nranks, 64).rank_map()
    d = Deduper(n, nranks=nranks, frag_map=torch.from_numpy(fm.astype(np.int32)), gdim=dim,
                device=dev, mode="bucket")
    r = d(torch.from_numpy(keys).to(dev))
    st = torch.cuda.current_stream().cuda_stream
    U = nranks * d.ucap
    uvals = torch.randn(U, dim, device=dev) * 0.1
    y = torch.from_numpy((rng.random(B) < 0.4).astype(np.float32)).to(dev)
    g_at = torch.zeros(U, dim, device=dev)
    l_at = torch.zeros(256 * 32, device=dev)
    h.fm_fwd_bwd(r.inv.data_ptr(), y.data_ptr(), B, F, dim, uvals.data_ptr(), g_at.data_ptr(),
                 l_at.data_ptr(), 0, st)
    gs = torch.empty(B, device=dev)
    gss = torch.empty(B * (dim - 1), device=dev)
    g_b = torch.full((U, dim), float("nan"), device=dev)
    l_b = torch.zeros(256 * 32, device=dev)
    h.fm_fwd_g(0, d.index_ptrs(n), y.data_ptr(), B, F, dim,
               uvals.data_ptr(), gs.data_ptr(), gss.data_ptr(), l_b.data_ptr(), 0, st)
    h.bd_reduce_fm(n, nranks, d.scratch.data_ptr(), d.pj.data_ptr(), d.luid.data_ptr(),
                   gs.data_ptr(), gss.data_ptr(), F, dim, uvals.data_ptr(), g_b.data_ptr(), st,
                   ndest=d.ndest)
    # the sorted-list form (default with an overflow list)
    ovf = torch.zeros(h.bd_fm_ovf_words(n), dtype=torch.int32, device=dev)
    g_s = torch.full((U, dim), float("nan"), device=dev)
    h.bd_reduce_fm(n, nranks, d.scratch.data_ptr(), d.pj.data_ptr(), d.luid.data_ptr(),
                   gs.data_ptr(), gss.data_ptr(), F, dim, uvals.data_ptr(), g_s.data_ptr(), st,
                   ovf.data_ptr(), ndest=d.ndest)
    torch.cuda.synchronize()
    uc = r.ucount.cpu().numpy()
    for q in range(nranks):
        a, b = q * d.ucap, q * d.ucap + uc[q]
        ref = g_at[a:b].cpu().numpy()
        for got in (g_b[a:b].cpu().numpy(), g_s[a:b].cpu().numpy()):
            # fp32 sums in different orders (LDS atomics, sorted lists, global
            # atomics): a Zipf-head key sums hundreds of mixed-sign terms, so
            # a rare coordinate cancels to a few 1e-3 relative (seen: 1 of
            # 177701 at 2.6e-3); nearly all tight, every one loosely
            assert np.isclose(got, ref, rtol=2e-3, atol=2e-4).mean() > 0.9999
            np.testing.assert_allclose(got, ref, rtol=2e-2, atol=2e-3)
    np.testing.assert_allclose(l_b.sum().item(), l_at.sum().item(), rtol=1e-4)


@pytest.mark.parametrize("dim", [5, 9])
def test_fm_sorted_reduce_overflow_buckets(dev, dim):
    """Sorted-list FM reduce with buckets too large to sort in LDS (a key
    with 30K occurrences): those go to the LDS-atomic form; both == the
    per-occurrence atomic kernel."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper

    h = hip()
    B, F = 16000, 8
    n = B * F
    rng = np.random.default_rng(17)
    keys = rng.integers(0, 1 << 40, size=n).astype(np.int64)
    keys[rng.random(n) < 0.25] = 12345  # ~32K occurrences of one key
    d = Deduper(n, nranks=1, gdim=dim, device=dev, mode="bucket")
    r = d(torch.from_numpy(keys).to(dev))
    st = torch.cuda.current_stream().cuda_stream
    U = d.ucap
    uvals = torch.randn(U, dim, device=dev) * 0.1
    y = torch.from_numpy((rng.random(B) < 0.4).astype(np.float32)).to(dev)
    g_at = torch.zeros(U, dim, device=dev)
    h.fm_fwd_bwd(r.inv.data_ptr(), y.data_ptr(), B, F, dim, uvals.data_ptr(), g_at.data_ptr(),
                 0, 0, st)
    gs = torch.empty(B, device=dev)
    gss = torch.empty(B * (dim - 1), device=dev)
    h.fm_fwd_g(0, d.index_ptrs(n), y.data_ptr(), B, F, dim,
               uvals.data_ptr(), gs.data_ptr(), gss.data_ptr(), 0, 0, st)
    ovf = torch.zeros(h.bd_fm_ovf_words(n), dtype=torch.int32, device=dev)
    g_s = torch.full((U, dim), float("nan"), device=dev)
    h.bd_reduce_fm(n, 1, d.scratch.data_ptr(), d.pj.data_ptr(), d.luid.data_ptr(),
                   gs.data_ptr(), gss.data_ptr(), F, dim, uvals.data_ptr(), g_s.data_ptr(), st,
                   ovf.data_ptr(), ndest=d.ndest)
    torch.cuda.synchronize()
    assert int(ovf[0]) >= 1  # the hot key's bucket overflowed
    u = int(r.ucount[0])
    np.testing.assert_allclose(g_s[:u].cpu().numpy(), g_at[:u].cpu().numpy(), rtol=2e-3,
                               atol=5e-3)


def test_fm_trains_world1(dev):
    from swiftsnails_amd.models.fm import FMWorker, fm_table_args
    from swiftsnails_amd.models.sparse_lr import CtrSynth
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    data = CtrSynth(batch_size=4096, num_fields=16, num_features=100_000, tail_frac=0.0)
    opt, init = fm_table_args(8)
    table = HbmTable(9, 200_000, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, None, max_keys=4096 * 16, dim=9, device=dev)
    w = FMWorker(eng, data)
    losses = [float(w.step().sum().item()) / 4096 for _ in range(50)]
    table.check()
    assert np.mean(losses[-5:]) < np.mean(losses[:3]) - 0.02, losses


def test_word2vec_trains_world1(dev):
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    data = W2VSynth(batch_size=2048, window=3, vocab=5000, noise=0.05)
    opt, init = make_w2v_table_args(64, None)
    table = HbmTable(64, 40000, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, None, max_keys=data.n_keys, dim=64, device=dev)
    w = Word2VecWorker(eng, data)
    losses = []
    for _ in range(40):
        w.step()
        losses.append(w.mean_loss())
    table.check()
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < 0.8 * np.mean(losses[:3]), losses


def _graph_worker(model, dev, **ek):
    from swiftsnails_amd.models.fm import FMWorker, fm_table_args
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    if model == "lr":
        data = CtrSynth(batch_size=4096, num_fields=13, num_features=1_000_000, tail_frac=0.1)
        table = make_lr_table(data.num_features, 1, Optimizer("adagrad", lr=0.1), device=dev)
        eng = PSEngine(table, ek.pop("transport", None), max_keys=4096 * 13, dim=1, device=dev,
                       **ek)
        return SparseLRWorker(eng, data), table
    if model == "fm":
        data = CtrSynth(batch_size=2048, num_fields=16, num_features=100_000, tail_frac=0.1)
        opt, init = fm_table_args(8)
        table = HbmTable(9, 200_000, optimizer=opt, init=init, device=dev)
        eng = PSEngine(table, ek.pop("transport", None), max_keys=2048 * 16, dim=9, device=dev,
                       **ek)
        return FMWorker(eng, data), table
    data = W2VSynth(batch_size=1024, window=3, vocab=5000, noise=0.05,
                    mode="pairs" if model == "w2v_pairs" else "window")
    opt, init = make_w2v_table_args(64, None)
    table = HbmTable(64, 40000, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, ek.pop("transport", None), max_keys=data.n_keys, dim=64, device=dev, **ek)
    return Word2VecWorker(eng, data), table


def test_graph_capture_after_mode_switch_xgmi(dev):
    """N>1 path (a size-1 xGMI arena): pulled-ahead rounds, then synchronous
    ones (the launcher calibration's last switch), then the hipGraph capture.
    Synchronous rounds run the keys wait + server merge in their routes; the
    capture must start from a round routed that way (enable_graph settles one
    eager step), else every replay's first pull waits a second time on its
    slot's keys and the job hangs (here: a mailbox timeout).  (Graph tests run
    in a child process: tests/_mp.py in_child.)"""
    in_child(_graph_after_mode_switch_body, dev)


def _graph_after_mode_switch_body(dev):
    os.environ["SS_XGMI_TIMEOUT"] = "20"
    os.environ["SS_PULL_AHEAD"] = "auto"
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    torch.cuda.set_device(dev)
    w, t = _graph_worker("w2v", dev, transport=XgmiTransport(0, 1, dev, None))
    assert w.set_pull_ahead(True)
    for _ in range(3):
        w.step()
    w.set_pull_ahead(False)
    w.drain()
    assert w.enable_graph()
    assert w.engine.last_route_matches()
    for _ in range(3 * w._gper):
        w.step()
    torch.cuda.synchronize()
    w.engine.check()
    t.check()
    assert np.isfinite(w.mean_loss())


def test_graph_teardown_then_replay_same_process(dev, monkeypatch):
    """The hipGraph teardown order: a worker with captured graphs
    on the N>1 path (a size-1 xGMI arena: mailbox puts / waits and the round
    engine's events in the graph) is dropped inside a reference cycle
    without close(), and the cyclic GC collects it while a second worker's
    graphs are replaying in the same process.  The graphs are reset before the engine's events and
    arenas go away (models/base.py _GraphSet), so the replays go on and the
    second worker trains; the first worker's graphs trained as well."""
    import gc

    monkeypatch.setenv("SS_XGMI_TIMEOUT", "20")
    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    torch.cuda.set_device(dev)
    a, ta = _graph_worker("lr", dev, transport=XgmiTransport(0, 1, dev, None))
    first = [float(a.step().sum().item()) for _ in range(2)]
    assert a.enable_graph()
    for _ in range(3 * a._gper):
        a.step()
    torch.cuda.synchronize()
    a.engine.check()
    ta.check()
    assert np.isfinite(a.mean_loss()) and a.mean_loss() < first[0]
    a.cycle = a  # only the cyclic GC can free it now
    del a, ta
    b, tb = _graph_worker("lr", dev)
    b.step()
    assert b.enable_graph()
    for i in range(4 * b._gper):
        b.step()
        if i == b._gper:
            gc.collect()  # the first worker goes while these replays run
    torch.cuda.synchronize()
    tb.check()
    b.engine.check()
    assert np.isfinite(b.mean_loss()) and 0 < b.mean_loss() < 0.7
    b.close()  # explicit teardown; eager steps still work afterwards
    b.step()
    torch.cuda.synchronize()
    assert np.isfinite(b.mean_loss())


@pytest.mark.parametrize("occ", ["own", "arena"])
def test_record_exchange_world1_matches_unique(dev, monkeypatch, occ):
    """The record exchange (every occurrence shipped; the server dedups what
    it receives, fills a row per occurrence and merges the per-occurrence
    gradients with the AdaGrad update fused — no worker dedup or merge)
    through a size-1 xGMI arena trains like the unique-key exchange on the
    same path: the same keys, the same losses and parameters up to float
    summation order (SS_REC_OCC: own = the own records' rows in a cached
    buffer and their gradients read through spj by the server merge; arena =
    through the mailbox).  Graph tests run in a child process (tests/_mp.py)."""
    in_child(_record_exchange_body, dev, occ)


def _record_exchange_body(dev, occ):
    os.environ["SS_ENGINE_GENERAL"] = "xgmi"
    os.environ["SS_PULL_AHEAD"] = "0"
    os.environ["SS_REC_OCC"] = occ
    os.environ["SS_XGMI_TIMEOUT"] = "30"
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    torch.cuda.set_device(dev)
    out = {}
    for ex in ("unique", "records"):
        w, t = _graph_worker("lr", dev, transport=XgmiTransport(0, 1, dev, None), exchange=ex)
        assert w.engine.records == (ex == "records")
        assert (w.gring is not None) == (ex == "records" and occ == "own")
        losses = [float(w.step().sum().item()) for _ in range(12)]
        torch.cuda.synchronize()
        w.engine.check()
        t.check()
        out[ex] = (losses, t.to_dict(with_state=True))
        if ex == "records":  # the record round captured as hipGraphs
            assert w.enable_graph()
            for _ in range(2 * w._gper):
                w.step()
            torch.cuda.synchronize()
            w.engine.check()
            t.check()
            assert np.isfinite(w.mean_loss()) and 0 < w.mean_loss() < 0.7
    (lu, tu), (lr_, tr) = out["unique"], out["records"]
    np.testing.assert_allclose(lr_, lu, rtol=1e-4, atol=1e-5)
    assert tr.keys() == tu.keys()
    ks = list(tu.keys())
    a, b = np.stack([tu[k] for k in ks]), np.stack([tr[k] for k in ks])
    np.testing.assert_allclose(b, a, rtol=1e-3, atol=1e-5)


def test_lr_slot32_matches_slot64(dev, monkeypatch):
    """One-GPU sparse LR with the pull storing 4-byte slot indices for the
    fused merge + AdaGrad update (default, shards under 2^31 slots) trains
    exactly like 8-byte slots: same per-step losses, same table."""
    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    out = {}
    for s32 in ("1", "0"):
        monkeypatch.setenv("SS_SLOT32", s32)
        w, t = _graph_worker("lr", dev)
        assert w.engine.slot32 == (s32 == "1")
        w.step()
        # zero-initialised weights: every logit 0, the first step's loss is
        # ln 2 per sample — moved out of the forward's accumulator by the
        # merge kernel, which leaves the accumulator zero
        assert abs(w.mean_loss() - np.log(2.0)) < 1e-4
        assert float(w._acc.abs().sum()) == 0.0
        losses = [float(w.step().sum().item()) for _ in range(6)]
        torch.cuda.synchronize()
        t.check()
        out[s32] = (losses, t.to_dict(with_state=True))
    (l1, d1), (l0, d0) = out["1"], out["0"]
    np.testing.assert_allclose(l1, l0, rtol=1e-5, atol=1e-6)
    assert d1.keys() == d0.keys()
    ks = list(d0.keys())
    np.testing.assert_allclose(np.stack([d1[k] for k in ks]), np.stack([d0[k] for k in ks]),
                               rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model", ["lr", "fm", "w2v", "w2v_pairs"])
def test_hipgraph_replay_matches_eager(dev, model):
    """hipGraph replays (one graph per ring phase, device step counter for
    the generator) train exactly like eager steps: same per-step losses and
    the same table (up to float-atomic summation order).  Pull-ahead is off
    here: with it, which of round i's updates round i+1 reads depends on
    timing (staleness 1), in eager mode as much as in graphs.  (In a child
    process: tests/_mp.py in_child.)"""
    in_child(_replay_matches_eager_body, dev, model)


def _replay_matches_eager_body(dev, model):
    os.environ["SS_PULL_AHEAD"] = "0"
    torch.cuda.set_device(dev)
    wb, tb = _graph_worker(model, dev)
    lb = [float(wb.step().sum().item())]
    assert wb.enable_graph()
    per = wb._gper  # steps per graph (SS_GRAPH_STEPS; default 4 ring periods)
    n = 1 + 3 * per
    lb += [float(wb.step().sum().item()) for _ in range(n - 1)]
    wa, ta = _graph_worker(model, dev)
    la = [float(wa.step().sum().item()) for _ in range(n)]
    torch.cuda.synchronize()
    ta.check()
    tb.check()
    # a multi-step graph (SS_GRAPH_STEPS) leaves the loss of its last step
    idx = [0] + [k for k in range(1, n) if (k - 1) % per == per - 1]
    np.testing.assert_allclose(np.array(lb)[idx], np.array(la)[idx], rtol=2e-4, atol=1e-3)
    da, db = ta.to_dict(), tb.to_dict()
    assert da.keys() == db.keys()
    ks = list(da.keys())[:5000]
    a, b = np.stack([da[k] for k in ks]), np.stack([db[k] for k in ks])
    # float-atomic summation order differs between any two runs; AdaGrad's
    # division by a still-small accumulator amplifies it for a rare
    # coordinate: a near-zero summed gradient whose sign depends on the order
    # moves the weight by +-lr on its first update (seen: 1 of 320000 off by
    # 0.05 at lr 0.05).  So: nearly all coordinates tight, and every
    # coordinate within the largest AdaGrad excursion, |step| <= lr per round
    assert np.isclose(b, a, rtol=1e-3, atol=5e-4).mean() >= 0.9995
    np.testing.assert_allclose(b, a, rtol=0, atol=2 * ta.opt.lr * n)


@pytest.mark.parametrize("model", ["fm", "w2v", "w2v_pairs"])
def test_hipgraph_pull_ahead_trains(dev, model):
    """Graph replays of the pull-ahead pipeline (rows of round i+1 pulled on
    the route stream while round i computes) keep training.  (In a child
    process: tests/_mp.py in_child.)"""
    in_child(_pull_ahead_trains_body, dev, model)


def _pull_ahead_trains_body(dev, model):
    torch.cuda.set_device(dev)
    w, t = _graph_worker(model, dev)
    assert w.engine.pull_ahead
    first = [float(w.step().sum().item()) for _ in range(3)]
    assert w.enable_graph()
    last = [float(w.step().sum().item()) for _ in range(30)]
    torch.cuda.synchronize()
    t.check()
    assert np.isfinite(last).all()
    assert np.mean(last[-5:]) < np.mean(first), (first, last[-5:])


@pytest.mark.parametrize("D,B,W", [(128, 1000, 5), (32, 640, 2), (64, 4096, 15)])
def test_word2vec_window_grad_reduce_matches_atomics(dev, monkeypatch, D, B, W):
    """Window tile gradients as occurrence rows summed per unique key
    (k_w2v_osort + k_w2v_oreduce: counting sort per dedup bucket, one wave per
    <= 32-occurrence item, shared window rows through the tail buffer, Zipf
    heads split over several items) == the tile's own row atomics; the
    per-step loss moved out of the zeroed accumulator by the reduce == the
    zero-filled one.  Partial
    last tile (B % 64 != 0), W from 2 to the maximum 15.  (The atomic form
    is what a non-bucketed dedup, SS_DEDUP=hash, runs.)"""
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    out = {}
    for mode in ("reduce", "atomic"):
        monkeypatch.setenv("SS_DEDUP", "bucket" if mode == "reduce" else "hash")
        data = W2VSynth(batch_size=B, window=W, vocab=3000, noise=0.05, mode="window")
        opt, init = make_w2v_table_args(D, None)
        t = HbmTable(D, 40000, optimizer=opt, init=init, device=dev)
        eng = PSEngine(t, None, max_keys=data.n_keys, dim=D, device=dev)
        w = Word2VecWorker(eng, data)
        assert w.occ_reduce == (mode == "reduce")
        losses = []
        for _ in range(5):
            w.step()
            losses.append(w.mean_loss())
        torch.cuda.synchronize()
        t.check()
        if mode == "reduce":  # k_w2v_oreduce handed the accumulators off and zeroed them
            assert w._out is not w._acc and float(w._acc.abs().sum()) == 0.0
        out[mode] = (losses, t.to_dict(with_state=True))
    (lr, tr), (la, ta) = out["reduce"], out["atomic"]
    np.testing.assert_allclose(lr, la, rtol=1e-4)
    assert tr.keys() == ta.keys()
    ks = list(tr.keys())
    a, b = np.stack([ta[k] for k in ks]), np.stack([tr[k] for k in ks])
    assert np.isclose(b, a, rtol=1e-3, atol=5e-4).mean() > 0.9999
    np.testing.assert_allclose(b, a, rtol=5e-2, atol=2e-2)


@pytest.mark.parametrize("comms", [1, 3])
@pytest.mark.parametrize("model", ["lr", "fm", "w2v"])
def test_general_path_rccl_world1_matches_loopback(dev, model, comms, monkeypatch):
    """The N>1 engine path (send segments, count exchange with pinned D2H,
    bucket runs, the server's merge of received keys and merged update) on
    one GPU through real size-1 RCCL communicators — one on its comm stream
    (SS_RCCL_COMMS=1) or three on the engine's streams (3) — trains exactly
    like the same path over loopback transports: the multi-GPU RCCL call
    sequence, minus peers."""
    monkeypatch.setenv("SS_ENGINE_GENERAL", "1")
    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    n = 12
    wa, ta = _graph_worker(model, dev)
    assert not wa.engine.fast1
    la = [float(wa.step().sum().item()) for _ in range(n)]
    wb, tb = _graph_worker(model, dev, **_rccl1(dev, comms))
    lb = [float(wb.step().sum().item()) for _ in range(n)]
    torch.cuda.synchronize()
    ta.check()
    tb.check()
    np.testing.assert_allclose(lb, la, rtol=2e-4, atol=1e-3)
    assert ta.size() == tb.size()


def _rccl1(dev, comms=1):
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.parallel.transport import RcclTransport

    if comms == 1:
        t = RcclTransport(0, 1, dev, uid=hip().RcclComm.unique_id())
        assert t.nranks() == 1
        return {"transport": t}
    t, c, p = (RcclTransport(0, 1, dev, uid=hip().RcclComm.unique_id(), serial=False)
               for _ in range(3))
    return {"transport": t, "count_transport": c, "pull_transport": p}


@pytest.mark.parametrize("comms", [1, 3])
@pytest.mark.parametrize("model", ["lr", "fm", "w2v"])
def test_general_path_rccl_world1_pull_ahead_trains(dev, model, comms, monkeypatch):
    """The production N>1 pipeline — pull-ahead of round i+1 on a third
    stream while round i computes, the server's update a read-modify-write —
    on one GPU through size-1 RCCL communicators: trains and keeps the table
    sane."""
    monkeypatch.setenv("SS_ENGINE_GENERAL", "1")
    monkeypatch.setenv("SS_PULL_AHEAD", "1")  # LR runs synchronous rounds by default
    w, t = _graph_worker(model, dev, **_rccl1(dev, comms))
    assert w.engine.pull_ahead and w.engine.pull_stream is not None
    losses = [float(w.step().sum().item()) for _ in range(40)]
    torch.cuda.synchronize()
    t.check()
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < np.mean(losses[:3]), losses


@pytest.mark.parametrize("dim", [5, 9])
def test_fm_fused_update_matches_separate_apply(dev, dim):
    """bd_reduce_fm with the fused optimizer update (sorted lists and the
    overflow bucket of a 32K-occurrence key) leaves the table exactly as the
    gradient store followed by k_apply."""
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.ops.dedup import Deduper
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable

    h = hip()
    B, F = 16000, 8
    n = B * F
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 1 << 40, size=n).astype(np.int64)
    keys[rng.random(n) < 0.25] = 12345
    d = Deduper(n, nranks=1, gdim=dim, device=dev, mode="bucket")
    r = d(torch.from_numpy(keys).to(dev))
    st = torch.cuda.current_stream().cuda_stream
    u = int(r.ucount[0])
    uk = r.ukeys[:u].clone()
    tabs, slots = [], []
    for _ in range(2):
        t = HbmTable(dim, 1 << 18, optimizer=Optimizer("adagrad", lr=0.2),
                     init=InitConfig("uniform", 0.1, 0.1, seed=7), device=dev)
        v, s = t.pull(uk, unique=True)
        tabs.append(t)
        slots.append(s)
    uvals = torch.zeros(d.ucap, dim, device=dev)
    uvals[:u] = v
    y = torch.from_numpy((rng.random(B) < 0.4).astype(np.float32)).to(dev)
    gs = torch.empty(B, device=dev)
    gss = torch.empty(B * (dim - 1), device=dev)
    h.fm_fwd_g(0, d.index_ptrs(n), y.data_ptr(), B, F, dim,
               uvals.data_ptr(), gs.data_ptr(), gss.data_ptr(), 0, 0, st)
    ovf = torch.zeros(h.bd_fm_ovf_words(n), dtype=torch.int32, device=dev)
    g = torch.zeros(d.ucap, dim, device=dev)
    args = (n, 1, d.scratch.data_ptr(), d.pj.data_ptr(), d.luid.data_ptr(), gs.data_ptr(),
            gss.data_ptr(), F, dim, uvals.data_ptr(), g.data_ptr(), st, ovf.data_ptr())
    h.bd_reduce_fm(*args)
    tabs[0].push_slots(slots[0][:u], g[:u].contiguous())
    h.bd_reduce_fm(*args, t=tabs[1].dt, slots=slots[1].data_ptr(), op=tabs[1].opt.native())
    torch.cuda.synchronize()
    assert int(ovf[0]) >= 1
    a, b = tabs[0].to_dict(with_state=True), tabs[1].to_dict(with_state=True)
    assert a.keys() == b.keys() and len(a) == u
    ks = list(a.keys())
    # rtol 3e-5: the hot key's 32000 occurrences are summed with LDS float
    # atomics in either order (one coordinate measured 1.05e-5 apart)
    np.testing.assert_allclose(np.stack([b[k] for k in ks]), np.stack([a[k] for k in ks]),
                               rtol=3e-5, atol=1e-6)


@pytest.mark.parametrize("pull_stream", ["0", "1"])
def test_fm_trains_with_pull_ahead_staleness_bound(dev, monkeypatch, pull_stream):
    """FM pulls round i+1 ahead on a side stream (the route stream, or its own
    with SS_PULL_STREAM=1), bounded to staleness exactly 1 (the pull waits for
    round i-1's push) — trains on both.  (Unbounded, a side stream running
    ahead read several rounds stale: on the bench configuration FM's loss then
    stayed at chance, 0.69; at this small size the unbounded run still trains,
    with larger early swings: 0.90 / 0.98 vs 0.64 / 0.77.)"""
    from swiftsnails_amd.models.fm import FMWorker, fm_table_args
    from swiftsnails_amd.models.sparse_lr import CtrSynth
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_PULL_STREAM", pull_stream)
    data = CtrSynth(batch_size=16384, num_fields=39, num_features=2_000_000, tail_frac=0.1)
    opt, init = fm_table_args(8)
    table = HbmTable(9, 4_000_000, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, None, max_keys=16384 * 39, dim=9, device=dev)
    w = FMWorker(eng, data)
    assert eng.pull_ahead and eng.staleness == 1
    assert (eng.pull_stream is not None) == (pull_stream == "1")
    losses = []
    for _ in range(60):
        w.step()
        losses.append(w.mean_loss())
    torch.cuda.synchronize()
    table.check()
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < min(0.66, np.mean(losses[5:10]) - 0.01), losses


def _bench_1gpu(extra):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + extra, cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_graph_mode_times_whole_periods():
    """bench.py --graph on: the timed region runs exactly --steps steps.  With
    16 timed steps the graph holds 16 steps (2 ring periods of the one-GPU
    8-slot ring, or 4 of a 4-slot one) and the warm-up one graph, so the job
    runs warmup + 16 + 16 steps in all — the same training as an eager run of
    warmup + 32 steps (identical final loss)."""
    base = ["--batch", "4096", "--features", "2000000", "--warmup", "3"]
    g = _bench_1gpu(base + ["--steps", "16", "--graph", "on"])
    e = _bench_1gpu(base + ["--steps", "32"])
    assert g["config"]["hipgraph"] is True and e["config"]["hipgraph"] is False
    assert g["steps"] == 16 and g["ms_per_step"] > 0
    assert g["config"]["loss_last"] == pytest.approx(e["config"]["loss_last"], rel=1e-4, abs=1e-5)


def _planted_corpus(path, clusters=20, words=40, sentences=6000, length=12, seed=5):
    """Sentences of one cluster each: word ids c*1000 + i (i < words)."""
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for _ in range(sentences):
            c = int(rng.integers(clusters))
            ids = c * 1000 + rng.integers(0, words, size=length)
            f.write(" ".join(str(int(x)) for x in ids) + "\n")
    return clusters, words


@pytest.mark.parametrize("mode,neg_mode,tile,rows", [("window", "shared", "bf16", "fp32"),
                                                     ("pairs", "shared", "bf16", "fp32"),
                                                     ("pairs", "shared", "f32", "fp32"),
                                                     ("window", "per_pair", "f32", "fp32"),
                                                     ("window", "shared", "bf16", "bf16"),
                                                     ("window", "per_pair", "f32", "bf16")])
def test_word2vec_learns_planted_clusters(dev, tmp_path, monkeypatch, mode, neg_mode, tile, rows):
    """Embedding quality, not just a falling loss: on a corpus whose
    sentences each draw from one of 20 word clusters, the learned input
    vectors of words of the same cluster are far more similar (cosine) than
    of words of different clusters — for every objective variant: the
    shared-negative tile (window layout: bf16 MFMA; pairs layout: bf16 and
    fp32 MFMA) and per-pair negatives (classic SGNS, fp32 dot products), on
    fp32 rows and on compact bf16 rows (row_dtype: bf16: updated in fp32 by the
    fused reduce, stored with stochastic rounding)."""
    from swiftsnails_amd.models.word2vec import Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.utils.dataio import FileCorpusSource

    monkeypatch.setenv("SS_W2V_MFMA", tile)
    C, M = _planted_corpus(tmp_path / "corpus.txt")
    data = FileCorpusSource(str(tmp_path / "corpus.txt"), batch_size=2048, window=4,
                            negatives=5, mode=mode, neg_mode=neg_mode, device=dev)
    opt, init = make_w2v_table_args(64, None)
    table = HbmTable(64, 1 << 14, optimizer=opt, init=init, device=dev, row_dtype=rows)
    eng = PSEngine(table, None, max_keys=data.n_keys, dim=64, device=dev)
    w = Word2VecWorker(eng, data)
    assert w.mfma_bf16 == (tile == "bf16") and w.per_pair == (neg_mode == "per_pair")
    assert getattr(w, "fuse", True)  # the reduce runs the update, fp32 or bf16 rows
    for _ in range(3 * data.steps_per_pass()):  # 3 passes
        w.step()
    torch.cuda.synchronize()
    table.check()
    ids = torch.tensor([c * 1000 + i for c in range(C) for i in range(M)], device=dev)
    v, _ = table.pull(ids, insert=False)
    v = torch.nn.functional.normalize(v.double(), dim=1).cpu().numpy()
    sim = v @ v.T
    lab = np.repeat(np.arange(C), M)
    same = lab[:, None] == lab[None, :]
    off = ~np.eye(len(lab), dtype=bool)
    within, across = sim[same & off].mean(), sim[~same].mean()
    assert within - across > 0.4, (within, across)
    # nearest neighbour of almost every word is in its own cluster
    np.fill_diagonal(sim, -2)
    assert (lab[sim.argmax(1)] == lab).mean() > 0.95


@pytest.mark.parametrize("row_dtype", ["fp32", "bf16"])
def test_fm_learns_planted_model_auc(dev, row_dtype):
    """FM held-out AUC against the planted model the labels come from (not
    only a falling loss), with full fp32 rows and with compact bf16 rows
    (config 5's capacity option): both learn to within 10% of the
    Bayes-optimal AUC, and compact rows lose < 0.01 AUC against fp32."""
    from swiftsnails_amd.models.fm import FMWorker, fm_table_args
    from swiftsnails_amd.models.sparse_lr import CtrSynth
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    res = {}
    for dt in sorted({"fp32", row_dtype}):
        data = CtrSynth(batch_size=4096, num_fields=16, num_features=16 * 4000, tail_frac=0.0,
                        truth_scale=4.0)
        opt, init = fm_table_args(8)
        opt.lr = 0.2
        table = HbmTable(9, 1 << 17, optimizer=opt, init=init, device=dev, row_dtype=dt)
        eng = PSEngine(table, None, max_keys=4096 * 16, dim=9, device=dev)
        w = FMWorker(eng, data)
        for _ in range(150):
            w.step()
        table.check()
        res[dt] = w.evaluate(batches=2)
    r = res[row_dtype]
    assert r["auc_truth"] > 0.8
    assert r["auc"] > 0.9 * r["auc_truth"], res
    assert r["auc"] > res["fp32"]["auc"] - 0.01, res


@pytest.mark.parametrize("opt", ["sgd", "adagrad"])
@pytest.mark.parametrize("neg_mode", ["shared", "per_pair"])
def test_w2v_fused_update_matches_apply(dev, monkeypatch, neg_mode, opt):
    """One-GPU word2vec with the optimizer update fused into the occurrence-row
    reduce (every key whose gradient row is one reduce item; the apply kernel
    masked to the keys summed over several items) trains like the reduce +
    apply pair (SS_W2V_FUSE=0): the same sums and update, up to the order of
    the hot keys' row atomics (run-to-run float noise, ~1e-6 relative).  SGD
    keeps that noise at its size (a few coordinates near cancellation: 2e-5).  AdaGrad's
    first step moves a coordinate by lr * sign(g), so a near-zero gradient
    whose sign the noise flips differs by up to 2 lr (a few hundred of 1.4M
    coordinates): 99.9 % within 1e-4, and no coordinate beyond 2 lr."""
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    monkeypatch.setenv("SS_PULL_AHEAD", "0")
    lr = 0.05
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("SS_W2V_FUSE", fuse)
        data = W2VSynth(batch_size=2048, window=3, vocab=20000, noise=0.05, mode="window",
                        neg_mode=neg_mode, negatives=5)
        opt_, init = make_w2v_table_args(64, Optimizer(opt, lr=lr))
        table = HbmTable(64, 200_000, optimizer=opt_, init=init, device=dev)
        eng = PSEngine(table, None, max_keys=data.n_keys, dim=64, device=dev)
        w = Word2VecWorker(eng, data)
        assert (w.uhot is not None) == (fuse == "1")
        losses = [None] * 0
        for _ in range(8):
            w.step()
            losses.append(w.mean_loss())
        torch.cuda.synchronize()
        table.check()
        out[fuse] = (losses, table.to_dict(with_state=True))
    (l1, t1), (l0, t0) = out["1"], out["0"]
    assert t1.keys() == t0.keys()
    np.testing.assert_allclose(np.array(l1), np.array(l0), rtol=1e-5)
    ks = list(t0)
    a, b = np.stack([t1[k] for k in ks]), np.stack([t0[k] for k in ks])
    if opt == "sgd":
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)
    else:
        close = np.isclose(a, b, rtol=1e-4, atol=1e-7)
        assert close.mean() > 0.999, (close.size - close.sum(), close.size)
        assert np.abs(a - b).max() <= 2 * lr + 1e-3
