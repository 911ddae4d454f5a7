"""Native data input (csrc/host/dataio.h): parsing parity with a Python reader,
sharding, batch padding, corpus sampling, and the pinned prefetch ring."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host():
    from swiftsnails_amd._native import host
    return host()


def _write_libsvm(path, rows=997, seed=0):
    rng = np.random.default_rng(seed)
    ref = []
    with open(path, "w") as f:
        for i in range(rows):
            n = int(rng.integers(0, 9))
            idx = rng.integers(0, 10**12, n)
            val = np.round(rng.standard_normal(n), 3)
            lab = int(rng.integers(0, 2)) * 2 - 1 if i % 3 else int(rng.integers(0, 2))
            toks = [f"{a}:{b}" if j % 2 else f"{a}" for j, (a, b) in enumerate(zip(idx, val))]
            f.write(f"{lab} " + " ".join(toks) + ("\r\n" if i % 7 == 0 else "\n"))
            vals = [float(b) if j % 2 else 1.0 for j, b in enumerate(val)]
            ref.append((1.0 if lab > 0 else 0.0, [int(a) for a in idx], vals))
    return ref


def test_libsvm_parse_matches_python(tmp_path):
    p = str(tmp_path / "a.svm")
    ref = _write_libsvm(p)
    for nthreads in (1, 3, 8):
        ds = _host().SparseDataset(p, "libsvm", nthreads, 0, 1)
        assert ds.rows == len(ref)
        offs = ds.offsets()
        keys, vals, labels = ds.keys(), ds.vals(), ds.labels()
        for r, (lab, idx, val) in enumerate(ref):
            a, b = int(offs[r]), int(offs[r + 1])
            assert labels[r] == lab
            assert keys[a:b].tolist() == idx
            np.testing.assert_allclose(vals[a:b], val, rtol=1e-6)
        assert ds.has_values
        assert ds.max_nnz == max(len(x[1]) for x in ref)


def test_shards_partition_rows(tmp_path):
    p = str(tmp_path / "a.svm")
    ref = _write_libsvm(p, rows=501, seed=3)
    for world in (2, 3, 5):
        got = []
        for r in range(world):
            ds = _host().SparseDataset(p, "libsvm", 2, r, world)
            offs, keys = ds.offsets(), ds.keys()
            got += [keys[int(offs[i]):int(offs[i + 1])].tolist() for i in range(ds.rows)]
        assert got == [x[1] for x in ref]  # contiguous shards, in file order


def test_ctr_tsv_fields_and_hashing(tmp_path):
    from swiftsnails_amd.utils.hashing import fmix64  # noqa: F401 (module import check)
    p = str(tmp_path / "a.tsv")
    lines = ["1\ta\tb\t\tc", "0\t\tx\ty\t", "1\tq"]
    with open(p, "w") as f:
        f.write("\n".join(lines) + "\n")
    ds = _host().SparseDataset(p, "ctr", 2, 0, 1)
    assert ds.rows == 3
    assert ds.labels().tolist() == [1.0, 0.0, 1.0]
    offs, keys = ds.offsets(), ds.keys()
    fields = [[int(k) >> 48 for k in keys[int(offs[i]):int(offs[i + 1])]] for i in range(3)]
    assert fields == [[0, 1, 3], [1, 2], [0]]
    # same token in the same field -> same key; different field -> different key
    k0 = keys[int(offs[0]):int(offs[1])]
    assert len(set(int(k) & ((1 << 48) - 1) for k in k0)) == 3
    assert not ds.has_values


def test_fill_pads_truncates_and_wraps(tmp_path):
    p = str(tmp_path / "a.svm")
    ref = _write_libsvm(p, rows=37, seed=5)
    ds = _host().SparseDataset(p, "libsvm", 4, 0, 1)
    B, F = 50, 4
    keys = np.empty(B * F, dtype=np.uint64)
    vals = np.empty(B * F, dtype=np.float32)
    labels = np.empty(B, dtype=np.float32)
    nxt = ds.fill(30, B, F, keys.ctypes.data, vals.ctypes.data, labels.ctypes.data, 3)
    assert nxt == (30 + B) % 37
    for b in range(B):
        lab, idx, val = ref[(30 + b) % 37]
        row = keys[b * F:(b + 1) * F]
        m = min(F, len(idx))
        assert row[:m].tolist() == idx[:m]
        assert (row[m:] == np.uint64(0xFFFFFFFFFFFFFFFF)).all()
        np.testing.assert_allclose(vals[b * F:b * F + m], val[:m], rtol=1e-6)
        assert (vals[b * F + m:(b + 1) * F] == 0).all()
        assert labels[b] == lab


def test_file_ctr_source_prefetch_cpu(tmp_path):
    from swiftsnails_amd.utils.dataio import FileCtrSource
    p = str(tmp_path / "a.svm")
    _write_libsvm(p, rows=123, seed=9)
    src = FileCtrSource(p, "libsvm", batch_size=16, num_fields=5, pin=False, prefetch=3,
                        resident="host")
    ds = _host().SparseDataset(p, "libsvm", 1, 0, 1)
    keys = torch.empty(16 * 5, dtype=torch.int64)
    labels = torch.empty(16)
    xval = torch.empty(16 * 5)
    for step in range(12):
        src.generate(step, 0, 1, keys, labels, xval=xval)
        ek = np.empty(80, dtype=np.uint64)
        ev = np.empty(80, dtype=np.float32)
        el = np.empty(16, dtype=np.float32)
        ds.fill((step * 16) % 123, 16, 5, ek.ctypes.data, ev.ctypes.data, el.ctypes.data, 1)
        assert keys.numpy().view(np.uint64).tolist() == ek.tolist()
        assert labels.numpy().tolist() == el.tolist()
        assert xval.numpy().tolist() == ev.tolist()
    src.close()


def test_corpus_and_skipgram_sampling(tmp_path):
    p = str(tmp_path / "w2v.txt")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_word2vec_data.py"), p,
                           "--lines", "500", "--seed", "1"])
    sents = [list(map(int, ln.split())) for ln in open(p)]
    c = _host().Corpus(p, 4, 0, 1, 1, 0.0)
    assert c.size == sum(len(s) for s in sents)
    assert c.sentences == len(sents)
    vocab = dict(c.vocab())
    assert sum(vocab.values()) == c.size
    assert max(vocab) <= 300
    B, W = 256, 3
    C = 2 * W
    nneg = 64
    keys = np.empty(B + B * C + nneg, dtype=np.uint64)
    c.fill_skipgram(7, 0, B, C, W, nneg, keys.ctypes.data, 4)
    out = np.uint64(1 << 40)
    centers, ctx, neg = keys[:B], keys[B:B + B * C], keys[B + B * C:]
    assert (ctx & out).all() and (neg & out).all() and not (centers & out).any()
    assert set((neg & ~out).tolist()) <= set(vocab)
    # every context is within +-W of SOME occurrence of the center in one sentence
    for b in range(0, B, 17):
        cw = int(centers[b])
        ok_ctx = set()
        for s in sents:
            for i, w in enumerate(s):
                if w == cw:
                    ok_ctx |= set(s[max(0, i - W):i] + s[i + 1:i + 1 + W])
        for x in ctx[b * C:(b + 1) * C]:
            assert int(x & ~out) in ok_ctx
    # deterministic per (seed, step)
    k2 = np.empty_like(keys)
    c.fill_skipgram(7, 0, B, C, W, nneg, k2.ctypes.data, 2)
    np.testing.assert_array_equal(keys, k2)


def _splitmix64(x: int) -> int:
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


@pytest.mark.parametrize("step,B", [(0, 64), (3, 64), (0, 5000)])
def test_corpus_window_runs(tmp_path, step, B):
    """Windowed skip-gram runs (ss/w2v_window.h): a run is B + 2W consecutive
    positions of the corpus stream starting at step*B - W (wrapping around the
    corpus, laps tagged apart), centers are its middle B, meta carries the
    sentence tag and the reduced window 1 + hash % W (checked against a
    Python re-implementation of the hash)."""
    p = str(tmp_path / "w2v.txt")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_word2vec_data.py"), p,
                           "--lines", "300", "--seed", "2"])
    sents = [list(map(int, ln.split())) for ln in open(p)]
    stream = [w for s in sents for w in s]
    sid = [i for i, s in enumerate(sents) for _ in s]
    c = _host().Corpus(p, 2, 0, 1, 1, 0.0)
    N, S, W, nneg, seed = len(stream), len(sents), 4, 64, 11
    R = B + 2 * W
    keys = np.empty(B + R + nneg, dtype=np.uint64)
    meta = np.empty(R, dtype=np.int32)
    c.fill_skipgram_window(seed, step, B, W, nneg, keys.ctypes.data, meta.ctypes.data)
    out = np.uint64(1 << 40)
    run, neg = keys[B:B + R], keys[B + R:]
    assert (run & out).all() and (neg & out).all() and not (keys[:B] & out).any()
    np.testing.assert_array_equal(keys[:B], run[W:W + B] & ~out)
    m64 = (1 << 64) - 1
    for i in range(R):
        x = (step * B) % N - W + i
        lap, idx = x // N, x % N
        assert int(run[i] & ~out) == stream[idx]
        h = _splitmix64(seed ^ 0x5EEDB0A7 ^ ((x & m64) * 0x9E3779B97F4A7C15 & m64))
        b = 1 + ((h * W) >> 64)
        tag = (sid[idx] + (lap + 1) * S) & 0x7FFFFFF
        assert int(meta[i]) == (tag << 4 | b), i
    k2, m2 = np.empty_like(keys), np.empty_like(meta)
    c.fill_skipgram_window(seed, step, B, W, nneg, k2.ctypes.data, m2.ctypes.data)
    np.testing.assert_array_equal(keys, k2)
    np.testing.assert_array_equal(meta, m2)


def test_window_pair_mask_reference():
    """window_pairs_reference: same sentence, 0 < |d| <= reduced window,
    masked positions never pair."""
    from swiftsnails_amd.models.word2vec import window_pairs_reference

    B, W = 6, 2
    tags = [0, 0, 0, 0, 1, 1, 1, 1, 1, 1]
    bs = [1, 2, 2, 1, 2, 2, 1, 2, 2, 2]
    meta = np.array([(t << 4) | b for t, b in zip(tags, bs)], dtype=np.int32)
    meta[6] = -1
    m = window_pairs_reference(meta, B, W)
    # center 0 = run position 2 (b = 2, sentence 0): positions 0, 1, 3
    assert m[0].nonzero()[0].tolist() == [0, 1, 3]
    # center 2 = run position 4 (b = 2, sentence 1): 5 (6 is masked)
    assert m[2].nonzero()[0].tolist() == [5]
    # center 4 = run position 6 is masked
    assert not m[4].any()


def test_corpus_hashes_words_and_min_count(tmp_path):
    p = str(tmp_path / "t.txt")
    with open(p, "w") as f:
        f.write("the cat sat\nthe dog\nrare the\n")
    c = _host().Corpus(p, 2, 0, 1, 2, 0.0)  # min_count 2 keeps only "the"
    assert c.vocab_size == 1
    assert c.size == 3


@pytest.mark.gpu
@pytest.mark.parametrize("resident", ["hbm", "host"])
def test_sparse_lr_trains_from_libsvm_file(tmp_path, resident):
    from swiftsnails_amd.models.sparse_lr import SparseLRWorker, make_lr_table
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.transport import LoopbackTransport
    from swiftsnails_amd.utils.dataio import FileCtrSource

    rng = np.random.default_rng(0)
    w = rng.standard_normal(5000)
    p = str(tmp_path / "train.svm")
    with open(p, "w") as f:
        for _ in range(20000):
            idx = rng.choice(5000, 8, replace=False)
            z = w[idx].sum() * 0.5
            y = int(rng.random() < 1 / (1 + np.exp(-z)))
            f.write(f"{y} " + " ".join(f"{i}:0.5" for i in idx) + "\n")
    dev = torch.device("cuda", 0)
    src = FileCtrSource(p, "libsvm", batch_size=1024, num_fields=8, resident=resident)
    assert src.resident == resident
    assert src.has_values
    table = make_lr_table(10000, device=dev)
    eng = PSEngine(table, LoopbackTransport(), max_keys=1024 * 8, dim=1, device=dev)
    wk = SparseLRWorker(eng, src)
    losses = []
    for i in range(60):
        wk.step()
        if i % 10 == 9:
            losses.append(wk.mean_loss())
    torch.cuda.synchronize()
    assert losses[-1] < losses[0] - 0.02, losses
    src.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sample", [0.0, 1e-3])
@pytest.mark.parametrize("mode,batch", [("pairs", 256), ("window", 256), ("window", 40000)])
def test_hbm_resident_skipgram_matches_host_sampler(tmp_path, sample, mode, batch):
    """data_resident: hbm for a corpus — the device batchers (k_w2v_corpus_batch,
    k_w2v_corpus_window) write the same keys (and window meta) as the host
    ones, with and without frequent-word sub-sampling, from a host step or a
    device step counter; a 40000-center run wraps the corpus."""
    from swiftsnails_amd.utils.dataio import FileCorpusSource

    p = str(tmp_path / "w2v.txt")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_word2vec_data.py"), p,
                           "--lines", "3000", "--zipf", "1.2", "--vocab", "700"])
    with open(p, "a") as f:
        f.write("42\n7 word\n")  # one-word sentences draw noise contexts; a hashed token
    dev = torch.device("cuda", 0)
    kw = dict(batch_size=batch, window=3, negatives=5, min_count=2, sample=sample, seed=99,
              mode=mode)
    dsrc = FileCorpusSource(p, resident="hbm", device=dev, **kw)
    hsrc = FileCorpusSource(p, resident="host", pin=False, **kw)
    assert dsrc.resident == "hbm" and dsrc.graph_capturable
    keys = torch.empty(dsrc.n_keys, dtype=torch.int64, device=dev)
    hk = torch.empty(hsrc.n_keys, dtype=torch.int64)
    win = mode == "window"
    meta = torch.empty(dsrc.run_len, dtype=torch.int32, device=dev) if win else None
    hm = torch.empty(hsrc.run_len, dtype=torch.int32) if win else None
    step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
    for step in (0, 1, 5):
        hsrc.generate(step, 0, 1, hk, meta=hm)
        dsrc.generate(step, 0, 1, keys, meta=meta)
        torch.cuda.synchronize()
        assert torch.equal(keys.cpu(), hk), step
        if win:
            assert torch.equal(meta.cpu(), hm), step
            if sample:
                assert (hm < 0).any()  # some tokens sub-sampled away
        step_dev.fill_(step + 1)
        dsrc.generate(0, 0, 1, keys, step_dev=step_dev.data_ptr(), step_delta=-1, meta=meta)
        torch.cuda.synchronize()
        assert torch.equal(keys.cpu(), hk), step
        if win:
            assert torch.equal(meta.cpu(), hm), step
    hsrc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("resident,mode", [("hbm", "window"), ("host", "window"),
                                           ("hbm", "pairs"), ("host", "pairs")])
def test_word2vec_trains_from_corpus_file(tmp_path, resident, mode):
    from swiftsnails_amd.models.word2vec import Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.transport import LoopbackTransport
    from swiftsnails_amd.utils.dataio import FileCorpusSource

    p = str(tmp_path / "w2v.txt")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_word2vec_data.py"), p,
                           "--lines", "5000", "--zipf", "1.3", "--vocab", "2000"])
    dev = torch.device("cuda", 0)
    src = FileCorpusSource(p, batch_size=1024, window=2, negatives=5, resident=resident,
                           mode=mode)
    assert src.resident == resident
    opt, init = make_w2v_table_args(32)
    table = HbmTable(capacity=16384, dim=32, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, LoopbackTransport(), max_keys=src.n_keys, dim=32, device=dev)
    wk = Word2VecWorker(eng, src)
    first = None
    for i in range(40):
        wk.step()
        if i == 4:
            first = wk.mean_loss()
    torch.cuda.synchronize()
    assert wk.mean_loss() < first, (first, wk.mean_loss())
    src.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["libsvm", "ctr"])
def test_hbm_resident_batches_match_host_fill(tmp_path, fmt):
    """data_resident: hbm — the batch cut out of the uploaded CSR shard by
    k_csr_batch equals SparseDataset.fill (padding, truncation, wrap-around,
    values), also when the kernel reads its step from device memory (the
    hipGraph replay form)."""
    from swiftsnails_amd.utils.dataio import FileCtrSource

    p = str(tmp_path / ("a.svm" if fmt == "libsvm" else "a.tsv"))
    if fmt == "libsvm":
        _write_libsvm(p, rows=211, seed=11)
    else:
        rng = np.random.default_rng(4)
        with open(p, "w") as f:
            for i in range(173):
                cols = ["" if rng.random() < 0.2 else f"t{int(rng.integers(0, 50))}"
                        for _ in range(int(rng.integers(1, 7)))]
                f.write(f"{i % 2}\t" + "\t".join(cols) + "\n")
    dev = torch.device("cuda", 0)
    B, F = 64, 5
    src = FileCtrSource(p, fmt, batch_size=B, num_fields=F, resident="hbm", device=dev)
    assert src.resident == "hbm" and src.graph_capturable
    ds = _host().SparseDataset(p, fmt, 1, 0, 1)
    keys = torch.empty(B * F, dtype=torch.int64, device=dev)
    labels = torch.empty(B, device=dev)
    xval = torch.empty(B * F, device=dev)
    step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
    for step in (0, 1, 3, 7):
        for mode in ("host_step", "device_step"):
            if mode == "host_step":
                src.generate(step, 0, 1, keys, labels, xval=xval)
            else:
                step_dev.fill_(step - 2)
                src.generate(999, 0, 1, keys, labels, xval=xval, step_dev=step_dev.data_ptr(),
                             step_delta=2)
            torch.cuda.synchronize()
            ek = np.empty(B * F, dtype=np.uint64)
            ev = np.empty(B * F, dtype=np.float32)
            el = np.empty(B, dtype=np.float32)
            ds.fill((step * B) % ds.rows, B, F, ek.ctypes.data, ev.ctypes.data, el.ctypes.data, 1)
            assert keys.cpu().numpy().view(np.uint64).tolist() == ek.tolist(), (step, mode)
            assert labels.cpu().numpy().tolist() == el.tolist()
            np.testing.assert_array_equal(xval.cpu().numpy(), ev)
    src.close()


@pytest.mark.gpu
def test_sparse_lr_file_resident_graph_replay(tmp_path):
    """A file-fed LR job with the shard in HBM replays its step as hipGraphs
    and trains exactly like the eager steps."""
    from swiftsnails_amd.models.sparse_lr import SparseLRWorker, make_lr_table
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.utils.dataio import FileCtrSource

    rng = np.random.default_rng(1)
    w = rng.standard_normal(3000)
    p = str(tmp_path / "train.svm")
    with open(p, "w") as f:
        for _ in range(9000):
            idx = rng.choice(3000, 6, replace=False)
            y = int(rng.random() < 1 / (1 + np.exp(-w[idx].sum() * 0.5)))
            f.write(f"{y} " + " ".join(str(i) for i in idx) + "\n")
    dev = torch.device("cuda", 0)
    losses = {}
    for graph in (False, True):
        src = FileCtrSource(p, "libsvm", batch_size=512, num_fields=6, resident="hbm", device=dev)
        table = make_lr_table(6000, device=dev)
        eng = PSEngine(table, None, max_keys=512 * 6, dim=1, device=dev)
        wk = SparseLRWorker(eng, src)
        out = [float(wk.step().sum().item())]
        if graph:
            assert wk.enable_graph()
            per = wk._gper  # steps per replayed graph (a multiple of the ring depth)
        out += [float(wk.step().sum().item()) for _ in range(2 * 4 * eng.depth)]
        torch.cuda.synchronize()
        table.check()
        losses[graph] = out
    # a replay leaves the loss of the graph's last step in the buffer
    n = len(losses[True]) - 1
    idx = [0] + [k for k in range(1, 1 + n) if (k - 1) % per == per - 1]
    assert len(idx) >= 2
    np.testing.assert_allclose(np.array(losses[True])[idx], np.array(losses[False])[idx],
                               rtol=2e-4, atol=1e-3)
