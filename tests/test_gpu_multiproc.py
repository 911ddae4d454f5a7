"""Multi-rank engine on ONE MI355X: two processes share cuda:0.

* gloo transport + HBM tables: exercises the device server path (segmented
  probe/gather, per-source apply, dedup routing into per-rank segments) with
  world > 1 against the same single-table oracle as the CPU tests.
* RCCL transport, 2 ranks on the same GPU: exercises the native
  communicator's alltoallv (skipped if RCCL refuses duplicate devices).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import collect, file_init, init_gloo
from test_engine_cpu import DIM, ROUNDS, _grads_for, _keys_for, _oracle

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, world, init, servers, workers, opt_kind, transport, q, env=None):
    os.environ.update(env or {})
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.ops.table import HbmTable
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import RcclTransport, TorchDistTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if transport == "rccl":
            try:
                tr = RcclTransport(rank, world, dev,
                                   store=dist.distributed_c10d._get_default_store())
            except RuntimeError as e:
                q.put((rank, "skip", str(e)))
                return
        elif transport == "xgmi":
            from swiftsnails_amd.parallel.xgmi import XgmiTransport

            tr = XgmiTransport(rank, world, dev, dist.distributed_c10d._get_default_store(),
                               aux=TorchDistTransport(), timeout_s=60)
        else:
            tr = TorchDistTransport()
        table = (HbmTable(DIM, 4096, Optimizer(opt_kind, lr=0.1), InitConfig("uniform", 0.2, 0.01),
                          device=dev) if rank in servers else None)
        eng = PSEngine(table, tr, max_keys=300, dim=DIM, frag_num=64, server_ranks=servers,
                       device=dev)
        pulled = {}
        for rnd in range(ROUNDS):
            k = _keys_for(rank, rnd) if rank in workers else np.zeros(0, np.int64)
            r = eng.pull(torch.from_numpy(k).to(dev))
            pulled[(rank, rnd)] = eng.gather(r, len(k)).cpu().numpy().copy()
            if len(k):
                eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)).to(dev))
            eng.push(r)
        torch.cuda.synchronize()
        eng.check()
        eng.poll()
        if hasattr(tr, "check"):
            tr.check()
        state = table.to_dict(with_state=True) if table is not None else {}
        if hasattr(tr, "describe"):
            pulled["_plane"] = tr.describe()
        q.put((rank, pulled, state))
    finally:
        dist.destroy_process_group()


def _run(world, servers, workers, opt, transport, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_rank,
                         args=(r, world, init, servers, workers, opt, transport, q, env))
             for r in range(world)]
    for p in procs:
        p.start()
    res = collect(q, procs, world, 180)
    for p in procs:
        p.join(60)
    if any(r[1] == "skip" for r in res):
        for p in procs:
            if p.is_alive():
                p.kill()
        pytest.skip("RCCL refused 2 ranks on one GPU: " + str([r[2] for r in res if r[1] == "skip"]))
    for p in procs:
        assert p.exitcode == 0
    merged, pulled, planes = {}, {}, []
    for rank, pl, st in res:
        assert not (set(st) & set(merged))
        merged.update(st)
        planes.append(pl.pop("_plane", None))
        pulled.update(pl)
    ref_state, ref_pulled = _oracle(world, workers, opt)
    assert set(merged) == set(ref_state)
    for k in ref_state:
        np.testing.assert_allclose(merged[k], ref_state[k], rtol=3e-5, atol=3e-6)
    for key, v in ref_pulled.items():
        np.testing.assert_allclose(pulled[key], v, rtol=3e-5, atol=3e-6)
    return planes


@pytest.mark.parametrize("world,servers,workers,opt", [
    (2, [0, 1], [0, 1], "adagrad"),
    (2, [1], [0], "sgd"),
])
def test_engine_gpu_gloo(world, servers, workers, opt):
    _run(world, servers, workers, opt, "gloo")


def test_engine_gpu_rccl_same_device():
    _run(2, [0, 1], [0, 1], "adagrad", "rccl")


@pytest.mark.parametrize("world,servers,workers,opt", [
    (2, [0, 1], [0, 1], "adagrad"),
    (3, [0, 1, 2], [0, 1, 2], "sgd"),
    (2, [1], [0], "adagrad"),
    (4, [0, 1], [2, 3], "ftrl"),
    (8, list(range(8)), list(range(8)), "adagrad"),  # 4 server sub-buckets per bucket
])
def test_engine_gpu_xgmi_peers(world, servers, workers, opt):
    """The xGMI mailbox data plane with real peers: N processes on cuda:0
    map each other's arenas through IPC handles; puts, arrival counters,
    waits and the servers' merge of all sources run for real and reproduce
    the single-table oracle (pulled rows and final state)."""
    _run(world, servers, workers, opt, "xgmi")


def _run_lr_rank(rank, world, init, pull_ahead, grad_mode, q):
    os.environ["SS_PULL_AHEAD"] = "1" if pull_ahead else "0"
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        data = CtrSynth(batch_size=2048, num_fields=13, num_features=200_000, tail_frac=0.0)
        table = make_lr_table(data.num_features, world, device=dev)
        eng = PSEngine(table, TorchDistTransport(), max_keys=2048 * 13, dim=1, device=dev)
        assert eng.pull_ahead == pull_ahead
        w = SparseLRWorker(eng, data, rank=rank, world=world, grad_mode=grad_mode)
        losses = []
        for _ in range(40):
            w.step()
            losses.append(w.mean_loss())
        torch.cuda.synchronize()
        table.check()
        q.put((rank, losses, table.size()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grad_mode", ["segreduce", "atomic"])
def test_lr_worker_world2_pull_ahead(grad_mode):
    """Worker pipeline with N>1: pull-ahead (staleness 1, round i+1 pulled on
    the route stream while round i computes) trains like the synchronous
    pipeline."""
    ctx = mp.get_context("spawn")
    out = {}
    for pa in (False, True):
        q = ctx.Queue()
        init = file_init()
        procs = [ctx.Process(target=_run_lr_rank, args=(r, 2, init, pa, grad_mode, q))
                 for r in range(2)]
        for p in procs:
            p.start()
        res = collect(q, procs, 2, 240)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        out[pa] = {r: (l, n) for r, l, n in res}
    for pa, per_rank in out.items():
        for r, (losses, n) in per_rank.items():
            assert np.isfinite(losses).all()
            assert np.mean(losses[-5:]) < np.mean(losses[:3]) - 0.01, (pa, r, losses)
            assert n > 0
    sync_last = np.mean([np.mean(l[-5:]) for l, _ in out[False].values()])
    ahead_last = np.mean([np.mean(l[-5:]) for l, _ in out[True].values()])
    assert abs(ahead_last - sync_last) < 0.03, (sync_last, ahead_last)


def _bench_torchrun(nproc, extra, env_extra=None):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GLOO_SOCKET_IFNAME="lo", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(nproc)] + extra
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("transport", ["auto", "rccl"])
@pytest.mark.parametrize("world", [2, 4])  # N = 8 is the driver's scaling run
def test_bench_script_multi_gpu(world, transport):
    """The driver's scaling run in miniature: bench.py over `world` GPUs with
    the default xGMI mailboxes or the native RCCL communicator (skipped on
    boxes with fewer GPUs)."""
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs")
    j = _bench_torchrun(world, ["--steps", "5", "--warmup", "2", "--batch", "16384",
                                "--features", "10000000", "--transport", transport])
    assert j["n_gpus"] == world and j["value"] > 0
    assert j["config"]["parallelism"].startswith(f"ps{world}")
    assert j["config"]["devices"] == world
    if transport == "rccl":
        assert j["config"]["rccl_nranks"] == world and j["config"]["plane"] == "rccl"
    else:  # auto: the mailboxes ran (no silent fallback to RCCL)
        assert j["config"]["plane"] == "xgmi" and not j["config"]["fell_back"], j["config"]


def test_bench_script_world2_gloo_rehearsal():
    """bench.py itself at N = 2 under torch.distributed.run (the driver's
    launch), both ranks pinned to cuda:0 with the host-staged gloo data plane
    (RCCL refuses two ranks per device): the whole N>1 script path — table
    sizing per shard, pull-ahead worker, barriers, max-over-ranks timing and
    the one JSON line from rank 0."""
    j = _bench_torchrun(2, ["--steps", "4", "--warmup", "2", "--batch", "4096",
                            "--features", "2000000", "--transport", "gloo"],
                        {"SS_BENCH_DEVICE": "0"})
    assert j["n_gpus"] == 2 and j["steps"] == 4 and j["warmup"] == 2
    assert j["value"] > 0 and j["ms_per_step"] > 0
    assert j["config"]["global_batch"] == 2 * 4096
    assert j["config"]["parallelism"].startswith("ps2")


def _run_w2v_rank(rank, world, init, q):
    os.environ["SS_PULL_AHEAD"] = "0"
    init_gloo(init, rank, world)
    try:
        from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
        from swiftsnails_amd.ops.table import HbmTable
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        data = W2VSynth(batch_size=1000, window=4, vocab=4000, noise=0.05, mode="window")
        opt, init_cfg = make_w2v_table_args(64, None)
        table = HbmTable(64, 20000, optimizer=opt, init=init_cfg, device=dev)
        eng = PSEngine(table, TorchDistTransport(), max_keys=data.n_keys, dim=64, device=dev)
        assert not eng.fast1
        w = Word2VecWorker(eng, data, rank=rank, world=world)
        assert w.occ_reduce
        losses = []
        for _ in range(12):
            w.step()
            losses.append(w.mean_loss())
        torch.cuda.synchronize()
        table.check()
        q.put((rank, losses, table.to_dict(with_state=True)))
    finally:
        dist.destroy_process_group()


def test_word2vec_window_world2_trains():
    """N>1 engine path (two ranks on cuda:0, gloo data plane): the window
    tile's per-key merge of occurrence rows (k_w2v_osort / k_w2v_oreduce over
    the compact send layout), the servers' merge of both ranks' rows: every
    rank's loss falls and both shards fill."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_w2v_rank, args=(r, 2, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = collect(q, procs, 2, 240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    keys = set()
    for r, losses, table in res:
        assert np.isfinite(losses).all() and np.mean(losses[-3:]) < np.mean(losses[:2]), losses
        assert len(table) > 0 and not (keys & set(table))
        keys |= set(table)


def test_bench_script_world2_xgmi_one_gpu():
    """bench.py at N = 2 under torch.distributed.run with the DEFAULT data
    plane (xGMI mailboxes, device-side counts), both ranks on cuda:0: the
    driver's N>1 scaling path with a real peer — arena IPC mapping, the
    start-up self-test, puts into the peer's mailboxes, waits on its arrival
    counters, the servers' merge — and the one JSON line reporting what ran."""
    j = _bench_torchrun(2, ["--steps", "6", "--warmup", "3", "--batch", "8192",
                            "--features", "4000000"], {"SS_BENCH_DEVICE": "0"})
    assert j["n_gpus"] == 2 and j["value"] > 0
    c = j["config"]
    assert c["transport"].startswith("xGMI"), c["transport"]
    assert c["plane"] == "xgmi" and c["xgmi_tier"] == "drain" and not c["fell_back"]
    assert c["devices"] == 1
    assert c["server_unique_keys_per_step"] > 0
    assert c["server_unique_keys_per_step"] <= c["unique_recv_per_step"]
    assert c["a2a_bytes_per_step"] > 0
    assert c["loss_last"] < c["loss_first"]


def test_uneven_file_shards_terminate_together(tmp_path):
    """Two ranks on cuda:0 (xGMI mailboxes) training sparse LR on their OWN
    files of different lengths (data_path with {rank}): num_iters = 2 passes
    over each rank's file gives quotas of 2 x ceil(rows / B) steps; the rank
    that finishes first serves empty rounds until both are done; the job
    stops at the first agreed check round and dumps the final model."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rng = np.random.default_rng(3)
    rows = {0: 700, 1: 230}
    for r, n in rows.items():
        with open(tmp_path / f"d.{r}.txt", "w") as f:
            for _ in range(n):
                feats = sorted(set(rng.integers(1, 5000, size=6).tolist()))
                f.write(f"{int(rng.random() < 0.3)} " + " ".join(f"{x}:1" for x in feats) + "\n")
    out = tmp_path / "final"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "swiftsnails_amd.launch", "--config",
           os.path.join(root, "configs", "sparse_lr_10m.conf"),
           "--set", f"data_path={tmp_path}/d.{{rank}}.txt", "--set", "data_format=libsvm",
           "--set", "batch_size=64", "--set", "num_fields=8", "--set", "num_iters=2",
           "--set", "done_check_every=4", "--set", "table_capacity=100000",
           "--set", f"param_output={out}", "--set", "param_output_format=text",
           "--set", "transport=xgmi"]
    env = dict(os.environ, GLOO_SOCKET_IFNAME="lo", SS_DEVICE="0", PYTHONPATH=root)
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    quotas = {k: 2 * -(-n // 64) for k, n in rows.items()}  # 22 and 8 steps
    assert stats["passes"] == 2 and stats["rank0_quota"] == quotas[0]
    # the first multiple of done_check_every at which every rank is done
    assert stats["steps"] == -(-max(quotas.values()) // 4) * 4
    assert stats["samples"] == 64 * sum(quotas.values())
    dumped = {}
    for f in tmp_path.glob("final.shard*-of-2.txt"):
        for ln in f.read_text().splitlines():
            k, v = ln.split("\t")
            dumped[int(k)] = v
    feats = set()
    for n in rows:
        for ln in (tmp_path / f"d.{n}.txt").read_text().splitlines():
            feats |= {int(t.split(":")[0]) for t in ln.split()[1:]}
    assert set(dumped) == feats  # both ranks' keys, each on exactly one shard


def _run_access_rank_gpu(rank, world, init, q):
    init_gloo(init, rank, world)
    try:
        from test_engine_cpu import _init_rows, _pull_vals

        from swiftsnails_amd.ops.optim import InitConfig, Optimizer
        from swiftsnails_amd.ops.table import HbmTable
        from swiftsnails_amd.parallel.engine import PSEngine
        from swiftsnails_amd.parallel.transport import TorchDistTransport
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        tr = XgmiTransport(rank, world, dev, dist.distributed_c10d._get_default_store(),
                           aux=TorchDistTransport(), timeout_s=60)
        table = HbmTable(DIM, 4096, Optimizer("adagrad", lr=0.1), InitConfig("zero"), device=dev)
        table.set_init_method(lambda k: _init_rows(k.cpu()).to(dev))
        table.set_pull_method(_pull_vals)
        eng = PSEngine(table, tr, max_keys=300, dim=DIM, frag_num=64, device=dev)
        out = []
        for rnd in range(3):
            from test_engine_cpu import _grads_for, _keys_for

            k = _keys_for(rank, rnd)
            r = eng.pull(torch.from_numpy(k).to(dev))
            out.append((k, eng.gather(r, len(k)).cpu().numpy().copy()))
            eng.accumulate(r, torch.from_numpy(_grads_for(k, rank, rnd)).to(dev))
            eng.push(r)
        torch.cuda.synchronize()
        eng.check()
        q.put((rank, out, table.to_dict(with_state=True)))
    finally:
        dist.destroy_process_group()


def test_user_init_and_pull_methods_world2_gpu():
    """User init / pull methods (tensor code) on HBM shards of a 2-process
    job over the xGMI mailboxes: the same oracle as the CPU test."""
    from test_engine_cpu import check_access_results

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = file_init()
    procs = [ctx.Process(target=_run_access_rank_gpu, args=(r, 2, init, q)) for r in range(2)]
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


def test_split_roles_calibration_world3():
    """Split roles (rank 0 serves only, ranks 1-2 only train) through the
    launcher with warmup > 0 under SS_PULL_AHEAD=auto: the pull-ahead
    calibration is a collective (rounds, barriers, an all-reduce), so the
    server-only rank must take part in it — it used to skip it and the
    workers' calibration rounds waited for it forever.  All
    three ranks on cuda:0 over the xGMI mailboxes."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "swiftsnails_amd.launch", "--config",
           os.path.join(root, "configs", "sparse_lr_10m.conf"),
           "--steps", "6", "--warmup", "3",
           "--set", "batch_size=2048", "--set", "num_fields=13", "--set", "num_features=2000000",
           "--set", "server_ranks=0", "--set", "worker_ranks=1,2", "--set", "calibrate_steps=3",
           "--set", "transport=xgmi", "--set", "round_timeout=120"]
    env = dict(os.environ, GLOO_SOCKET_IFNAME="lo", SS_DEVICE="0", PYTHONPATH=root,
               SS_PULL_AHEAD="auto", SS_XGMI_TIMEOUT="60")
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    cal = stats.get("calibration") or {}
    assert cal, stats  # the calibration ran (on every rank: it returned)
    assert len(cal["sync_ms"]) == cal["windows"] == 2
    assert stats["steps"] == 6
