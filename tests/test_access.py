"""The reference-shaped access API (swiftsnails_amd/access.py) and user-defined
update rules (HbmTable.set_push_method), against numpy references."""
import numpy as np
import pytest
import torch


def _cpu_engine(opt="sgd", lr=0.5):
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    t = HostTable(2, 2, Optimizer(opt, lr=lr), InitConfig("zero"))
    return PSEngine(t, None, max_keys=1000, dim=2, device="cpu"), t


def test_pull_push_with_barrier_cpu_engine():
    from swiftsnails_amd.access import GlobalParamCache, global_pull_access, global_push_access

    eng, _ = _cpu_engine()
    cache = GlobalParamCache(2)
    keys = [9, 3, 3, 11, 9]
    global_pull_access(eng).pull_with_barrier(keys, cache)
    assert cache.keys.tolist() == [3, 9, 11] and not cache.params.any()
    cache.merge_grad([3, 9, 9], [[1, 0], [0, 1], [0, 1]])  # duplicates accumulate
    assert cache.grad(9).tolist() == [0, 2]
    global_push_access(eng).push_with_barrier(keys, cache)  # a key listed twice: pushed once
    assert not cache.grads.any()
    global_pull_access(eng).pull_with_barrier([3, 9, 11, 12], cache)
    np.testing.assert_allclose(cache.param(3).numpy(), [-0.5, 0.0])
    np.testing.assert_allclose(cache.param(9).numpy(), [0.0, -1.0])
    np.testing.assert_allclose(cache.param(12).numpy(), [0.0, 0.0])
    # subset push + per-key views
    cache.merge_grad([12], [[2, 2]])
    cache.merge_grad([11], [[4, 4]])
    global_push_access(eng).push_with_barrier([12], cache)
    assert cache.grad(11).tolist() == [4, 4] and cache.grad(12).tolist() == [0, 0]
    global_pull_access(eng).pull_with_barrier([11, 12], cache)
    np.testing.assert_allclose(cache.params.numpy(), [[0, 0], [-1, -1]])


def test_access_host_client_and_hooks():
    """A host client (pull/push over numpy, e.g. a BaseAlgorithm of the TCP
    cluster) behind the same calls; the GradPramProcMethod hooks."""
    from swiftsnails_amd.access import (GlobalParamCache, global_pull_access, global_push_access,
                                        set_global_target)

    class Client:
        def __init__(self):
            self.w = {}

        def pull(self, keys):
            return np.stack([self.w.get(int(k), np.zeros(3, np.float32)) for k in keys])

        def push(self, keys, grads):
            for k, g in zip(keys, grads):
                self.w[int(k)] = self.w.get(int(k), np.zeros(3, np.float32)) - 0.1 * g

    c = Client()
    set_global_target(c)
    try:
        cache = GlobalParamCache(3)
        ks = np.array([5, 2**63 + 7, 5], dtype=np.uint64)  # u64 keys beyond int64 range
        global_pull_access().pull_with_barrier(ks, cache)
        assert len(cache) == 2
        cache.grads += 1.0
        global_push_access().push_with_barrier(None, cache)
        global_pull_access().pull_with_barrier(ks, cache)
        np.testing.assert_allclose(cache.params.numpy(), -0.1)
        cache.rewrite_param(ks[:1], [[1, 2, 3]])
        np.testing.assert_allclose(cache.param(5).numpy(), [1, 2, 3])
        cache.grads.fill_(1.0)
        cache.update_param(lambda p, g: p - g)
        np.testing.assert_allclose(cache.param(5).numpy(), [0, 1, 2])
        with pytest.raises(KeyError):
            cache.param(6)
        # an empty key set returns at once (the reference blocks forever)
        global_pull_access().pull_with_barrier([], cache)
        assert len(cache) == 0
        global_push_access().push_with_barrier(None, cache)
    finally:
        set_global_target(None)


@pytest.mark.gpu
def test_pull_push_with_barrier_gpu_engine():
    from swiftsnails_amd.access import GlobalParamCache, global_pull_access, global_push_access
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, apply_reference, init_reference
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    opt = Optimizer("adagrad", lr=0.2)
    init = InitConfig("uniform", 0.3, 0.01)
    t = HbmTable(4, 4096, optimizer=opt, init=init, device=dev)
    eng = PSEngine(t, None, max_keys=4096, dim=4, device=dev)
    rng = np.random.default_rng(0)
    keys = rng.integers(0, 10**12, 600)
    cache = GlobalParamCache(4, device=dev)
    global_pull_access(eng).pull_with_barrier(keys, cache)
    uk = np.unique(keys)
    assert cache.keys.cpu().tolist() == uk.tolist()
    ref = init_reference(init, uk, 4, t.width)
    np.testing.assert_array_equal(cache.params.cpu().numpy(), ref[:, :4])
    g = rng.standard_normal((len(uk), 4)).astype(np.float32)
    cache.grads.copy_(torch.from_numpy(g))
    global_push_access(eng).push_with_barrier(None, cache)
    global_pull_access(eng).pull_with_barrier(uk, cache)
    exp = apply_reference(opt, ref, g, 4)[:, :4]
    np.testing.assert_allclose(cache.params.cpu().numpy(), exp, rtol=2e-5, atol=2e-6)


def _sign_momentum(lr, beta):
    """A rule not in the menu: momentum on the gradient sign, state = velocity."""

    def fn(rows, g):
        d = g.shape[1]
        w, v = rows[:, :d], rows[:, d:2 * d]
        v = beta * v + torch.sign(g)
        return torch.cat([w - lr * v, v], 1)

    def ref(rows, g):
        d = g.shape[1]
        w, v = rows[:, :d], rows[:, d:2 * d]
        v = np.float32(beta) * v + np.sign(g)
        return np.concatenate([w - np.float32(lr) * v, v], 1)

    return fn, ref


@pytest.mark.gpu
def test_custom_push_method_table_and_engine():
    """HbmTable.set_push_method: a user-defined update (the reference's
    PushAccessMethod) through table.push, the engine's push_keys and the
    1-GPU round path (pull -> accumulate -> push)."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, init_reference
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    dev = torch.device("cuda", 0)
    fn, ref = _sign_momentum(0.1, 0.5)
    init = InitConfig("uniform", 0.5, 0.0)
    # adagrad's layout: one state column per coordinate (the velocity here)
    t = HbmTable(3, 8192, optimizer=Optimizer("adagrad"), init=init, device=dev)
    t.set_push_method(fn)
    assert not t.snapshot_ok
    rng = np.random.default_rng(1)
    uk = np.unique(rng.integers(0, 10**9, 500))
    kt = torch.from_numpy(uk).to(dev)
    rows = init_reference(init, uk, 3, t.width)
    for _ in range(3):
        g = rng.standard_normal((len(uk), 3)).astype(np.float32)
        t.push(kt, torch.from_numpy(g).to(dev))
        rows = ref(rows, g)
    torch.cuda.synchronize()
    d = t.to_dict(with_state=True)
    np.testing.assert_allclose(np.stack([d[int(k)] for k in uk]), rows, rtol=1e-5, atol=1e-6)

    # the engine's round path at world 1: duplicates merged before the rule
    eng = PSEngine(t, None, max_keys=4096, dim=3, device=dev)
    occ = np.concatenate([uk[:200], uk[:200], uk[200:300]])
    r = eng.pull(torch.from_numpy(occ).to(dev))
    gocc = rng.standard_normal((len(occ), 3)).astype(np.float32)
    eng.accumulate(r, torch.from_numpy(gocc).to(dev))
    eng.push(r)
    torch.cuda.synchronize()
    merged = {}
    for k, gg in zip(occ.tolist(), gocc):
        merged[k] = merged.get(k, 0) + gg
    sel = np.array(sorted(merged))
    idx = np.searchsorted(uk, sel)
    rows[idx] = ref(rows[idx], np.stack([merged[k] for k in sel]).astype(np.float32))
    d = t.to_dict(with_state=True)
    np.testing.assert_allclose(np.stack([d[int(k)] for k in uk]), rows, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_custom_push_method_n2_server_apply():
    """World 2 (in-process ranks on one GPU): the server-side per-source apply
    runs the custom rule; an SGD written as a custom rule gives the same
    shards as the built-in SGD."""
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.inproc import InprocGroup, run_ranks

    dev = torch.device("cuda", 0)

    def run(custom):
        groups = (InprocGroup(2, timeout=60), InprocGroup(2, timeout=60))

        def rank(r):
            torch.cuda.set_device(dev)
            tr, ct = (g.transports(dev)[r] for g in groups)
            try:
                with torch.cuda.stream(torch.cuda.Stream(dev)):
                    t = HbmTable(2, 4096, optimizer=Optimizer("sgd", lr=0.25),
                                 init=InitConfig("uniform", 0.2), device=dev)
                    if custom:
                        t.set_push_method(lambda rows, g: rows - 0.25 * g)
                    eng = PSEngine(t, tr, max_keys=512, dim=2, device=dev, count_transport=ct)
                    rng = np.random.default_rng(10 + r)
                    for _ in range(3):
                        k = rng.integers(0, 300, 400)
                        rd = eng.pull(torch.from_numpy(k).to(dev))
                        g = torch.from_numpy(rng.standard_normal((400, 2)).astype(np.float32))
                        eng.accumulate(rd, g.to(dev))
                        eng.push(rd)
                    torch.cuda.synchronize()
                    return t.to_dict(with_state=True)
            except BaseException:
                for g in groups:
                    g.abort()
                raise

        out = {}
        for d in run_ranks(2, rank, timeout=120):
            out.update(d)
        return out

    a, b = run(True), run(False)
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_allclose(a[k], b[k], rtol=1e-5, atol=1e-6)


def test_host_table_push_method_and_cluster_server():
    """User-defined update rule on the CPU table (batched per push, torch
    tensors) and on a host-mode server of a real TCP cluster (the
    reference's PushAccessMethod on its own deployment shape)."""
    import threading

    from swiftsnails_amd.framework.cluster import BaseAlgorithm, SwiftMaster, SwiftServer, SwiftWorker
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.utils.config import Config
    from test_transfer_cluster import _free_port

    def rule(rows, g):  # sign-SGD with a push counter in the state column
        out = rows.clone()
        out[:, :2] -= 0.5 * torch.sign(g)
        out[:, 2:] += 1.0
        return out

    t = HostTable(2, 3, Optimizer("adagrad"), InitConfig("zero"))
    t.set_push_method(rule)
    k = np.array([4, 8, 15])
    t.push_keys(k, np.array([[1, -1], [0, 2], [-3, 0]], np.float32))
    d = t.to_dict(with_state=True)
    np.testing.assert_allclose(d[4], [-0.5, 0.5, 1, 1])
    np.testing.assert_allclose(d[8], [0, -0.5, 1, 1])
    np.testing.assert_allclose(d[15], [0.5, 0, 1, 1])

    port = _free_port()
    cfg = Config.from_dict({
        "listen_addr": f"tcp://127.0.0.1:{port}", "master_addr": f"tcp://127.0.0.1:{port}",
        "expected_node_num": 2, "master_time_out": 30, "init_timeout": 30, "frag_num": 16,
        "shard_num": 2, "async_exec_num": 2, "param_backup_period": 0,
        "param_output": "", "num_iters": 1, "learning_rate": 0.5, "optimizer": "adagrad",
        "local_train": 0})
    got = {}

    class Alg(BaseAlgorithm):
        def train(self):
            keys = np.array([1, 2, 3], dtype=np.uint64)
            self.pull(keys)
            self.push(keys, np.array([[1, 1], [-1, 0], [0, 2]], np.float32))
            self.push(keys, np.array([[1, 1], [-1, 0], [0, 2]], np.float32))
            got["w"] = self.pull(keys)

    master = SwiftMaster(cfg)
    server = SwiftServer(cfg, dim=2, push_method=rule)
    worker = SwiftWorker(cfg, Alg(), dim=2)
    errs = []

    def wrap(f):
        def g():
            try:
                f()
            except Exception as e:  # pragma: no cover - reported below
                errs.append(e)
        return g

    ths = [threading.Thread(target=wrap(x.run)) for x in (master, server, worker)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(60)
    assert not errs, errs
    np.testing.assert_allclose(got["w"], [[-1, -1], [1, 0], [0, -1]])
    assert server.push_count == 2


def test_host_table_tensor_rule_sees_duplicate_keys_once():
    """A tensor-code update rule on the host table gets each key once per
    push, with the gradients of its duplicates summed (no update dropped by
    the last write-back winning)."""
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    t = HostTable(1, 2, Optimizer("sgd", lr=1.0), InitConfig("zero"))
    seen = []

    def rule(rows, g):
        seen.append(rows.shape[0])
        rows[:, 0] -= g[:, 0]
        return rows

    t.set_push_method(rule)
    keys = np.array([5, 7, 5, 5, 9, 7], dtype=np.int64)
    t.push_keys(keys, np.array([[1], [2], [3], [4], [5], [6]], dtype=np.float32))
    assert seen == [3]
    np.testing.assert_allclose(t.pull_keys(np.array([5, 7, 9])).numpy()[:, 0], [-8, -8, -5])
