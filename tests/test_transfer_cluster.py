"""TCP RPC layer and the master/server/worker protocol on CPU.

Mirrors the reference's only distributed test — a self-loopback Transfer
(unitest/core/transfer/transfer_test.h:13-80) — and goes further: a real
1 master + 2 servers + 2 workers cluster in one process (threads), checked
against a single-table oracle.
"""
import struct
import threading
import time

import numpy as np
import pytest

from swiftsnails_amd._native import host


def test_transfer_loopback_request_response():
    h = host()
    t = h.Transfer()
    t.listen("tcp://127.0.0.1:0")
    t.service_start(2)
    t.client_id = 1
    t.register_node(1, t.addr)  # its own address as node 1
    t.add_handler(1, lambda p: struct.pack("<i", struct.unpack("<i", p)[0] + 1))
    got = []
    ev = threading.Event()
    t.send(1, struct.pack("<i", 2008), 1, lambda rsp: (got.append(struct.unpack("<i", rsp)[0]),
                                                        ev.set()))
    assert ev.wait(5)
    assert got == [2009]
    assert struct.unpack("<i", t.call(1, struct.pack("<i", 41), 1))[0] == 42
    assert t.pending_callbacks() == 0
    t.service_end()


def test_transfer_deferred_reply():
    h = host()
    a, b = h.Transfer(), h.Transfer()
    for x in (a, b):
        x.listen("tcp://127.0.0.1:0")
        x.service_start(2)
    a.client_id, b.client_id = 0, 5
    b.register_node(0, a.addr)
    seen = []
    a.add_handler(7, lambda p: (seen.append(p), b"")[1])  # empty response => no reply
    b.send(7, b"x", 0)
    time.sleep(0.3)
    assert seen == [b"x"]
    assert b.pending_callbacks() == 0
    ev = threading.Event()
    b.send(7, b"y", 0, lambda r: ev.set())
    time.sleep(0.3)
    assert not ev.is_set() and b.pending_callbacks() == 1  # still waiting
    a.service_end()
    b.service_end()


def _cluster_cfg(port, backup_root, out_path, S=2, W=2, extra=None):
    from swiftsnails_amd.utils.config import Config

    d = {
        "listen_addr": f"tcp://127.0.0.1:{port}",
        "master_addr": f"tcp://127.0.0.1:{port}",
        "expected_node_num": S + W,
        "master_time_out": 30,
        "init_timeout": 30,
        "frag_num": 50,
        "shard_num": 3,
        "async_exec_num": 4,
        "param_backup_period": 2,
        "param_backup_root": backup_root,
        "param_output": out_path,
        "num_iters": 1,
        "learning_rate": 0.5,
        "optimizer": "sgd",
        "local_train": 0,
    }
    d.update(extra or {})
    return Config.from_dict(d)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cluster_master_servers_workers(tmp_path):
    from swiftsnails_amd.framework.cluster import BaseAlgorithm, SwiftMaster, SwiftServer, SwiftWorker

    port = _free_port()
    D = 2
    out_base = str(tmp_path / "final")
    results = {}

    class Alg(BaseAlgorithm):
        def __init__(self, wid):
            super().__init__()
            self.wid = wid

        def train(self):
            keys = np.array([1, 2, 3, 1000, 77777, 2**40 + 5], dtype=np.uint64)
            v0 = self.pull(keys)
            # zero init, or the other worker's SGD pushes (-0.5 each) if it got
            # there first: the two workers run concurrently
            assert v0.shape == (6, D)
            assert np.isin(v0, [0.0, -0.5, -1.0]).all(), v0
            for _ in range(2):
                self.push(keys, np.ones((6, D), np.float32))
            results[self.wid] = self.pull(keys)
            assert self.pull(np.zeros(0, np.uint64)).shape[0] == 0  # empty pull returns

    cfgs = [_cluster_cfg(port, str(tmp_path), f"{out_base}_{i}.txt") for i in range(5)]
    master = SwiftMaster(cfgs[0])
    servers = [SwiftServer(cfgs[1 + i], dim=D) for i in range(2)]
    workers = [SwiftWorker(cfgs[3 + i], Alg(i), dim=D) for i in range(2)]
    errs = []

    def wrap(f):
        def g():
            try:
                f()
            except Exception as e:  # pragma: no cover - reported below
                errs.append(e)
        return g

    ths = [threading.Thread(target=wrap(master.run))]
    ths += [threading.Thread(target=wrap(s.run)) for s in servers]
    ths += [threading.Thread(target=wrap(w.run)) for w in workers]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert not errs, errs
    assert all(not t.is_alive() for t in ths)
    # 2 workers x 2 pushes x (-lr * 1) on SGD, lr 0.5 => -2.0 after all pushes
    final = {}
    for i, sv in enumerate(servers):  # >1 server: each dumps <path>.s<id>
        for line in open(f"{out_base}_{1 + i}.txt.s{sv.client_id}"):
            k, v = line.rstrip("\n").split("\t")
            final[int(k)] = [float(x) for x in v.split()]
    assert sorted(final) == sorted([1, 2, 3, 1000, 77777, 2**40 + 5])
    for v in final.values():
        np.testing.assert_allclose(v, [-2.0, -2.0])
    # ids: servers 1..S, workers INT_MAX-1, INT_MAX-2 (ServerWorkerRoute.h:20-27)
    assert sorted(s.client_id for s in servers) == [1, 2]
    assert sorted(w.client_id for w in workers) == [2**31 - 3, 2**31 - 2]
    # periodic backup every 2 push requests (server/init.h:126-149)
    assert list(tmp_path.glob("param-*.txt.s*"))


def test_dense_lr_one_worker_one_server_loopback(tmp_path):
    """BASELINE config 1: dense LR, 1 worker + 1 server on CPU over TCP loopback."""
    from swiftsnails_amd.framework.cluster import SwiftMaster, SwiftServer, SwiftWorker
    from swiftsnails_amd.models.dense_lr import DenseLR, DenseLRData

    port = _free_port()
    cfg = lambda: _cluster_cfg(port, str(tmp_path), "", S=1, W=1,  # noqa: E731
                               extra={"optimizer": "adagrad", "learning_rate": 0.2,
                                      "param_backup_period": 0})
    alg = DenseLR(DenseLRData(dim=32), steps=60, batch=256)
    m, s, w = SwiftMaster(cfg()), SwiftServer(cfg(), dim=1), SwiftWorker(cfg(), alg, dim=1)
    ths = [threading.Thread(target=x.run) for x in (m, s, w)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert all(not t.is_alive() for t in ths)
    assert np.mean(alg.losses[-5:]) < alg.losses[0] - 0.1, alg.losses


def test_local_train_mode():
    from swiftsnails_amd.framework.cluster import BaseAlgorithm, SwiftWorker

    out = {}

    class Alg(BaseAlgorithm):
        def train(self):
            k = np.array([5, 6], np.uint64)
            self.push(k, np.array([[1.0], [2.0]], np.float32))
            out["v"] = self.pull(k)

    cfg = {"num_iters": 1, "learning_rate": 1.0, "optimizer": "sgd", "local_train": 1}
    SwiftWorker(cfg, Alg(), dim=1).run()
    np.testing.assert_allclose(out["v"][:, 0], [-1.0, -2.0])
