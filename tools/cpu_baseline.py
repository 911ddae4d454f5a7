#!/usr/bin/env python3
"""Reference-semantics CPU baseline (BASELINE.md "What we will measure instead", config 1).

The reference publishes no numbers and cannot be built here (ZeroMQ,
sparsehash and glog are absent, its unit tests do not compile — SURVEY §4), so
the baseline is the SAME architecture re-implemented in this repo's host C++
runtime: 1 master + S servers + W workers as separate roles talking over TCP
loopback (csrc/host/transfer.h), CPU hash-table shards with lock striping
(csrc/host/host_table.h), workers that pull the batch's keys, compute the LR
gradient on the CPU and push it back — i.e. SwiftSnails' pull/compute/push
loop, with binary SoA payloads instead of per-key BinaryBuffer streams (which
only makes this baseline faster than the original).

Workload: the same synthetic CTR stream as bench.py (39 fields, 1B-feature
key space, Zipf ids + uniform tail, AdaGrad).  Prints one JSON line.

    python tools/cpu_baseline.py [--servers 1] [--workers 1] [--batch 4096] [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--servers", type=int, default=1)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--shard-num", type=int, default=8)
    a = ap.parse_args(argv)

    from swiftsnails_amd.framework.cluster import BaseAlgorithm, SwiftMaster, SwiftServer, SwiftWorker
    from swiftsnails_amd.models.ctr_data import gen_ctr_np, lr_grad_np
    from swiftsnails_amd.utils.config import Config

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    base = {
        "listen_addr": f"tcp://127.0.0.1:{port}", "master_addr": f"tcp://127.0.0.1:{port}",
        "expected_node_num": a.servers + a.workers, "master_time_out": 60, "init_timeout": 60,
        "frag_num": 1000, "shard_num": a.shard_num, "async_exec_num": 4,
        "param_backup_period": 0, "param_output": "", "num_iters": 1, "learning_rate": 0.05,
        "optimizer": "adagrad", "local_train": 0,
    }
    V = a.features // a.fields
    times = {}

    class LR(BaseAlgorithm):
        def __init__(self, wid):
            super().__init__()
            self.wid = wid

        def train(self):
            losses = []
            for step in range(a.warmup + a.steps):
                if step == a.warmup:
                    t0 = time.perf_counter()
                keys, labels = gen_ctr_np(20150404, (step * a.workers + self.wid) * a.batch,
                                          a.batch, a.fields, V)
                u, inv = np.unique(keys.view(np.uint64), return_inverse=True)
                w = self.pull(u)[:, 0]
                g_occ, loss = lr_grad_np(w[inv], labels, a.fields)
                gu = np.bincount(inv, weights=g_occ, minlength=len(u)).astype(np.float32)
                self.push(u, gu[:, None])
                losses.append(loss / a.batch)
            times[self.wid] = (time.perf_counter() - t0, losses[0], losses[-1])

    master = SwiftMaster(Config.from_dict(base))
    servers = [SwiftServer(Config.from_dict(base), dim=1) for _ in range(a.servers)]
    workers = [SwiftWorker(Config.from_dict(base), LR(i), dim=1) for i in range(a.workers)]
    ths = [threading.Thread(target=master.run)] + [threading.Thread(target=x.run)
                                                   for x in servers + workers]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = max(v[0] for v in times.values())
    value = a.batch * a.workers * a.steps / el
    print(json.dumps({
        "metric": "reference-semantics CPU baseline: sparse LR samples/s over TCP loopback",
        "value": round(value, 1), "unit": "samples/s", "servers": a.servers,
        "workers": a.workers, "batch": a.batch, "steps": a.steps,
        "ms_per_step": round(1000 * el / a.steps, 2), "cpu_threads": os.cpu_count(),
        "loss_first": round(times[0][1], 4), "loss_last": round(times[0][2], 4)}))


if __name__ == "__main__":
    main()
