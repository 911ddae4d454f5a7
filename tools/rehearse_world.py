#!/usr/bin/env python3
"""Rehearse an N-rank job on ONE MI355X: N rank threads, in-process transport.

Each rank has what a rank of the multi-GPU job has — its own table shard
(sized for 1/S of the key space), route-buffer ring, route / main / pull
streams and three communicators — and runs the N>1 engine path (send
segments, count exchange, server-side pull of received segments, per-source
apply, pull-ahead); only RCCL is replaced by device copies between the
ranks' buffers (``swiftsnails_amd/parallel/inproc.py``).  All ranks share
the one GPU, so the step time is NOT the N-GPU step time; what this checks
at full scale is correctness: per-shard sizing, the dedup bucket sizing for
N destinations (overflow is an error), pull-ahead ordering, split roles,
the collective call order (a mismatch deadlocks or raises), training
progress, and that every key lives on the shard the router names.

    python tools/rehearse_world.py --world 8                       # bench config, N = 8
    python tools/rehearse_world.py --world 4 --model word2vec --servers 0-1 --workers 2-3
    python tools/rehearse_world.py --world 8 --model fm --batch 65536

Prints one JSON line (per-rank losses, keys, table load; aggregate timing).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _ranks(spec: str, world: int) -> list[int]:
    if spec in ("", "all"):
        return list(range(world))
    out = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return sorted(out)


def build_rank(a, rank: int, world: int, servers, workers, tr, ct, pt, dev):
    from swiftsnails_amd.models.fm import FMWorker, fm_table_args
    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, make_lr_table
    from swiftsnails_amd.models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine

    S = len(servers)
    serve, work = rank in servers, rank in workers
    if a.model in ("sparse_lr", "fm"):
        data = CtrSynth(batch_size=a.batch, num_fields=a.fields, num_features=a.features,
                        tail_frac=a.tail)
        if a.model == "sparse_lr":
            opt = Optimizer("adagrad", lr=0.05)
            table = make_lr_table(a.features, S, optimizer=opt, load=a.load,
                                  device=dev) if serve else None
            dim = 1
        else:
            dim = 9
            opt, init = fm_table_args(dim - 1)
            table = (HbmTable(dim, int(a.features / S / a.load) + 1024, optimizer=opt, init=init,
                              device=dev) if serve else None)
        eng = PSEngine(table, tr, max_keys=a.batch * a.fields, dim=dim, server_ranks=servers,
                       device=dev, count_transport=ct, pull_transport=pt)
        cls = SparseLRWorker if a.model == "sparse_lr" else FMWorker
        w = cls(eng, data, rank=rank, world=world, active=work)
    else:
        data = W2VSynth(batch_size=a.batch, window=a.window, vocab=a.vocab, mode=a.w2v_mode)
        opt, init = make_w2v_table_args(a.dim, None)
        table = (HbmTable(a.dim, int(2 * a.vocab / S / a.load) + 1024, optimizer=opt, init=init,
                          device=dev) if serve else None)
        eng = PSEngine(table, tr, max_keys=data.n_keys, dim=a.dim, server_ranks=servers,
                       device=dev, count_transport=ct, pull_transport=pt)
        w = Word2VecWorker(eng, data, rank=rank, world=world, active=work)
    return w, table, eng


def rank_main(rank, a, world, servers, workers, groups, dev):
    torch.cuda.set_device(dev)
    tr, ct, pt = (g.transports(dev)[rank] for g in groups)
    try:
        main = torch.cuda.Stream(dev)  # this rank's "default" stream
        with torch.cuda.stream(main):
            w, table, eng = build_rank(a, rank, world, servers, workers, tr, ct, pt, dev)
            losses = []
            for _ in range(a.warmup):
                w.step()
            torch.cuda.synchronize()
            eng.check()
            losses.append(w.mean_loss())
            tr.barrier()
            t0 = time.perf_counter()
            for i in range(a.steps):
                w.step()
                if a.log_every and (i + 1) % a.log_every == 0:
                    losses.append(w.mean_loss())
            torch.cuda.synchronize()
            tr.barrier()
            el = time.perf_counter() - t0
            eng.check()  # dedup bucket overflow / full table: raise
            losses.append(w.mean_loss())
            out = {"rank": rank, "server": table is not None, "worker": rank in workers,
                   "losses": [round(x, 5) for x in losses], "seconds": el,
                   "pull_ahead": bool(eng.pull_ahead), "depth": eng.depth,
                   "engine": {k: int(v) for k, v in eng.metrics.counters.items()}}
            if table is not None:
                st = table.stats()
                out["table_keys"] = int(st["size"])
                out["table_load"] = round(st["load_factor"], 4)
                out["probe_p99"] = st["probe_p99"]
                # every key of the first 4M slots routes to this rank
                k, _ = next(table.export(chunk_slots=1 << 22, to_host=True), (None, None))
                if k is not None:
                    from swiftsnails_amd.utils.hashing import fmix64

                    keys = k.numpy().view(np.uint64)
                    fm = eng.frag_map
                    owner = fm[(fmix64(keys) % np.uint64(len(fm))).astype(np.int64)]
                    out["keys_checked"] = int(len(keys))
                    out["misrouted"] = int((owner != rank).sum())
            return out
    except BaseException:
        for g in groups:
            g.abort()
        raise


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="sparse_lr", choices=["sparse_lr", "fm", "word2vec"])
    ap.add_argument("--servers", default="all")
    ap.add_argument("--workers", default="all")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--tail", type=float, default=0.1)
    ap.add_argument("--load", type=float, default=0.5)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--w2v-mode", default="window", choices=["window", "pairs"])
    ap.add_argument("--log-every", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=1500)
    a = ap.parse_args(argv)

    from swiftsnails_amd.parallel.inproc import InprocGroup, run_ranks

    world = a.world
    servers, workers = _ranks(a.servers, world), _ranks(a.workers, world)
    dev = torch.device("cuda", int(os.environ.get("SS_DEVICE", "0")))
    groups = tuple(InprocGroup(world, timeout=a.timeout) for _ in range(3))
    t0 = time.perf_counter()
    res = run_ranks(world, rank_main, a, world, servers, workers, groups, dev,
                    timeout=a.timeout)
    wall = time.perf_counter() - t0
    el = max(r["seconds"] for r in res)
    samples = a.batch * len(workers) * a.steps
    summary = {
        "rehearsal": f"{world} ranks on one GPU (in-process transport)",
        "model": a.model, "servers": servers, "workers": workers,
        "batch_per_worker": a.batch, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step_all_ranks_one_gpu": round(1000 * el / max(1, a.steps), 3),
        "samples_per_s_one_gpu": round(samples / el, 1),
        "table_keys_total": sum(r.get("table_keys", 0) for r in res),
        "misrouted": sum(r.get("misrouted", 0) for r in res),
        "wall_s": round(wall, 1),
        "ranks": res,
    }
    print(json.dumps(summary), flush=True)
    ok = summary["misrouted"] == 0 and all(
        (not r["worker"]) or (np.isfinite(r["losses"]).all()) for r in res)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
