#!/usr/bin/env python3
"""Headline benchmark: sparse-LR training throughput on the MI355X parameter server.

Metric (BASELINE.json): training samples/sec for the whole node, 1B-feature
sparse logistic regression, at 1/2/4/8 MI355X.

Each rank is a colocated worker + server shard (one process per GPU):
  * its table shard holds 1/N of the 1B-feature space (AdaGrad, 16-byte slots);
  * its worker trains on its own synthetic CTR stream (B samples x 39 fields
    per step, generated on-device inside the timed step);
  * for N > 1 pull/push rounds exchange keys, rows and gradients as peer
    stores into xGMI-mapped HBM mailboxes (device-side counts; a start-up
    litmus picks the publish tier, RCCL all-to-all-v is the fallback).

Weak scaling: the per-GPU batch is fixed, the global batch is N*B.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
        (N > 1 via: python -m torch.distributed.run --nproc-per-node N
         --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "training samples/sec (whole node), 1B-feature sparse LR at 1/2/4/8 MI355X"
BASELINE_SAMPLES_PER_SEC = None  # reference publishes no number


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    # 262144 x 39 = 10.2M key occurrences per GPU per step: a working set sized
    # for one MI355X (the step takes ~1 ms), which also amortises the per-round
    # collective latency when N > 1
    ap.add_argument("--batch", type=int, default=262144, help="samples per GPU per step")
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    # 0.5: measured 0.905 vs 0.927 ms/step (0.7) and 0.914 (0.35) on a shard whose
    # feature space fills up (125M features = one rank of 8): shorter probe runs
    ap.add_argument("--load", type=float, default=0.5, help="table load factor at full feature space")
    ap.add_argument("--tail", type=float, default=0.1)
    ap.add_argument("--optimizer", default="adagrad")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--grad-mode", default="segreduce", choices=["segreduce", "atomic"])
    ap.add_argument("--dedup", default=None, choices=["bucket", "hash"],
                    help="batch dedup implementation (default: bucket)")
    ap.add_argument("--transport", default="auto", choices=["auto", "xgmi", "rccl", "gloo"],
                    help="N>1 data plane: xgmi (peer stores into IPC-mapped HBM mailboxes, "
                         "device-side counts), rccl, or auto = xgmi, falling back to rccl if "
                         "its start-up self-test fails; gloo is a host-staged rehearsal "
                         "transport (tests)")
    # hipGraph replays: neutral at the default batch (GPU-bound), 74 -> 54
    # us/step at batch 1024 where host launch work bounds the step
    ap.add_argument("--graph", default="off", choices=["auto", "on", "off"],
                    help="replay the step as hipGraphs (1 GPU; auto = on for N=1)")
    # uniform (default, BASELINE.json: random-init weights): (u - 0.5) * scale
    # per key, drawn from a key-seeded hash when the key is inserted.  With
    # claimed pulls (one GPU, region tables) a new key's row is written once,
    # by the fused merge's [w | h | key] store, whatever the initialiser, so
    # random init costs nothing over zero init; zero: the usual LR start
    ap.add_argument("--init", default="uniform", choices=["zero", "uniform"],
                    help="weight initialiser of the table")
    ap.add_argument("--init-scale", type=float, default=0.01)
    ap.add_argument("--cal-steps", type=int, default=10,
                    help="N>1: timed steps per window and mode of the pull-ahead calibration "
                         "(0: off); pulled-ahead rounds are kept only if they win by >= 3%% in "
                         "every window")
    ap.add_argument("--cal-windows", type=int, default=2,
                    help="N>1: alternating (synchronous, pulled-ahead) calibration windows")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)

    # SS_BENCH_TRACE_AFTER=S: dump every thread's Python stack to stderr after
    # S seconds (a wedged rank shows where it waits)
    if os.environ.get("SS_BENCH_TRACE_AFTER"):
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["SS_BENCH_TRACE_AFTER"]), exit=False)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print("bench.py: --gpus > 1 must be launched with torch.distributed.run", file=sys.stderr)
            return 2
    if a.dedup:
        os.environ["SS_DEDUP"] = a.dedup
    if a.graph == "on":  # replays run the server half on the main stream (framework/gpu.py)
        os.environ.setdefault("SS_SERVER_STREAM", "0")
    # SS_BENCH_DEVICE pins every rank to one device: a multi-rank rehearsal
    # of this script on a 1-GPU box (with --transport gloo)
    dev_idx = int(os.environ.get("SS_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    # SS_MAIN_PRIO=1: the step's main stream (pull, model kernels, push) at
    # the highest stream priority, above the route stream's dedup
    if os.environ.get("SS_MAIN_PRIO", "0") != "0":
        lo, hi = torch.cuda.Stream.priority_range()
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=min(lo, hi)))

    from swiftsnails_amd.models.sparse_lr import CtrSynth, SparseLRWorker, lr_init, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine

    store = None
    if world > 1:
        from swiftsnails_amd.parallel.transport import default_gloo_ifname

        default_gloo_ifname()
        dist.init_process_group("gloo", rank=rank, world_size=world)
        store = dist.distributed_c10d._get_default_store()

    data = CtrSynth(batch_size=a.batch, num_fields=a.fields, num_features=a.features,
                    tail_frac=a.tail)
    opt = Optimizer(a.optimizer, lr=a.lr)
    table = make_lr_table(a.features, world, optimizer=opt, load=a.load, device=dev,
                          init=lr_init(a.init, a.init_scale))

    # data plane: xGMI mailboxes (fence-free, then fenced publish; each tier
    # must pass the start-up litmus on every rank) -> RCCL (parallel/select.py)
    from swiftsnails_amd.parallel.select import build_engine

    # N>1 exchange (SS_XCHG): unique (each source's unique keys; the worker
    # merges its occurrences), records (every occurrence; the servers dedup
    # and merge), or auto (default): both are built on the same table and
    # timed on the live world after the warm-up, the faster kept — records
    # do less kernel work per rank but ship twice the link bytes, so which
    # wins depends on the links (models/base.py calibrate_exchange)
    xchg = os.environ.get("SS_XCHG", "auto") if a.grad_mode == "segreduce" else "unique"
    if xchg not in ("auto", "unique", "records"):
        print(f"bench.py: SS_XCHG={xchg!r}: auto, unique or records", file=sys.stderr)
        return 2

    def make_engine_for(ex, streams_of=None):
        def make(tr, ct, pt):
            return PSEngine(table, tr, max_keys=a.batch * a.fields, dim=1, device=dev,
                            count_transport=ct, pull_transport=pt, exchange=ex,
                            streams_of=streams_of)
        return make

    free0 = torch.cuda.mem_get_info(dev)[0]
    engine, (transport, ctrans, ptrans), plane = build_engine(
        a.transport, rank, world, dev, store,
        make_engine_for("unique" if xchg == "auto" else xchg),
        log=lambda m: print(f"bench.py: {m}", file=sys.stderr))
    comms = plane.comms
    worker = SparseLRWorker(engine, data, rank=rank, world=world, grad_mode=a.grad_mode)
    # the record-exchange candidate: only over the mailboxes (its own arenas),
    # and only if every rank has room for a second engine of the first one's
    # size (+ 25 %, + 2 GiB) — agreed before any rank builds it, since its
    # set-up is collective (8 ranks sharing one GPU do not fit two engines)
    alt = None
    want = (xchg == "auto" and not engine.fast1 and plane.plane == "xgmi" and worker.bucketed
            and a.cal_steps > 0 and not engine.pull_ahead)  # (timed in synchronous rounds)
    if want:
        torch.cuda.synchronize(dev)
        free1 = torch.cuda.mem_get_info(dev)[0]
        fits = free1 > 1.25 * max(0, free0 - free1) + (2 << 30)
        ok = torch.tensor([1 if fits else 0], dtype=torch.int64)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()):
            want = False
            print("bench.py: no room for the record-exchange candidate on some rank; unique only",
                  file=sys.stderr)
    if want:
        try:
            e2, trs2, plane2 = build_engine("xgmi", rank, world, dev, store,
                                            make_engine_for("records", engine),
                                            prefix="ss_xgmi_rec")
        except (RuntimeError, ValueError) as e:  # agreed collectively: every rank skips it
            print(f"bench.py: record exchange unavailable ({e}); unique only", file=sys.stderr)
        else:
            alt = (e2, trs2, plane2, SparseLRWorker(e2, data, rank=rank, world=world,
                                                    grad_mode=a.grad_mode))

    # a wedged collective ends the job (exit 3) instead of hanging the node
    from swiftsnails_amd.parallel.watchdog import FailureHandler, Watchdog

    failure = FailureHandler()
    for t in {id(x): x for x in (transport, ctrans, ptrans) + (alt[1] if alt else ())
              if x is not None}.values():
        if hasattr(t, "abort"):
            failure.add_hook(t.abort)
    wd = Watchdog(float(os.environ.get("SS_BENCH_ROUND_TIMEOUT", "300")), failure, name="bench")

    def barrier():
        if world > 1:
            dist.barrier()

    # SS_FAULT=delay:<rank>:<ms>: a straggler rank (sleeps every step)
    from swiftsnails_amd.parallel.watchdog import FaultInjector

    fault = FaultInjector(rank=rank)
    for i in range(a.warmup):
        fault.maybe(i)
        worker.step()
        wd.beat(i)
    cal = {}
    if alt is not None:
        torch.cuda.synchronize()
        e2, trs2, plane2, w2 = alt
        for i in range(a.warmup):
            w2.step()
            wd.beat(i)
        pick, cal_x = SparseLRWorker.calibrate_exchange(
            {"unique": worker, "records": w2}, "unique", a.cal_steps, a.cal_windows)
        cal["exchange"] = cal_x
        # the loser's arenas go: every rank's rounds through them are done
        # (synchronised + barrier in the calibration) before any rank frees
        lose_w, lose_trs = (w2, trs2) if pick == "unique" else (worker, (transport, ctrans, ptrans))
        if pick == "records":
            engine, worker, plane = e2, w2, plane2
            transport, ctrans, ptrans = trs2
            comms = plane.comms
        barrier()
        lose_w.close()
        for t in {id(x): x for x in lose_trs if x is not None}.values():
            t.close()
        del lose_w, lose_trs, alt, e2, w2, trs2
        import gc

        gc.collect()
        torch.cuda.empty_cache()
        barrier()
    # N>1 (SS_PULL_AHEAD=auto): time synchronous vs pulled-ahead rounds on
    # the live world and keep the faster (untimed; reported as "calibration")
    if a.cal_steps > 0:
        cal.update(worker.calibrate_pull_ahead(a.cal_steps, a.cal_windows))
    # ... and the server stream (SS_SERVER_STREAM=auto, ranks with a device of
    # their own): kept only if it costs <= 1 % on the live world
    cal_ss = (worker.calibrate_server_stream(a.cal_steps, a.cal_windows)
              if a.cal_steps > 0 else {})
    if cal_ss:
        cal = dict(cal, server_stream=cal_ss)
    # hipGraph replays of the whole step (captured here, outside the timed
    # region; the data generator then reads its step from a device counter)
    graphed = False
    if a.graph == "on" or (a.graph == "auto" and world == 1):
        # a replay runs a whole graph of `per` steps on the first step() of
        # its period, so the timed region must start on a period boundary and
        # span whole periods: per = the longest multiple of the ring depth (up
        # to 4 periods) that divides --steps, else one graph per step
        per = next((m * engine.depth for m in (4, 3, 2, 1) if a.steps % (m * engine.depth) == 0),
                   1)
        os.environ["SS_GRAPH_STEPS"] = str(per)
        graphed = worker.enable_graph()
        if graphed:
            per = worker._gper
            warm = per * max(1, -(-2 * engine.depth // per))  # whole periods, >= 2 ring periods
            for i in range(warm):  # warm every graph
                worker.step()
            assert (worker.step_idx - worker._gbase) % per == 0 and a.steps % per == 0
    torch.cuda.synchronize()
    engine.check()
    first_loss = worker.mean_loss()

    # a roctx range around exactly the timed steps (rocprofv3 --marker-trace):
    # tools/kstats.py --range timed attributes a kernel to the steps iff it
    # starts inside it, so start-up, litmus and calibration kernels never
    # count as per-step work (two host calls; no device work)
    from swiftsnails_amd.utils.tracing import Tracer

    rx = Tracer(enabled=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with rx.range("timed"):
        for i in range(a.steps):
            fault.maybe(a.warmup + i)
            worker.step()
            wd.beat(i)  # one attribute store: no measurable cost
        torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64)
    t_min = t.clone()
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(t_min, op=dist.ReduceOp.MIN)
    elapsed = float(t.item())
    # the fastest rank's own timed region (the reported step is the slowest's)
    fastest_ms = 1000.0 * float(t_min.item()) / a.steps
    engine.check()  # table full / dedup overflow: fail instead of reporting
    last_loss = worker.mean_loss()
    # unique keys per step this rank routed (mean over the ring slots)
    uniq = sum(int(dd.ucount.sum()) for dd in engine.dedupers) // len(engine.dedupers)
    keys_in_table = torch.tensor([table.size()], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(keys_in_table)
    # what the engine moved per step (this rank; host-known counts)
    m = engine.metrics.counters
    nsteps = max(1, engine.rounds)
    a2a = int(m.get("a2a_bytes", 0) / nsteps)
    srv_unique = int(m.get("server_unique", 0) / nsteps)
    recv = int(m.get("unique_recv", 0) / nsteps)
    if engine.fast1:
        tlabel = "none (world 1: colocated worker + server, no exchange)"
    else:
        tlabel = plane.transport
    rccl_n = transport.nranks() if hasattr(transport, "nranks") else None

    samples = a.batch * world * a.steps
    value = samples / elapsed
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_SAMPLES_PER_SEC, 2)
                            if BASELINE_SAMPLES_PER_SEC else None),
            "dtype": "fp32",
            "data": (f"synthetic (on-device CTR generator, {a.fields} fields, Zipf ids over "
                     f"{a.features / 1e9:g}B features; "
                     + ("zero-initialised weights" if a.init == "zero" else
                        f"random-initialised weights, uniform (u-0.5)*{a.init_scale:g}") + ")"),
            "config": {
                "model": f"sparse_lr_{a.features // 1_000_000}M_features",
                "global_batch": a.batch * world,
                "seq_len": a.fields,
                "parallelism": f"ps{world}" + (" (colocated worker + server shard per GPU"
                                                + (f", pull-ahead staleness {engine.lookahead})"
                                                   if getattr(engine, "pull_ahead", False)
                                                   else ")")),
                "pull_ahead": bool(getattr(engine, "pull_ahead", False)),
                "staleness": engine.lookahead if getattr(engine, "pull_ahead", False) else 0,
                **({"calibration": cal} if cal else {}),
                "transport": tlabel,
                "plane": plane.plane if not engine.fast1 else "none",
                "xgmi_tier": plane.xgmi_tier,
                # N>1 rounds: each source's unique keys, or every occurrence
                # (SS_XCHG=records, PSEngine exchange=)
                "exchange": None if engine.fast1 else
                ("records" if getattr(engine, "records", False) else "unique"),
                "fell_back": plane.fell_back,
                **({"fallback_reason": plane.fallback_reason[:300]} if plane.fell_back else {}),
                "devices": plane.devices,
                **({"litmus": plane.litmus} if plane.litmus else {}),
                "init": a.init,
                # the round layout that produced this number (ring depth, server
                # stream, N>1 bucket / sub-bucket layout, claimed server inserts)
                "layout": engine.layout_info(),
                "comms": comms,
                "rccl_nranks": rccl_n,
                "a2a_bytes_per_step": a2a,
                "unique_recv_per_step": recv,
                "server_unique_keys_per_step": srv_unique,
                "optimizer": a.optimizer,
                "hipgraph": graphed,
                "fastest_rank_ms_per_step": round(fastest_ms, 4),
                "keys_per_step_per_gpu": a.batch * a.fields,
                "unique_keys_per_step_per_gpu": uniq,
                "table_keys": int(keys_in_table.item()),
                "loss_first": round(first_loss, 5),
                "loss_last": round(last_loss, 5),
            },
        }
        print(json.dumps(out), flush=True)
    wd.stop()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
