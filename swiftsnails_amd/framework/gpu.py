"""MI355X collective mode: one process per GPU, HBM shards, collective rounds.

This is the GPU-native counterpart of the reference's three roles
(/root/reference/src/core/framework/Swift{Master,Server,Worker}.h):

* master   -> rank 0 + the torch.distributed TCPStore: rendezvous, the
              mailbox IPC handles / RCCL unique-id broadcast, the role table,
              the termination agreement (replaces registration / route /
              hashfrag messages, S3-S5, S8);
* server   -> the ranks in ``server_ranks``: an ``HbmTable`` shard each;
* worker   -> the ranks in ``worker_ranks``: a model worker each.
Colocated (every rank both) is the default: "4 servers + 4 workers on 4
GPUs" (BASELINE config 3) is 4 colocated ranks; split roles are
``server_ranks`` / ``worker_ranks`` (e.g. 0,1,2,3 / 4,5,6,7 on 8 ranks).

Data plane (``transport``): ``auto`` (default) = the xGMI mailboxes
(parallel/xgmi.py, device-side counts), falling back to RCCL if their
start-up self-test fails on any rank; ``xgmi``; ``rccl``; ``gloo`` (host-
staged, tests).  ``PSContext`` owns the per-rank pieces (process group,
transport, table, round engine) and the reference's periodic backup /
final dump behaviour (``param_backup_period``/``param_backup_root`` counted
in rounds, ``param_output`` at the end), plus resume (``resume_from``), which
the reference lacks.  ``run_training`` drives a model from a config.
"""
from __future__ import annotations

import os
import re
import sys
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops.optim import InitConfig, Optimizer
from ..ops.table import HbmTable
from ..parallel.engine import PSEngine
from ..parallel.watchdog import FailureHandler, FaultInjector, Heartbeat, Watchdog
from ..utils import checkpoint as ck
from ..utils.config import Config
from ..utils.logging import get_logger
from ..utils.tracing import Tracer

log = get_logger("swiftsnails.gpu")


def _ranks(spec, world: int) -> list[int]:
    if spec is None or str(spec).strip() in ("", "all"):
        return list(range(world))
    out = sorted({int(x) for x in str(spec).replace(";", ",").split(",") if x.strip()})
    if not out or out[-1] >= world or out[0] < 0:
        raise ValueError(f"bad rank list {spec!r} for world {world}")
    return out


class PSContext:
    def __init__(self, cfg: Config, dim: int, optimizer: Optimizer, init: InitConfig,
                 max_keys: int, capacity: int, exchange: str = "unique"):
        self.cfg = cfg
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # SS_DEVICE pins every rank to one device: multi-rank rehearsals on a
        # 1-GPU box (with transport: gloo — RCCL refuses two ranks per GPU)
        dev_idx = int(os.environ.get("SS_DEVICE", self.local_rank))
        torch.cuda.set_device(dev_idx)
        self.device = torch.device("cuda", dev_idx)
        self.servers = _ranks(cfg.get("server_ranks"), self.world)
        self.workers = _ranks(cfg.get("worker_ranks"), self.world)
        self.is_server = self.rank in self.servers
        self.is_worker = self.rank in self.workers
        store = None
        if self.world > 1:
            from ..parallel.transport import default_gloo_ifname

            default_gloo_ifname()
            if not dist.is_initialized():
                timeout = float(cfg.get("init_timeout", 600))
                import datetime

                dist.init_process_group("gloo", rank=self.rank, world_size=self.world,
                                        timeout=datetime.timedelta(seconds=timeout))
            store = dist.distributed_c10d._get_default_store()
        self.table = (HbmTable(dim, capacity, optimizer=optimizer, init=init, device=self.device,
                               row_dtype=cfg.get("row_dtype", "fp32"))
                      if self.is_server else None)
        ek = dict(max_keys=max_keys, dim=dim, frag_num=int(cfg.get("frag_num", 0) or 0),
                  server_ranks=self.servers, device=self.device, exchange=exchange)
        # data plane (parallel/select.py): auto = xGMI mailboxes (drain, then
        # fenced publish, each litmus-tested on every rank) falling back to
        # RCCL; xgmi; rccl; gloo (host-staged, tests).  World 1: loopback, or
        # SS_ENGINE_GENERAL=xgmi|rccl (the N>1 path through a size-1 plane)
        from ..parallel.select import build_engine

        self.engine, (tr, ct, pt), self.plane = build_engine(
            cfg.get("transport", "auto"), self.rank, self.world, self.device, store,
            lambda tr, ct, pt: PSEngine(self.table, tr, count_transport=ct, pull_transport=pt,
                                        **ek),
            log=log.warning)
        self.transport = tr
        self.backup_period = int(cfg.get("param_backup_period", 0) or 0)
        self._last_backup = -1
        self.backup_root = cfg.get("param_backup_root", ".")
        self.ckpt_format = cfg.get("checkpoint_format", "bin")
        self.tracer = Tracer(enabled=str(cfg.get("trace", "0")) not in ("0", "false"))
        self.engine.tracer = self.tracer  # per-phase ranges: route / pull / compute / push
        # failure detection (parallel/watchdog.py): round watchdog + heartbeats
        self.failure = FailureHandler(exit_process=str(cfg.get("watchdog_exit", "1")) != "0")
        for t in [x for x in (tr, ct, pt) if x is not None]:
            if hasattr(t, "abort"):
                self.failure.add_hook(t.abort)
        rt = float(cfg.get("round_timeout", 600) or 0)
        self.watchdog = Watchdog(rt, self.failure) if rt > 0 else None
        self.heartbeat = None
        if store is not None and float(cfg.get("peer_timeout", 30) or 0) > 0:
            self.heartbeat = Heartbeat(store, self.rank, self.world, self.failure,
                                       interval=float(cfg.get("heartbeat_interval", 2.0)),
                                       peer_timeout=float(cfg.get("peer_timeout", 30)))
        self.fault = FaultInjector(rank=self.rank)
        # resume_from: a checkpoint prefix, or "latest" = the newest complete
        # periodic backup under param_backup_root (restart-after-failure:
        # tools/run_gpu.sh MAX_RESTARTS=k relaunches the job, which picks up
        # where its last backup left off); start_round continues the round
        # count (data stream position, backup numbering)
        self.start_round = 0
        resume = cfg.get("resume_from")
        if resume == "latest":
            found = self._agree(ck.latest_checkpoint(self.backup_root), store)
            if found is not None:
                self.resume(found[0], world=found[2], fmt=found[3])
                self.start_round = found[1]
            else:
                log.info("resume_from latest: no complete backup under %s", self.backup_root)
        elif resume:
            self.resume(resume)
            m = re.match(r".*param-(\d+)$", str(resume))
            self.start_round = int(m.group(1)) if m else 0
        self._last_backup = self.start_round  # the resumed state is already on disk

    def _agree(self, found, store):
        """Rank 0's choice of checkpoint ``(prefix, round, world, fmt)``, for
        every rank (one filesystem view)."""
        if self.world == 1 or store is None:
            return found
        key = "ss_resume_latest"
        enc = "" if found is None else f"{found[1]}:{found[2]}:{found[3]}:{found[0]}"
        if self.rank == 0:
            store.set(key, enc)
        v = store.get(key).decode() if self.rank != 0 else enc
        if not v:
            return None
        rnd, w, fmt, prefix = v.split(":", 3)
        return prefix, int(rnd), int(w), fmt

    # ------------------------------------------------------------ ckpt
    def _owner(self):
        return ck.owner_filter(self.engine.frag_map, self.rank)

    def save(self, prefix: str, fmt: Optional[str] = None) -> Optional[str]:
        torch.cuda.synchronize()
        p = None
        if self.table is not None:
            p = ck.save_sharded(self.table, prefix, self.servers.index(self.rank),
                                len(self.servers), fmt or self.ckpt_format)
        self.barrier()
        return p

    def resume(self, prefix: str, world: Optional[int] = None, fmt: Optional[str] = None) -> int:
        """Load one complete shard set of ``prefix`` (``world``: the set
        written by that many servers; ``fmt``: of that format), re-routed to
        this job's shards."""
        n = 0
        if self.table is not None:
            n = ck.load_sharded(self.table, prefix, owner_fn=self._owner(), world=world, fmt=fmt)
            log.info("rank %d resumed %d keys from %s", self.rank, n, prefix)
        self.barrier()
        return n

    def maybe_backup(self, round_idx: int) -> None:
        """Reference: every param_backup_period pushes -> param-<n>.txt.

        ``round_idx`` is the number of rounds the device has applied
        (``PipelinedWorker.rounds_done``, which runs ahead of the step count
        under hipGraph replays and then repeats): one backup per label."""
        # a backup whenever the applied rounds crossed a period boundary:
        # under hipGraph replays rounds_done() advances a whole graph at a
        # time, so an exact multiple of the period may never be seen
        p = self.backup_period
        if p > 0 and round_idx > 0 and round_idx // p > max(self._last_backup, 0) // p:
            self._last_backup = round_idx
            if self.watchdog:
                self.watchdog.pause()
            # never back up rounds whose keys were silently dropped
            self.engine.check()
            self.save(os.path.join(self.backup_root, f"param-{round_idx}"))
            if self.watchdog:
                self.watchdog.resume()

    def round_done(self, round_idx: int) -> None:
        """Per-round progress mark for the watchdog (+ fault injection point)."""
        if self.watchdog:
            self.watchdog.beat(round_idx)
        self.engine.poll()  # a timed-out / out-of-order mailbox round raises now
        self.fault.maybe(round_idx)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def finish(self):
        if self.watchdog:
            self.watchdog.pause()
        out = self.cfg.get("param_output")
        if out:
            self.save(out, fmt=self.cfg.get("param_output_format", "text"))
        self.engine.check()
        self.barrier()

    def close(self):
        for x in (self.watchdog, self.heartbeat):
            if x is not None:
                x.stop()
        if self.world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def build_worker(cfg: Config):
    """(ctx, worker) for the configured model."""
    from ..models.fm import FMWorker, fm_table_args
    from ..models.sparse_lr import CtrSynth, SparseLRWorker
    from ..models.word2vec import W2VSynth, Word2VecWorker, make_w2v_table_args

    model = cfg.get("model", "sparse_lr")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if str(cfg.get("graph", "0")) not in ("0", "false", ""):
        # hipGraph replays run the server half on the main stream: a server
        # stream that existed during the eager start-up made the replays of
        # word2vec's N>1 step 2x slower (0.28 vs 0.135 ms)
        os.environ.setdefault("SS_SERVER_STREAM", "0")
    nserv = len(_ranks(cfg.get("server_ranks"), world))
    load = float(cfg.get("table_load", 0.7))
    opt = Optimizer(cfg.get("optimizer", "adagrad"), lr=float(cfg.get("learning_rate", 0.05)),
                    l1=float(cfg.get("l1", 0.0)), l2=float(cfg.get("l2", 0.0)))
    rank = int(os.environ.get("RANK", "0"))
    dev = None
    if torch.cuda.is_available():  # the rank's device before data is uploaded to it
        dev = torch.device("cuda", int(os.environ.get("SS_DEVICE",
                                                      os.environ.get("LOCAL_RANK", "0"))))
        torch.cuda.set_device(dev)
    if model in ("sparse_lr", "fm"):
        if cfg.get("data_path", ""):
            from ..utils.dataio import make_ctr_source
            data = make_ctr_source(cfg, rank, world, device=dev)
        else:
            data = CtrSynth(batch_size=int(cfg.get("batch_size", 65536)),
                            num_fields=int(cfg.get("num_fields", 39)),
                            num_features=int(float(cfg.get("num_features", 1e9))),
                            tail_frac=float(cfg.get("tail_frac", 0.1)))
        dim = 1 if model == "sparse_lr" else int(cfg.get("dim", 9))
        init = InitConfig("zero") if model == "sparse_lr" else fm_table_args(dim - 1, opt)[1]
        cap = int(cfg.get("table_capacity", 0) or data.num_features / nserv / load + 1024)
        # sparse LR may ship every occurrence at N>1 (exchange: records /
        # SS_XCHG=records; PSEngine), else each source's unique keys
        # (SS_XCHG=auto, bench.py's start-up measurement of both, runs the
        # unique exchange here)
        xch = str(cfg.get("exchange", os.environ.get("SS_XCHG", "unique")))
        xch = "unique" if xch == "auto" else xch
        ctx = PSContext(cfg, dim, opt, init, data.batch_size * data.num_fields, cap,
                        exchange=xch if model == "sparse_lr" else "unique")
        cls = SparseLRWorker if model == "sparse_lr" else FMWorker
        w = cls(ctx.engine, data, rank=ctx.rank, world=world, active=ctx.is_worker)
    elif model == "word2vec":
        if cfg.get("data_path", ""):
            from ..utils.dataio import make_corpus_source
            data = make_corpus_source(cfg, rank, world, device=dev)
        else:
            data = W2VSynth(batch_size=int(cfg.get("batch_size", 16384)),
                            window=int(cfg.get("window", 5)),
                            vocab=int(float(cfg.get("vocab", 1e6))),
                            negatives=int(cfg.get("negatives", 5)),
                            mode=cfg.get("w2v_mode", "window"),
                            sentence_len=int(cfg.get("sentence_len", 24)),
                            neg_mode=cfg.get("neg_mode", "shared"))
        dim = int(cfg.get("dim", 128))
        opt, init = make_w2v_table_args(dim, opt)
        cap = int(cfg.get("table_capacity", 0) or 2 * data.vocab / nserv / load + 1024)
        ctx = PSContext(cfg, dim, opt, init, data.n_keys, cap)
        w = Word2VecWorker(ctx.engine, data, rank=ctx.rank, world=world, active=ctx.is_worker)
    else:
        raise ValueError(f"unknown model {model!r}")
    return ctx, w


def run_training(cfg: Config, steps: Optional[int] = None, warmup: int = 0,
                 log_every: int = 0) -> dict:
    """Train and return throughput stats.

    File data (a source with ``steps_per_pass``): ``num_iters`` is the number
    of PASSES over each rank's own shard (the reference's num_iters,
    SwiftWorker.h:77), so ranks with unequal shards have unequal step quotas;
    a rank past its quota keeps serving empty rounds, and every
    ``done_check_every`` rounds the ranks agree whether all are done
    (PSEngine.all_done).  Synthetic data: ``num_iters`` (or ``steps``) rounds."""
    ctx, w = build_worker(cfg)
    # resumed job: continue the round count where the checkpoint was taken
    w.step_idx = ctx.start_round
    spp = getattr(getattr(w, "data", None), "steps_per_pass", None)
    passes = None
    if spp is not None and steps is None:
        passes = int(cfg.get("num_iters", 1))
        if w.active:
            w.quota = ctx.start_round + passes * int(spp())
        steps = None
    else:
        steps = int(steps if steps is not None else cfg.get("num_iters", 100))
    every = max(1, int(cfg.get("done_check_every", 8) or 8))
    log_every = log_every or int(cfg.get("log_every", 0) or 0)
    for _ in range(warmup if passes is None else 0):
        w.step()
    # N>1, SS_PULL_AHEAD=auto: keep whichever of synchronous / pulled-ahead
    # rounds runs faster on this world (synthetic data only: the calibration
    # steps consume batches)
    cal = {}
    # a collective (rounds, barriers, an all-reduce): every rank calls it,
    # pure servers too (they step with empty key sets)
    if passes is None and warmup > 0 and int(cfg.get("calibrate_steps", 10) or 0) > 0:
        cal = w.calibrate_pull_ahead(int(cfg.get("calibrate_steps", 10)))
        cal_ss = w.calibrate_server_stream(int(cfg.get("calibrate_steps", 10)))
        if cal_ss:
            cal = dict(cal, server_stream=cal_ss)
    # config `graph: 1`: replay the step as hipGraphs (1 GPU, synthetic data;
    # a no-op where unsupported — see PipelinedWorker.enable_graph)
    graphed = str(cfg.get("graph", "0")) not in ("0", "false", "") and w.enable_graph()
    torch.cuda.synchronize()
    ctx.barrier()
    r0 = w.rounds_done()
    t0 = time.perf_counter()
    i = 0
    while True:
        if passes is None and i >= steps:
            break
        if passes is not None and i % every == 0 and ctx.engine.all_done(w.done):
            break
        with ctx.tracer.range("step"):
            w.step()
        i += 1
        ctx.round_done(w.step_idx)
        ctx.maybe_backup(w.rounds_done())
        if log_every and i % log_every == 0 and ctx.rank == 0:
            log.warning("step %d loss %.5f", i, w.mean_loss())
    steps = i
    torch.cuda.synchronize()
    ctx.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    if ctx.world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    # rounds the device ran in the timed region: with hipGraphs the last
    # replay runs its whole graph, so this can exceed `steps`
    done = max(steps, w.rounds_done() - r0)
    # samples this rank trained in the timed rounds (a rank past its quota
    # served empty rounds)
    mine = done if w.quota is None else max(0, min(done, w.quota - r0))
    n = torch.tensor([w.samples_per_step() * mine], dtype=torch.int64)
    if ctx.world > 1:
        dist.all_reduce(n)
    stats = {"model": cfg.get("model", "sparse_lr"), "world": ctx.world,
             "servers": len(ctx.servers), "workers": len(ctx.workers), "steps": steps,
             "seconds": el, "ms_per_step": 1000 * el / max(1, done),
             "samples_per_s": int(n.item()) / el if el > 0 else 0.0,
             "samples": int(n.item()),
             "rounds_timed": done,
             "loss": w.mean_loss() if ctx.is_worker else None, "hipgraph": bool(graphed),
             "start_round": ctx.start_round, "passes": passes,
             "rank0_quota": w.quota,
             "transport": getattr(ctx.transport, "label", type(ctx.transport).__name__),
             "pull_ahead": bool(getattr(ctx.engine, "pull_ahead", False)),
             "calibration": cal, "layout": ctx.engine.layout_info(),
             "plane": ctx.plane.plane, "xgmi_tier": ctx.plane.xgmi_tier,
             "fell_back": ctx.plane.fell_back, "devices": ctx.plane.devices}
    if cfg.get("model", "sparse_lr") == "word2vec" and ctx.is_worker:
        d = w.data
        stats["w2v"] = {"layout": d.mode, "neg_mode": getattr(d, "neg_mode", "shared"),
                        "mfma": ("none (fp32 dot products)" if w.per_pair else
                                 "bf16" if d.mode == "window" or w.mfma_bf16 else "fp32"),
                        "negatives": d.negatives}
    m = ctx.engine.metrics.counters
    if m:
        stats["rank0_engine"] = {k: int(v) for k, v in m.items()}
    if getattr(w, "window_mode", False) and ctx.is_worker:
        # word2vec sliding-window batches: samples are words (centers); the
        # positive pairs per step depend on sentence edges and reduced windows
        stats["rank0_pairs_last_step"] = w.step_pairs()
        stats["rank0_pairs_per_s_est"] = (stats["rank0_pairs_last_step"] * done / el
                                          if el > 0 else 0.0)
    if ctx.tracer.enabled:
        stats["trace"] = ctx.tracer.summary()
    if ctx.table is not None and str(cfg.get("table_stats", "1")) != "0":
        stats["rank0_table"] = ctx.table.stats()
    ctx.finish()
    ctx.close()
    return stats


if __name__ == "__main__":  # pragma: no cover
    print("use: python -m swiftsnails_amd.launch --config <file>", file=sys.stderr)
    np.zeros(0)
