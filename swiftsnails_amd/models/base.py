"""Common driver for PS-backed model workers on MI355X.

A worker step = route (route stream, one step of lookahead) -> pull -> fused
model kernel (main stream) -> push.  Subclasses provide ``_produce`` (write
the batch's keys for a step into ring slot `slot`, on `stream`) and
``_compute`` (launch the fused forward/backward over the pulled round).

``active=False`` is a rank that only serves (split server/worker roles): it
still enters every collective round, with an empty key set — the
reference's servers never train, and in a lockstep collective round a
non-worker contributes zero keys.
"""
from __future__ import annotations

import collections
import gc
import logging
import os
import time
from typing import Optional

import torch

log = logging.getLogger(__name__)


class _GraphSet(list):
    """A worker's captured hipGraphs, owned so that they are destroyed BEFORE
    what their nodes reference.  A captured step records and waits the round
    engine's HIP events and launches kernels on its mailbox arenas; a graph
    exec that outlived them (a worker collected by the cyclic GC, which
    clears the objects of a cycle in no set order) left the HIP runtime with
    dangling event nodes, and a later replay in the same process crashed
    inside hipGraphLaunch.  The set keeps the engine alive and resets every
    graph after the device drains — from ``close()``, or from its finaliser,
    which the GC runs before it clears any object of the cycle (PEP 442) and
    refcounting runs before the set's own references are dropped."""

    def __init__(self, graphs, keep):
        super().__init__(graphs)
        self.keep = keep  # the engine: its RoundEngine events and arenas

    def close(self) -> None:
        if len(self):
            torch.cuda.synchronize()
            for g in self:
                g.reset()
            self.clear()
        self.keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class PipelinedWorker:
    def __init__(self, engine, rank: int = 0, world: int = 1, active: bool = True):
        self.engine, self.rank, self.world, self.active = engine, rank, world, active
        from ..ops.table import loss_buffer

        self.loss_sum = loss_buffer(engine.device)
        self.step_idx = 0
        self._next = None
        # pull-ahead: rounds pulled ahead of the one computing (round i at
        # the head, up to i + lookahead - 1), oldest first
        self._pulled: collections.deque = collections.deque()
        self._empty = torch.empty(0, dtype=torch.int64, device=engine.device)
        # hipGraph mode (enable_graph): one captured graph per ring phase
        self._graphs = None
        self._gstep = None      # device int64: the step a replay executes
        self._gbase = 0
        self._gper = 1
        self._cap_base = 0
        # steps this worker has data for (absolute step index bound; None =
        # unbounded, e.g. synthetic data): past it the rank routes empty key
        # sets and skips the model kernels, but keeps entering every
        # collective round as a server until all workers are done
        # (PSEngine.all_done) — the reference's worker finishing on its own
        # while the master waits for the rest (SwiftWorker.h:87-113,
        # worker/terminate.h:37-51, master/terminate.h:44-62)
        self.quota: Optional[int] = None

    # -- subclass hooks
    # optional ``(dd, slot, stream_ptr)`` hook run on the route stream right
    # after the dedup (planning that depends on the key layout only)
    _post_route = None

    def _produce(self, step: int, slot: int, stream) -> torch.Tensor:
        raise NotImplementedError

    def _compute(self, rnd, slot: int, stream_ptr: int) -> None:
        raise NotImplementedError

    def samples_per_step(self) -> int:
        raise NotImplementedError

    # -- driver
    def has_data(self, step: int) -> bool:
        """This rank trains on step ``step`` (a worker within its quota)."""
        return self.active and (self.quota is None or step < self.quota)

    @property
    def done(self) -> bool:
        """No data left for the next step (always true for a pure server)."""
        return not self.has_data(self.step_idx)

    def _route(self, step: int):
        slot = self.engine._next_slot
        if not self.has_data(step):
            return self.engine.route(produce=lambda stream: self._empty)

        def produce(stream):
            return self._produce(step, slot, stream.cuda_stream if stream is not None else None)

        return self.engine.route(produce=produce, post=self._post_route)

    def _gen_kwargs(self, step: int) -> dict:
        """Generator arguments: inside a hipGraph capture the batch index is
        read from the device counter (kernel arguments freeze at capture)."""
        if self._gstep is None or self.engine.capture_tag is None:
            return {}
        return {"step_dev": self._gstep.data_ptr(), "step_delta": step - self._cap_base}

    def enable_graph(self) -> bool:
        """Capture the training step as hipGraphs and replay them from now on.

        The route-buffer ring has ``depth`` slots, so the launch sequence of
        the pipelined step repeats with that period: one graph records
        ``depth`` whole steps on both streams — lookahead route on the route
        stream, pull / fused model kernel / push on the main stream — joined
        at its end, plus the device step counter the data generator reads.
        ``step()`` replays it every ``depth`` steps (the loss buffer then
        holds the loss of the graph's last step).  Replays remove the ~75 us
        of host launch work per step that bounds small batches.  One GPU, or
        N>1 over the xGMI mailboxes (no host counts anywhere in a round);
        synthetic on-device data, an optimizer without per-round host state
        (not Adam) and no tensor-code update rule; returns False otherwise.
        Irreversible."""
        eng = self.engine
        data = getattr(self, "data", None)
        tab = eng.table
        if (not eng.gpu or not (eng.fast1 or getattr(eng, "xg", None) is not None)
                or not getattr(data, "graph_capturable", False)
                or (tab is not None and tab.opt.kind == "adam")
                # a tensor-code update rule syncs the host (its row count)
                or (tab is not None and getattr(tab, "push_fn", None) is not None)
                # a quota decides per step on the host whether to route keys
                or self.quota is not None
                or os.environ.get("SS_GRAPH", "1") == "0"):
            return False
        # more than 4 ranks on one GPU: replays ran every round at ~21.4 ms
        # (word2vec config 3, 8 processes colocated or split 4 + 4, one step
        # or 16 per graph; eager 0.86-1.12 ms, 4 processes replay faster than
        # eager: profiles/raw/r6_config3_split_roles.txt).  The constant
        # 21.4 ms looks like a scheduler time slice: likely more processes'
        # queues than the hardware keeps mapped, a replay's mailbox wait
        # spinning until the peer's queue is mapped again (not profiled)
        xg = getattr(eng, "xg", None)
        if (xg is not None and eng.shared_device
                and eng.world / max(1, getattr(xg, "devices", 1)) > 4
                and os.environ.get("SS_GRAPH", "1") != "force"):
            log.warning("hipGraph replay off: %d ranks share one GPU (eager rounds)", eng.world)
            return False
        if self._graphs is not None:
            return True
        # a pipeline switched to synchronous rounds but not drained still
        # holds pulled-ahead rounds: a capture would record drain steps, not
        # the periodic synchronous step
        self.drain()
        # replays run the server half of a round on the main stream: a
        # capture that forks the server stream in (and joins it back at the
        # end, like the route / pull streams) crashes inside
        # hipStreamEndCapture on the N>1 xGMI path, at the top or the default
        # stream priority alike (tools/exp/graph_server_stream.py); a server
        # stream also made word2vec's N>1 replays 2x slower (0.28 vs 0.135 ms)
        ss = getattr(eng, "server_stream", None)
        if ss is not None:
            torch.cuda.current_stream(eng.device).wait_stream(ss)
            eng.server_stream = None
        if self._next is None:
            self.step()  # prime the lookahead pipeline eagerly
        # N>1: a captured pull runs the keys wait and the server merge unless
        # its round's route ran them (synchronous rounds, PSEngine.route,
        # srv_ahead); the round routed last before the capture must have been
        # routed the way the captured routes are, or the graph's first pull bakes in a second keys wait for
        # its slot and every later replay waits for a round that never comes
        # (word2vec, 4 xGMI ranks: calibrated pulled-ahead, then synchronous
        # rounds, then the capture).  One eager step routes it in this mode.
        if getattr(eng, "xg", None) is not None and not eng.last_route_matches():
            self.step()
        torch.cuda.synchronize()
        self._gstep = torch.full((1,), self.step_idx, dtype=torch.int64, device=eng.device)
        saved = (self.step_idx, self._next, list(self._pulled), eng._next_slot, eng.rounds)
        # steps per graph: `depth` (default: one graph holding a whole ring
        # period, steps inside it overlap across their boundaries; a replay
        # advances `depth` steps) or 1 (SS_GRAPH_STEPS=1: one graph per ring
        # phase, joined at every step).  Measured, batch 1024 / 8192 / 65536:
        # eager 74 / 79 / 309 us, per-step graphs 68 / 92 / 318, ring-period
        # graphs 54 / 75 / 310
        # default: one graph of 4 ring periods.  A replay joins every stream at
        # its end, so the pipeline drains once per graph: word2vec (1M vocab,
        # 16K centers) 4 / 8 / 16 / 32 steps per graph: 0.093 / 0.088 / 0.086 /
        # 0.084 ms/step; sparse LR at batch 65536 unchanged (0.241 / 0.240).
        # SS_GRAPH_STEPS=1 (a graph per step) or any multiple of the depth
        per = 4 * eng.depth
        env = os.environ.get("SS_GRAPH_STEPS", "")
        if env.isdigit() and (int(env) == 1 or (int(env) > 0 and int(env) % eng.depth == 0)):
            per = int(env)
        graphs, pool = [], None
        # no garbage collection inside a capture: a collected object of an
        # earlier worker (its pooled events, streams) would destroy HIP
        # objects mid-capture, which aborts the process
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            for p in range(max(1, eng.depth // per)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    eng.capture_tag = p + 1
                    # fork the route stream into the capture at the start (no
                    # ordering: its work overlaps the whole step)
                    side = [x for x in (eng.route_stream, eng.pull_stream) if x is not None]
                    for x in side:
                        x.wait_stream(torch.cuda.current_stream())
                    self._cap_base = self.step_idx  # what the counter holds at replay
                    for _ in range(per):
                        self._step_eager()
                    cur = torch.cuda.current_stream()
                    for x in side:
                        cur.wait_stream(x)  # join the forked route / pull streams
                    self._gstep.add_(per)  # after the join: no generator still reads it
                pool = g.pool()
                graphs.append(g)
        finally:
            eng.capture_tag = None
            if gc_on:
                gc.enable()
        self._gper = per
        eng.graphed = True  # replays hold ring slots across calls (PSEngine.lookup)
        # the captures only recorded: the device is where it was before them,
        # and after `depth` steps the Python-side pipeline state is periodic
        self.step_idx, self._next, pulled, eng._next_slot, eng.rounds = saved
        self._pulled = collections.deque(pulled)
        self._graphs, self._gbase = _GraphSet(graphs, eng), self.step_idx
        return True

    def close(self) -> None:
        """Drain the device and destroy the captured graphs (before the
        engine's events and arenas go away).  The worker cannot replay
        afterwards; eager steps still work."""
        if self._graphs is not None:
            self._graphs.close()
            self._graphs = None
            self.engine.graphed = False

    def _zero_acc(self) -> None:
        """Zero the per-step device accumulators (the loss) on the current stream."""
        self.loss_sum.zero_()

    def step(self) -> torch.Tensor:
        if self._graphs is not None:
            k = self.step_idx - self._gbase
            if k % self._gper == 0:  # a multi-step graph runs on its first step
                self._graphs[(k // self._gper) % len(self._graphs)].replay()
            self.step_idx += 1
            self.engine.rounds += 1
            return self.loss_sum
        return self._step_eager()

    def _step_eager(self) -> torch.Tensor:
        eng = self.engine
        # pull-ahead, or draining it after it was switched off
        if getattr(eng, "pull_ahead", False) or self._pulled:
            return self._step_pull_ahead()
        r = self._next if self._next is not None else self._route(self.step_idx)
        self._next = self._route(self.step_idx + 1)  # lookahead on the route stream
        rnd = self.engine.pull(r)
        if self.has_data(self.step_idx):
            self._zero_acc()
            with self.engine.trace("compute"):
                self._compute(rnd, r.slot, self.engine.raw_stream())
        else:
            # no compute: a model whose merge kernel moves the loss (sparse
            # LR, word2vec) would otherwise report the previous step's loss
            self.loss_sum.zero_()
        self.engine.push(rnd)
        self.step_idx += 1
        return self.loss_sum

    def _step_pull_ahead(self) -> torch.Tensor:
        """Round i computes/pushes on the main stream while rounds i+1 ..
        i+L are pulled (L = engine.lookahead, the staleness bound) and round
        i+L+1 routed on the side streams.  Switched off, the pipeline drains:
        the pulled rounds compute and push without new pulls, then the
        synchronous pipeline continues from the routed round i+L."""
        eng = self.engine
        ahead = bool(eng.pull_ahead)
        if ahead and not self._pulled:  # (re)start: rounds i .. i+L-1 pulled, i+L routed
            L = max(1, int(getattr(eng, "lookahead", 1)))
            r = self._next if self._next is not None else self._route(self.step_idx)
            self._pulled.append(eng.pull_ahead_round(r))
            for j in range(1, L):
                self._pulled.append(eng.pull_ahead_round(self._route(self.step_idx + j)))
            self._next = self._route(self.step_idx + L)
        rnd = self._pulled.popleft()
        eng.begin(rnd)
        if self.has_data(self.step_idx):
            self._zero_acc()
            with eng.trace("compute"):
                self._compute(rnd, rnd.slot, eng.raw_stream())
        else:
            self.loss_sum.zero_()
        # round i+L's pull is enqueued before round i's push: with one comm
        # stream (RCCL, SS_RCCL_COMMS=1) its exchanges then go ahead of round
        # i's gradients instead of waiting behind round i's compute.  (Issuing
        # route i+2 and pull i+1 before round i's compute measured no better:
        # word2vec one GPU 0.097 -> 0.111 ms/step, N>1 path 0.171 -> 0.167)
        if ahead:
            self._pulled.append(eng.pull_ahead_round(self._next))
        eng.push(rnd)
        if ahead:
            self._next = self._route(self.step_idx + 1 + len(self._pulled))
        self.step_idx += 1
        return self.loss_sum

    def set_pull_ahead(self, on: bool) -> bool:
        """Switch between pulled-ahead (bounded staleness) and synchronous
        rounds between steps.  Off: the rounds already pulled drain over the
        next steps (they still train).  Returns the engine's mode."""
        eng = self.engine
        if on:
            return eng.enable_pull_ahead(True, force=True)
        eng.enable_pull_ahead(False)
        return False

    def drain(self) -> None:
        """Run steps until no pulled-ahead round is outstanding (the engine
        then is in a synchronous state)."""
        while self._pulled and not self.engine.pull_ahead:
            self.step()

    def calibrate_pull_ahead(self, steps: int = 10, windows: int = 2,
                             margin: float = 0.03) -> dict:
        """SS_PULL_AHEAD=auto at N>1: time synchronous and pulled-ahead steps
        on the live world and keep pulled-ahead rounds only if they win
        clearly.  ``windows`` alternating (synchronous, pulled-ahead) windows
        of ``steps`` timed steps each (max over ranks); the mode the model
        runs by default (synchronous for sparse LR, pulled ahead for word2vec
        and FM, which opt in) is kept unless the other beats the window next
        to it by at least ``margin`` in EVERY window.  Eager windows understate
        pulled-ahead rounds under hipGraph replay (word2vec at N>1: 0.105
        ahead vs 0.135 ms sync replayed), so a model that pulls ahead keeps
        doing so unless synchronous rounds win clearly.  A single short window let box noise flip the choice (the
        two modes overlap within a few percent on one GPU), which changes both
        the speed and the staleness semantics of a run.  On one GPU shared by
        all ranks there is no cross-device wait to hide and the synchronous
        snapshot update wins; across real xGMI links the keys -> rows chain of
        the next round can hide behind this round's compute.  Returns the
        choice, the per-window timings (ms per step, slowest rank) and the
        per-window spread over ranks, {} where it does not apply (one-GPU path,
        host-count transports without a pull stream, SS_PULL_AHEAD=0/1,
        SS_STALENESS=0).  A collective: every rank calls it."""
        eng = self.engine
        if not (getattr(eng, "gpu", False) and getattr(eng, "dist", False) and eng.depth >= 3
                and os.environ.get("SS_PULL_AHEAD", "auto") == "auto"
                and getattr(eng, "lookahead", 1) > 0 and self._graphs is None
                and os.environ.get("SS_STALENESS", "1") != "0"):
            return {}
        steps, windows = max(1, int(steps)), max(1, int(windows))
        # the model's own mode (pulled ahead for word2vec / FM, synchronous
        # for sparse LR) is kept unless the other wins clearly in every window
        default = bool(eng.pull_ahead)
        times = {False: [], True: []}
        spread = {False: [], True: []}
        for _ in range(windows):
            for mode in (False, True):
                self.set_pull_ahead(mode)
                self.drain()
                for _ in range(2):  # settle: the (re)started pipeline
                    self.step()
                torch.cuda.synchronize(eng.device)
                eng.barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    self.step()
                torch.cuda.synchronize(eng.device)
                el = time.perf_counter() - t0
                eng.barrier()
                hi = eng.max_over_ranks(el) / steps
                lo = -eng.max_over_ranks(-el) / steps
                times[mode].append(hi)
                spread[mode].append(hi - lo)
        if default:
            best = not all(s <= (1.0 - margin) * a for s, a in zip(times[False], times[True]))
        else:
            best = all(a <= (1.0 - margin) * s for s, a in zip(times[False], times[True]))
        pick = os.environ.get("SS_CAL_PICK", "")  # debug: force the outcome
        if pick in ("sync", "ahead"):
            best = pick == "ahead"
        self.set_pull_ahead(best)
        self.drain()
        ms = lambda xs: [round(1e3 * x, 4) for x in xs]  # noqa: E731
        return {"pull_ahead": best, "default": default,
                "staleness": eng.lookahead if best else 0,
                "sync_ms": ms(times[False]), "ahead_ms": ms(times[True]),
                "rank_spread_ms": {"sync": ms(spread[False]), "ahead": ms(spread[True])},
                "windows": windows, "steps_per_window": steps, "margin": margin}

    def calibrate_server_stream(self, steps: int = 10, windows: int = 2,
                                margin: float = 0.01) -> dict:
        """SS_SERVER_STREAM=auto at N>1 with a device per rank: the server
        half of every round on its own top-priority stream lets a peer's
        rows leave while this rank's compute is slow (a straggler absorbs
        43 % instead of 21 % of a device delay, profiles/
        r5_n_gt_1_straggler_lookup.md) but costs an extra stream's hand-offs
        when no rank straggles (one rank: 1.087 vs 1.064 ms).  Time
        ``windows`` alternating (off, on) windows on the live world in the
        current round mode and keep the stream only if it is within
        ``margin`` of the step without it in EVERY window.  A collective.
        Returns {} where it does not apply."""
        eng = self.engine
        if not (getattr(eng, "gpu", False) and getattr(eng, "dist", False)
                and getattr(eng, "server_stream", None) is not None
                and os.environ.get("SS_SERVER_STREAM", "auto") == "auto"
                and self._graphs is None):
            return {}
        steps, windows = max(1, int(steps)), max(1, int(windows))
        times = {False: [], True: []}
        for _ in range(windows):
            for on in (False, True):
                eng.set_server_stream(on)
                for _ in range(2):
                    self.step()
                torch.cuda.synchronize(eng.device)
                eng.barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    self.step()
                torch.cuda.synchronize(eng.device)
                el = time.perf_counter() - t0
                eng.barrier()
                times[on].append(eng.max_over_ranks(el) / steps)
        keep = all(a <= (1.0 + margin) * s for s, a in zip(times[False], times[True]))
        pick = os.environ.get("SS_CAL_SERVER_STREAM", "")  # debug: force the outcome
        if pick in ("0", "1"):
            keep = pick == "1"
        eng.set_server_stream(keep)
        ms = lambda xs: [round(1e3 * x, 4) for x in xs]  # noqa: E731
        return {"server_stream": keep, "off_ms": ms(times[False]), "on_ms": ms(times[True]),
                "windows": windows, "steps_per_window": steps, "margin": margin}

    @staticmethod
    def calibrate_exchange(cands: dict, default: str, steps: int = 10, windows: int = 2,
                           margin: float = 0.03) -> tuple:
        """Time workers that train the same model through different N>1
        exchanges (``cands``: name -> worker, every worker's engine on the
        same table, e.g. ``unique`` and ``records``) on the live world, in
        ``windows`` alternating windows of ``steps`` timed steps (max over
        ranks), and pick ``default`` unless another's best window beats the
        default's best window by ``margin``.  Which one is faster is a property of the machine: the
        record exchange does less kernel work per rank (no worker dedup or
        merge) but ships every occurrence, twice the unique exchange's link
        bytes — on one GPU (no links) it wins at 1-2 ranks and loses at 4-8
        (docs/PERFORMANCE.md), over real xGMI links only a measurement can
        tell.  Between windows the device is synchronised and the ranks
        barrier: the engines share the table, so one worker's rounds must be
        applied before the other pulls.  Workers run synchronous rounds here.
        A collective.  Returns (choice, report)."""
        names = list(cands)
        if default not in cands:
            raise ValueError("calibrate_exchange: the default must be a candidate")
        steps, windows = max(1, int(steps)), max(1, int(windows))
        times = {n: [] for n in names}

        def sync(eng):
            if getattr(eng, "gpu", False):
                torch.cuda.synchronize(eng.device)

        def quiesce(eng):
            sync(eng)
            eng.barrier()

        for _ in range(windows):
            for n in names:
                w = cands[n]
                eng = w.engine
                if getattr(eng, "pull_ahead", False) or w._pulled or w._graphs is not None:
                    raise RuntimeError("calibrate_exchange: synchronous eager rounds only")
                quiesce(eng)
                for _ in range(2):  # settle
                    w.step()
                quiesce(eng)
                t0 = time.perf_counter()
                for _ in range(steps):
                    w.step()
                sync(eng)
                el = time.perf_counter() - t0
                eng.barrier()
                times[n].append(eng.max_over_ranks(el) / steps)
        # each candidate's BEST window: noise (a cold first window, a busy
        # peer) only ever slows a window down, so the minimum is what the
        # exchange can do — the every-window rule let one slow first window
        # of records (2.25 vs 1.75 ms, 2 ranks) keep the slower unique
        best = default
        for n in names:
            if n != default and min(times[n]) <= (1.0 - margin) * min(times[default]):
                if best == default or min(times[n]) < min(times[best]):
                    best = n
        pick = os.environ.get("SS_CAL_XCHG", "")  # debug: force the outcome
        if pick in cands:
            best = pick
        quiesce(cands[best].engine)
        ms = lambda xs: [round(1e3 * x, 4) for x in xs]  # noqa: E731
        return best, {"exchange": best, "default": default,
                      **{f"{n}_ms": ms(times[n]) for n in names},
                      "windows": windows, "steps_per_window": steps, "margin": margin}

    def rounds_done(self) -> int:
        """Rounds whose pushes have been enqueued on the device.  Eagerly
        that is ``step_idx``; with hipGraphs a replay runs ``per`` steps on
        the first step of its period, so the device is up to the end of the
        current period (a backup taken now holds those rounds and must be
        labelled with them, or a resume would apply them twice)."""
        if self._graphs is None:
            return self.step_idx
        k = self.step_idx - self._gbase
        return self._gbase + -(-k // self._gper) * self._gper

    def mean_loss(self) -> float:
        n = self.samples_per_step()
        return float(self.loss_sum.sum().item()) / n if n else 0.0


EVAL_STEP = 1 << 28  # held-out sample range of the synthetic CTR generators


def evaluate_ctr(worker, batches: int, logits) -> dict:
    """Held-out metrics of a CTR model (sparse LR, FM) on fresh synthetic
    batches: AUC / log-loss of the learned logits and of the planted
    ground-truth logits the labels were drawn from (the Bayes-optimal
    reference).  Reads the table without inserting (unseen keys read zero).
    World > 1: a COLLECTIVE — every rank calls it; each worker rank scores
    its own held-out samples through ``PSEngine.lookup`` (the read-only pull
    from every shard) and the metrics are over all ranks' samples.
    ``logits(rows [B*F, D], B, F)`` -> [B] tensor."""
    import numpy as np

    from ..models.ctr_data import truth_weight
    from ..utils.metrics import auc, logloss

    eng, d = worker.engine, worker.data
    dev = eng.device
    B, F = d.batch_size, d.num_fields
    keys = torch.empty(B * F, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    empty = torch.empty(0, dtype=torch.int64, device=dev)
    zs, zt, ys = [], [], []
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)  # the route stream may still be producing
    for b in range(batches):
        if not worker.active:
            eng.lookup(empty)  # a pure server still answers the round
            continue
        d.generate(EVAL_STEP + b, worker.rank, worker.world, keys, labels)
        rows = eng.lookup(keys)
        zs.append(logits(rows, B, F).float().cpu().numpy())
        k = keys.cpu().numpy().view(np.uint64)
        zt.append(truth_weight(k, d.truth_scale).reshape(B, F).sum(1) + d.truth_bias)
        ys.append(labels.cpu().numpy())
    cat = (lambda xs: np.concatenate(xs) if xs else np.zeros(0))  # noqa: E731
    z, t, y = cat(zs), cat(zt), cat(ys)
    if worker.world > 1:
        import torch.distributed as dist

        parts = [None] * worker.world
        dist.all_gather_object(parts, (z, t, y))
        z, t, y = (np.concatenate([p[i] for p in parts]) for i in range(3))
    return {"auc": auc(z, y), "logloss": logloss(z, y), "auc_truth": auc(t, y),
            "logloss_truth": logloss(t, y), "samples": int(y.size)}
