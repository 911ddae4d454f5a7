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

import torch


class PipelinedWorker:
    def __init__(self, engine, rank: int = 0, world: int = 1, active: bool = True):
        self.engine, self.rank, self.world, self.active = engine, rank, world, active
        from ..ops.table import loss_buffer

        self.loss_sum = loss_buffer(engine.device)
        self.step_idx = 0
        self._next = None
        self._cur = None
        self._empty = torch.empty(0, dtype=torch.int64, device=engine.device)

    # -- subclass hooks
    def _produce(self, step: int, slot: int, stream) -> torch.Tensor:
        raise NotImplementedError

    def _compute(self, rnd, slot: int, stream_ptr: int) -> None:
        raise NotImplementedError

    def samples_per_step(self) -> int:
        raise NotImplementedError

    # -- driver
    def _route(self, step: int):
        slot = self.engine._next_slot
        if not self.active:
            return self.engine.route(produce=lambda stream: self._empty)

        def produce(stream):
            return self._produce(step, slot, stream.cuda_stream if stream is not None else None)

        return self.engine.route(produce=produce)

    def step(self) -> torch.Tensor:
        eng = self.engine
        if getattr(eng, "pull_ahead", False):
            return self._step_pull_ahead()
        r = self._next if self._next is not None else self._route(self.step_idx)
        self._next = self._route(self.step_idx + 1)  # lookahead on the route stream
        rnd = self.engine.pull(r)
        self.loss_sum.zero_()
        if self.active:
            self._compute(rnd, r.slot, torch.cuda.current_stream().cuda_stream)
        self.engine.push(rnd)
        self.step_idx += 1
        return self.loss_sum

    def _step_pull_ahead(self) -> torch.Tensor:
        """N>1: round i computes/pushes on the main stream while round i+1 is
        pulled and round i+2 routed on the route stream (staleness 1)."""
        eng = self.engine
        if self._cur is None:  # bootstrap the pipeline
            r = self._next if self._next is not None else self._route(self.step_idx)
            self._cur = eng.pull_ahead_round(r)
            self._next = self._route(self.step_idx + 1)
        rnd = self._cur
        eng.begin(rnd)
        self.loss_sum.zero_()
        if self.active:
            self._compute(rnd, rnd.slot, torch.cuda.current_stream().cuda_stream)
        eng.push(rnd)
        self._cur = eng.pull_ahead_round(self._next)
        self._next = self._route(self.step_idx + 2)
        self.step_idx += 1
        return self.loss_sum

    def mean_loss(self) -> float:
        n = self.samples_per_step()
        return float(self.loss_sum.sum().item()) / n if n else 0.0
