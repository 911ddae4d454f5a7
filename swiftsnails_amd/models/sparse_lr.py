"""Sparse logistic regression on the parameter server (BASELINE headline model).

The reference names a ``logistic_regression`` app that is absent from the
snapshot (/root/reference/src/tools/hadoop-server.sh:7, distribute.sh:8); its
worker would ``pull_with_barrier`` the batch's keys, compute per-sample
sigmoid(w·x) and push the per-key gradients (SwiftWorker/BaseAlgorithm::train,
/root/reference/src/core/framework/SwiftWorker.h:19-30).  This module is that
worker on MI355X:

    step:  gen batch (device)  ->  pull (dedup/route/[a2av]/probe-init-gather)
           ->  fused LR fwd/bwd kernel  ->  push (AdaGrad apply on the servers)

Synthetic CTR data (``CtrSynth``): ``num_fields`` categorical fields, field f
owning key range [f*V, (f+1)*V) of a ``num_features``-wide feature space
(1B in the headline config), log-uniform (Zipf-like) ids with a uniform tail,
labels drawn from a hidden ground-truth sparse LR model so loss goes down.
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .._native import hip
from ..ops.optim import InitConfig, Optimizer
from ..ops.table import HbmTable
from .base import PipelinedWorker, evaluate_ctr


@dataclass
class CtrSynth:
    batch_size: int = 65536
    num_fields: int = 39
    num_features: int = 1_000_000_000
    tail_frac: float = 0.1
    truth_scale: float = 1.0
    truth_bias: float = -1.0
    seed: int = 20150404

    @property
    def vocab_per_field(self) -> int:
        return max(1, self.num_features // self.num_fields)

    graph_capturable = True  # generate() can take its step from device memory

    def generate(self, step: int, rank: int, world: int, keys: torch.Tensor, labels: torch.Tensor,
                 stream=None, step_dev: int = 0, step_delta: int = 0):
        """Batch of global step ``step`` (samples [(step*world+rank)*B, +B)).
        With ``step_dev`` (a device int64 pointer; hipGraph replays) the step
        is ``*step_dev + step_delta`` instead, read by the kernel."""
        B, F = self.batch_size, self.num_fields
        base = (step * world + rank) * B
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        hip().gen_ctr(self.seed, base, B, F, self.vocab_per_field, self.tail_frac,
                      self.truth_scale, self.truth_bias, keys.data_ptr(), labels.data_ptr(), st,
                      step_dev, world * B, (step_delta * world + rank) * B)


class SparseLRWorker(PipelinedWorker):
    """Trains sparse LR through a ``PSEngine`` (one per rank).

    The batch of step i+1 is generated, deduplicated and routed on the
    engine's route stream while step i computes (one batch of lookahead; no
    parameter staleness — routing does not read parameters)."""

    def __init__(self, engine, data: CtrSynth, rank: int = 0, world: int = 1,
                 active: bool = True, grad_mode: str = "segreduce"):
        super().__init__(engine, rank, world, active)
        self.data = data
        dev = engine.device
        B, F = data.batch_size, data.num_fields
        n = B * F
        self.keys = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(engine.depth)]
        self.labels = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(engine.depth)]
        # feature values (file data with idx:val entries); synthetic data is binary
        self.xval = ([torch.empty(n, dtype=torch.float32, device=dev) for _ in range(engine.depth)]
                     if getattr(data, "has_values", False) else None)
        # grad_mode "segreduce": duplicate merge without global atomics.  With
        # the bucketed deduper (default) the dedup partition is the reduction
        # plan: the forward writes per-sample gradients and one workgroup per
        # bucket sums g*x over the bucket's occurrences in LDS and stores each
        # unique row once (so the deduper need not zero the gradient rows).
        # With the hash deduper the separate bin plan of segreduce.hip is
        # built on the route stream instead.  "atomic": one float atomicAdd
        # per occurrence.
        self.grad_mode = grad_mode
        self.bucketed = grad_mode == "segreduce" and all(
            getattr(dd, "mode", None) == "bucket" for dd in engine.dedupers)
        if grad_mode == "segreduce":
            # per-sample gradients (bucketed) or per-occurrence g*x (bin plan)
            self.gocc = torch.empty(B if self.bucketed else n, dtype=torch.float32, device=dev)
        # bucketed: parameters are filled per dedup bucket into
        # occurrence-position order (k_bd_fill_occ) and the forward reads one
        # word per occurrence, occ[pos_of[j]], instead of the dependent
        # gathers luid[pos_of[j]] -> uvals[ubase + luid] (0.941 -> 0.887
        # ms/step); the scatter then skips the bucket-of-occurrence array
        self.occ = torch.empty(n, dtype=torch.float32, device=dev) if self.bucketed else None
        if self.bucketed:
            # the forward adds the loss into _acc; the merge moves it to
            # loss_sum and leaves _acc zero (see _compute)
            self._acc = torch.zeros_like(self.loss_sum)
            # every pulled round is pushed through the fused snapshot merge:
            # the one-GPU engine may claim new keys' slots in the pull and let
            # the merge store them (PSEngine.claim, table.hip k_pull_claim_bk)
            engine.claim_rounds = True
            engine.claim_occ = self.occ  # ... and the claimed pull fills it (no fill_occ)
            for dd in engine.dedupers:
                dd.zero_grad = False         # the LDS reduce stores every unique row
                dd.materialize_inv = False   # the forward resolves occurrences itself
                dd.need_bkt = False
        elif grad_mode == "segreduce":
            h = hip()
            self.nbins = h.sr_nbins(n)
            self.hist = [torch.empty(h.sr_hist_words(n), dtype=torch.int32, device=dev)
                         for _ in range(engine.depth)]
            self.plan = [torch.empty(n, dtype=torch.int64, device=dev)
                         for _ in range(engine.depth)]
            mi = h.sr_max_items(n)
            self.items = [torch.empty(4 * mi, dtype=torch.int32, device=dev)
                          for _ in range(engine.depth)]
            self.nitems = [torch.zeros(1, dtype=torch.int32, device=dev)
                           for _ in range(engine.depth)]
        if getattr(engine, "records", False) and not self.bucketed:
            raise ValueError("the record exchange needs the bucketed segreduce merge "
                             "(SS_DEDUP=bucket, grad_mode segreduce)")
        # N>1 record exchange (PSEngine exchange="records"): the forward reads
        # the rows mailbox in place, its own records' rows from the cached
        # buffer its server filled (Round.own_vals), and the server merge reads
        # those records' gradients from the per-sample gradient through spj —
        # so that gradient is kept per ring slot (a server-stream merge of
        # round i may still read it while round i+1 computes)
        self.gring = ([torch.empty(B, dtype=torch.float32, device=dev)
                       for _ in range(engine.depth)]
                      if self.bucketed and getattr(engine, "own_vals", None) is not None else None)

    def _zero_acc(self) -> None:
        if not self.bucketed:
            self.loss_sum.zero_()

    def _post(self, dd, slot, st):
        hip().sr_plan(dd.inv.data_ptr(), dd.n, dd.ucount.data_ptr(), dd.nranks, dd.ucap,
                      self.hist[slot].data_ptr(), self.nbins, self.plan[slot].data_ptr(),
                      self.items[slot].data_ptr(), self.nitems[slot].data_ptr(), st)

    def _route(self, step: int):
        if not self.has_data(step):
            return super()._route(step)
        eng = self.engine
        slot = eng._next_slot
        return eng.route(produce=lambda stream: self._produce(step, slot, stream.cuda_stream),
                         post=None if (self.bucketed or self.grad_mode != "segreduce")
                         else self._post)

    def _produce(self, step, slot, stream):
        if self.xval is not None:
            self.data.generate(step, self.rank, self.world, self.keys[slot], self.labels[slot],
                               stream=stream, xval=self.xval[slot], **self._gen_kwargs(step))
        else:
            self.data.generate(step, self.rank, self.world, self.keys[slot], self.labels[slot],
                               stream=stream, **self._gen_kwargs(step))
        return self.keys[slot]

    def _compute(self, rnd, slot, st):
        d = self.data
        h = hip()
        dd = rnd.dd
        xp = self.xval[slot].data_ptr() if self.xval is not None else 0
        if self.bucketed and self.engine.records:
            # N>1 record exchange: the rows came back per occurrence at its
            # send-segment position (the forward reads occ[pos_of[j]] there),
            # the gradients go out the same way — no worker merge; the
            # servers merge per distinct key with the AdaGrad update fused
            o, eng = dd.owner, self.engine
            own = rnd.own_vals is not None and self.gring is not None
            gs = self.gring[slot] if own else self.gocc
            lo = eng.rank * o.ucap
            h.lr_fwd_g(0, xp, self.labels[slot].data_ptr(), d.batch_size, d.num_fields,
                       rnd.uvals.data_ptr(), gs.data_ptr(), 1, self._acc.data_ptr(),
                       0, st, o.index_ptrs(dd.n), occ=rnd.uvals.data_ptr(),
                       own=rnd.own_vals.data_ptr() if own else 0, own_lo=lo if own else 0,
                       own_hi=lo + o.ucap if own else 0)
            # the peers' records' gradients out per occurrence (own: skipped,
            # the push hands the server merge (gs, spj, F, x) instead)
            h.rec_grad(dd.ucount.data_ptr(), eng.world, o.ucap, o.spj.data_ptr(),
                       gs.data_ptr(), xp, d.num_fields, rnd.ugrad.data_ptr(), st,
                       acc=self._acc.data_ptr(), acc_out=self.loss_sum.data_ptr(),
                       acc_n=self._acc.numel(), skip=eng.rank if own else -1)
            if own:
                rnd.own_grad = (gs.data_ptr(), o.spj.data_ptr(), d.num_fields, xp)
        elif self.bucketed:
            o = dd.owner
            if not rnd.occ_filled:
                o.fill_occ(dd.n, rnd.uvals, self.occ, stream=st)
            h.lr_fwd_g(0, xp, self.labels[slot].data_ptr(), d.batch_size, d.num_fields,
                       rnd.uvals.data_ptr(), self.gocc.data_ptr(), 1, self._acc.data_ptr(),
                       0, st, o.index_ptrs(dd.n), occ=self.occ.data_ptr())
            # one GPU: the merge kernel runs the AdaGrad update itself
            # (engine.fuse_apply: pull snapshot still valid), push() then only
            # does the bookkeeping; N>1: compact rows in the send layout
            fa = self.engine.fuse_apply(rnd)
            # the merge also moves the step's loss out of the forward's
            # accumulator and zeroes it (no zero-fill launch per step)
            h.bd_reduce(dd.lay, dd.nranks, o.scratch.data_ptr(), o.pj.data_ptr(),
                        o.luid.data_ptr(), self.gocc.data_ptr(), xp, d.num_fields,
                        rnd.ugrad.data_ptr(), st, 0, 0, ndest=o.ndest, acc=self._acc.data_ptr(),
                        acc_out=self.loss_sum.data_ptr(), acc_n=self._acc.numel(), **(fa or {}))
        elif self.grad_mode == "segreduce":
            h.lr_fwd_g(rnd.inv.data_ptr(), xp, self.labels[slot].data_ptr(), d.batch_size,
                       d.num_fields, rnd.uvals.data_ptr(), self.gocc.data_ptr(), 0,
                       self.loss_sum.data_ptr(), 0, st)
            h.sr_reduce(self.plan[slot].data_ptr(), self.gocc.data_ptr(),
                        self.items[slot].data_ptr(), self.nitems[slot].data_ptr(), dd.n,
                        dd.ucount.data_ptr(), dd.nranks, dd.ucap, rnd.ugrad.data_ptr(), st)
        else:
            h.lr_fwd_bwd(rnd.inv.data_ptr(), xp, self.labels[slot].data_ptr(), d.batch_size,
                         d.num_fields, rnd.uvals.data_ptr(), rnd.ugrad.data_ptr(),
                         self.loss_sum.data_ptr(), 0, st)

    def samples_per_step(self) -> int:
        return self.data.batch_size if self.active else 0

    def evaluate(self, batches: int = 1) -> dict:
        """Held-out AUC / log-loss of the current model vs the planted
        ground truth (models/base.py evaluate_ctr).  World > 1: collective,
        over every shard through the engine's read-only pull."""
        return evaluate_ctr(self, batches, lambda rows, B, F: rows.view(B, F).sum(1))


def lr_init(kind: str = "zero", scale: float = 0.01) -> InitConfig:
    """Weight initialiser of a sparse-LR table: ``zero`` (the usual LR start;
    the table is prefilled, an insert is the key CAS alone) or ``uniform``
    (random (u - 0.5) * scale per key, drawn from a key-seeded hash when the
    key is inserted — the word2vec convention of vec1.h:223-226)."""
    if kind not in ("zero", "uniform"):
        raise ValueError("sparse LR init: zero or uniform")
    return InitConfig("zero") if kind == "zero" else InitConfig("uniform", scale)


def make_lr_table(num_features: int, world: int = 1, optimizer: Optional[Optimizer] = None,
                  load: float = 0.7, device=None, capacity: Optional[int] = None,
                  init: Optional[InitConfig] = None) -> HbmTable:
    """Shard sized for the whole feature space split over `world` servers."""
    opt = optimizer or Optimizer("adagrad", lr=0.05, eps=1e-8)
    cap = capacity or int(num_features / world / load) + 1024
    return HbmTable(1, cap, optimizer=opt, init=init or InitConfig("zero"), device=device)
