"""Factorization machine on a wide embedding table (BASELINE config 5:
FM-style wide table, 10B keys sharded across 8x288 GB HBM, async AdaGrad).

Each key's row is ``[w | v_0..v_{K-1}]`` (dim = 1 + K) — the second-order FM
of Rendle (2010) with binary features:

    z = sum_i w_i + 1/2 * sum_f [(sum_i v_if)^2 - sum_i v_if^2]

Sizing (``HbmTable.plan``): 10B keys, K=8, AdaGrad -> width 18 floats,
80-byte slots; 10e9/8 shards/0.7 load = 1.79e9 slots = 143 GB per MI355X,
well inside 288 GB (``plan_fm_table`` reports this).  "Async" here means the
reference's Hogwild semantics carried over: workers never wait for each
other beyond the lockstep collective round.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from .._native import hip
from ..ops.optim import InitConfig, Optimizer
from ..ops.table import HbmTable
from .base import PipelinedWorker, evaluate_ctr
from .sparse_lr import CtrSynth


def fm_table_args(k: int, optimizer: Optional[Optimizer] = None):
    opt = optimizer or Optimizer("adagrad", lr=0.05)
    init = InitConfig("normal", scale=0.01, state_init=0.0)
    return opt, init


def plan_fm_table(n_keys: int, k: int = 8, shards: int = 8, load: float = 0.7,
                  row_dtype: str = "fp32") -> dict:
    """Per-shard table plan of the config-5 FM table; ``row_dtype="bf16"``
    (compact rows) halves the row bytes: 10B keys at K = 16 are ~1.94 TB at
    fp32 (past 8 x 288 GB with the slot keys) and fit as bf16 rows."""
    p = HbmTable.plan(n_keys // shards, 1 + k, Optimizer("adagrad"), load, row_dtype)
    p["GB_per_shard"] = round(p["bytes"] / 1e9, 1)
    return p


class FMWorker(PipelinedWorker):
    def __init__(self, engine, data: CtrSynth, rank: int = 0, world: int = 1,
                 active: bool = True):
        if engine.dim not in (2, 5, 9, 17):
            raise ValueError("FMWorker: dim must be 1+K with K in {1,4,8,16}")
        super().__init__(engine, rank, world, active)
        self.data = data
        # the route stream is the light one for this model: pull the next
        # round's rows behind its dedup (bounded staleness 1)
        engine.enable_pull_ahead()
        dev = engine.device
        B, F = data.batch_size, data.num_fields
        self.keys = [torch.empty(B * F, dtype=torch.int64, device=dev) for _ in range(engine.depth)]
        self.labels = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(engine.depth)]
        # Atomic-free path (bucketed dedup, F <= 64): the forward emits per-sample
        # factors (gs, gs * sum v) and one workgroup per dedup bucket builds each
        # unique key's gradient row in LDS (bdedup.hip k_bd_reduce_fm).  Otherwise
        # the fused kernel adds per-occurrence rows with float atomics.
        K = engine.dim - 1
        lanes = 1 << max(0, (F - 1).bit_length())
        self.bucketed = (F <= 64 and lanes >= K and
                         all(getattr(dd, "mode", None) == "bucket" for dd in engine.dedupers))
        if self.bucketed:
            for dd in engine.dedupers:
                dd.zero_grad = False
                dd.materialize_inv = False  # the forward resolves luid[pos_of[j]] itself
            self.gs = torch.empty(B, dtype=torch.float32, device=dev)
            self.gss = torch.empty(B * K, dtype=torch.float32, device=dev)
            # overflow-bucket list of the sorted reduce (buckets too large to
            # sort in LDS go to the LDS-atomic form)
            self.ovf = torch.zeros(hip().bd_fm_ovf_words(B * F), dtype=torch.int32, device=dev)

    def _produce(self, step, slot, stream):
        self.data.generate(step, self.rank, self.world, self.keys[slot], self.labels[slot],
                           stream=stream, **self._gen_kwargs(step))
        return self.keys[slot]

    def _compute(self, rnd, slot, st):
        d = self.data
        if self.bucketed:
            h, o, dd = hip(), rnd.dd.owner, rnd.dd
            h.fm_fwd_g(0, o.index_ptrs(dd.n), self.labels[slot].data_ptr(),
                       d.batch_size, d.num_fields, self.engine.dim, rnd.uvals.data_ptr(),
                       self.gs.data_ptr(), self.gss.data_ptr(), self.loss_sum.data_ptr(), 0, st)
            # the sorted per-bucket merge sums each unique key's gradient row
            # once and stores it; the AdaGrad update is the separate lane-group
            # apply (k_apply_st, ~140 us: the random read-modify-write floor
            # of 1.35M 72-byte rows).  SS_FM_FUSE=1 fuses the update into the
            # merge instead — the row moved as 8- + 16-byte vectors per thread,
            # its loads issued before the occurrence gathers (bdedup.hip
            # fm9_row_update): measured 0.570-0.573 vs 0.542-0.546 ms per step
            # (two A/B pairs, round 6; the scalar fused form: 0.62 -> 1.04 ms),
            # the extra row registers cost the merge's occupancy more than the
            # gradient-row round trip it saves
            fa = (self.engine.fuse_apply(rnd, snapshot=False)
                  if os.environ.get("SS_FM_FUSE", "0") == "1" else None)
            kw = {}
            if fa is not None:
                assert not fa["slot32"]  # FM slots are never 4-byte (slot32: scalar rows)
                kw = {"t": fa["t"], "slots": fa["slots"], "op": fa["op"]}
            h.bd_reduce_fm(dd.lay, dd.nranks, o.scratch.data_ptr(), o.pj.data_ptr(),
                           o.luid.data_ptr(), self.gs.data_ptr(), self.gss.data_ptr(),
                           d.num_fields, self.engine.dim, rnd.uvals.data_ptr(),
                           rnd.ugrad.data_ptr(), st, self.ovf.data_ptr(), ndest=o.ndest, **kw)
            return
        hip().fm_fwd_bwd(rnd.inv.data_ptr(), self.labels[slot].data_ptr(), d.batch_size,
                         d.num_fields, self.engine.dim, rnd.uvals.data_ptr(),
                         rnd.ugrad.data_ptr(), self.loss_sum.data_ptr(), 0, st)

    def samples_per_step(self) -> int:
        return self.data.batch_size if self.active else 0

    def evaluate(self, batches: int = 1) -> dict:
        """Held-out AUC / log-loss of the FM logits vs the planted ground
        truth (models/base.py evaluate_ctr; unseen keys contribute zero).
        World > 1: collective, over every shard (read-only pull)."""
        D = self.engine.dim
        return evaluate_ctr(self, batches, lambda rows, B, F: fm_logits(rows.view(B, F, D)))


def fm_logits(rows: torch.Tensor) -> torch.Tensor:
    """FM logits of [B, F, 1 + K] rows: sum_i w_i + 1/2 sum_f [(sum_i v_if)^2
    - sum_i v_if^2]."""
    w, v = rows[..., 0], rows[..., 1:]
    return w.sum(1) + 0.5 * (v.sum(1) ** 2 - (v * v).sum(1)).sum(-1)


def fm_reference(rows: np.ndarray, labels: np.ndarray):
    """fp64 reference for one batch. rows [B, F, dim] (occurrence rows).
    Returns (loss_sum, pred [B], grad rows [B, F, dim])."""
    R = rows.astype(np.float64)
    w, v = R[..., 0], R[..., 1:]
    s = v.sum(1)                                   # [B, K]
    z = w.sum(1) + 0.5 * ((s ** 2).sum(1) - (v ** 2).sum((1, 2)))
    p = 1.0 / (1.0 + np.exp(-z))
    y = labels.astype(np.float64)
    loss = float(np.sum(np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z))) - y * z))
    g = (p - y)[:, None, None]
    grad = np.empty_like(R)
    grad[..., 0] = g[..., 0]
    grad[..., 1:] = g * (s[:, None, :] - v)
    return loss, p, grad
