"""word2vec skip-gram with (shared) negative sampling on the parameter server.

BASELINE config 3: 1M-vocab synthetic corpus, 4 servers + 4 workers on 4
MI355X (4 colocated ranks: each GPU one server shard and one worker).  The
reference's word2vec app is absent from the snapshot (named by
/root/reference/src/tools/copy_exec.sh:4-9); its corpus generator
(src/tools/gen-word2vec-data.py: lines of 6-15 random word ids) is mirrored by
``W2VSynth`` at scale, and the dense-vector math of utils/vec1.h (dot, scaled
add, random init (u-0.5)/size) lives in the fused ``k_w2v_sgns`` kernel
(csrc/hip/w2v.hip) which runs the shared-negative GEMMs on MFMA.

Parameters: one table of ``dim``-float rows.  Input vectors (syn0) are keyed
by the word id, output vectors (syn1neg) by ``id | 1<<40``; the output
namespace starts at zero (``InitConfig.zero_key_bit=40``), the input one at
``(u-0.5)/dim`` like the reference's Vec::randInit.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .._native import hip
from ..ops.optim import InitConfig, Optimizer
from .base import PipelinedWorker

OUT_BIT = 40
TILE = 64      # centers per workgroup tile
NEG_TILE = 64  # shared negatives per tile


class W2VLayout:
    """Key layout shared by the synthetic and the file-fed sources.

    ``mode="window"`` (default; csrc/include/ss/w2v_window.h): a batch is a
    run of ``B + 2W`` consecutive stream positions, keys = [B centers | B + 2W
    run positions (output namespace) | negatives] plus one int32 meta word per
    run position (sentence tag, reduced window, mask); the contexts of a
    center are its run neighbours, as in word2vec's sliding window.
    ``mode="pairs"``: i.i.d. centers with 2W sampled contexts each, keys =
    [B centers | B x 2W contexts | negatives].

    ``neg_mode="shared"`` (default): each 64-center tile trains against 64
    shared negatives weighted to K per pair (GEMMs on the MFMA);
    ``"per_pair"`` (window mode): word2vec's own objective, K negatives drawn
    for every positive pair (B x 2W x K negative keys per step)."""

    neg_mode = "shared"

    @property
    def n_neg(self) -> int:
        if getattr(self, "neg_mode", "shared") == "per_pair":
            return self.batch_size * self.contexts * self.negatives
        return self.tiles * NEG_TILE

    @property
    def contexts(self) -> int:
        return 2 * self.window

    @property
    def tiles(self) -> int:
        return (self.batch_size + TILE - 1) // TILE

    @property
    def run_len(self) -> int:
        return self.batch_size + 2 * self.window

    @property
    def n_keys(self) -> int:
        if self.mode == "window":
            return self.batch_size + self.run_len + self.n_neg
        return self.batch_size * (1 + self.contexts) + self.n_neg

    @property
    def neg_scale(self) -> float:
        """pairs layout: weight of each shared negative (2W pairs x K / S)."""
        return self.contexts * self.negatives / NEG_TILE

    @property
    def neg_per_pair(self) -> float:
        """window layout: per-pair weight K / S (a center with n pairs weighs
        its shared negatives n K / S)."""
        return self.negatives / NEG_TILE

    def _check_mode(self):
        if self.mode not in ("window", "pairs"):
            raise ValueError(f"word2vec batch mode must be window or pairs, not {self.mode!r}")
        if self.mode == "window" and not 1 <= self.window <= 15:
            raise ValueError("window mode: window must be in [1, 15]")
        if self.neg_mode not in ("shared", "per_pair"):
            raise ValueError(f"word2vec neg_mode must be shared or per_pair, not {self.neg_mode!r}")
        if self.neg_mode == "per_pair" and (self.mode != "window" or not 1 <= self.negatives <= 16):
            raise ValueError("per_pair negatives: window mode, 1..16 negatives per pair")


@dataclass
class W2VSynth(W2VLayout):
    batch_size: int = 16384        # centers per step per worker (multiple of 64)
    window: int = 5                # max window (contexts per center: up to 2*window)
    vocab: int = 1_000_000
    noise: float = 0.1
    negatives: int = 5             # K negatives per positive pair (sets the shared-negative weight)
    seed: int = 1234
    mode: str = "window"           # window | pairs (see W2VLayout)
    sentence_len: int = 24         # window mode: tokens per synthetic sentence
    neg_mode: str = "shared"       # shared | per_pair (see W2VLayout)

    def __post_init__(self):
        self._check_mode()

    graph_capturable = True  # generate() can take its step from device memory

    def generate(self, step: int, rank: int, world: int, keys: torch.Tensor, stream=None,
                 step_dev: int = 0, step_delta: int = 0, meta: Optional[torch.Tensor] = None):
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        B = self.batch_size
        base = (step * world + rank) * B
        if self.mode == "window":
            if meta is None or meta.numel() < self.run_len:
                raise ValueError("window mode: generate() needs a meta buffer of run_len int32")
            hip().w2v_stream_gen(self.seed, base, B, self.window, self.sentence_len,
                                 self.n_neg, self.vocab, self.noise, keys.data_ptr(),
                                 meta.data_ptr(), st, step_dev, world * B,
                                 (step_delta * world + rank) * B)
            return
        hip().w2v_gen(self.seed, base, B, self.contexts, self.window,
                      self.n_neg, self.vocab, self.noise, keys.data_ptr(), st,
                      step_dev, world * B, (step_delta * world + rank) * B)


def make_w2v_table_args(dim: int, optimizer: Optional[Optimizer] = None):
    opt = optimizer or Optimizer("adagrad", lr=0.05)
    init = InitConfig("uniform", scale=1.0 / dim, state_init=0.0, zero_key_bit=OUT_BIT)
    return opt, init


class Word2VecWorker(PipelinedWorker):
    """Trains skip-gram embeddings through a ``PSEngine`` (dim = embedding size)."""

    def __init__(self, engine, data: W2VSynth, rank: int = 0, world: int = 1,
                 active: bool = True):
        if engine.dim not in (32, 64, 128):
            raise ValueError("Word2VecWorker: dim must be 32, 64 or 128")
        super().__init__(engine, rank, world, active)
        self.data = data
        # the route stream is the light one for this model: pull the next
        # round's rows behind its dedup (bounded staleness 1)
        engine.enable_pull_ahead(pull_stream=True)
        self.keys = [torch.empty(data.n_keys, dtype=torch.int64, device=engine.device)
                     for _ in range(engine.depth)]
        self.window_mode = getattr(data, "mode", "pairs") == "window"
        self.meta = ([torch.empty(data.run_len, dtype=torch.int32, device=engine.device)
                      for _ in range(engine.depth)] if self.window_mode else None)
        # window layout: positive pairs of the last step (sharded counter),
        # beside the loss in one buffer: one zero-fill per step for both.
        # With the occurrence reduce the kernels add into _acc and
        # k_w2v_oreduce moves it to _out (loss_sum / pair_sum) and leaves it
        # zero: no fill launch per step
        self._acc = torch.zeros((2, self.loss_sum.numel()), dtype=torch.float32,
                                device=engine.device)
        self._out = self._acc
        self.loss_sum, self.pair_sum = self._acc[0], self._acc[1]
        # the tile's negative-sample GEMMs on the bf16 MFMA (center / negative
        # rows and score gradients rounded to bf16, fp32 accumulate; positive
        # pairs, parameters and optimizer state stay fp32): 77 KB of LDS
        # instead of 116, two workgroups per CU.  Measured 0.305 -> 0.278-0.282
        # ms/step (1M vocab, dim 128); SS_W2V_MFMA=f32 selects the fp32 tile
        self.mfma_bf16 = os.environ.get("SS_W2V_MFMA", "bf16") == "bf16"
        # window layout with the bucketed dedup: the tile stores one gradient
        # row per key position and the rows are summed per unique key
        # (w2v.hip k_w2v_osort on the route stream a round ahead,
        # k_w2v_oreduce on the main stream) instead of float row atomics from
        # the tile (0.101 -> 0.092 ms/step)
        self.occ_reduce = (self.window_mode and engine.gpu and
                           all(getattr(d, "mode", None) == "bucket" for d in engine.dedupers))
        self.per_pair = getattr(data, "neg_mode", "shared") == "per_pair"
        if self.per_pair and not self.occ_reduce:
            raise ValueError("per_pair negatives need the bucketed dedup (SS_DEDUP=bucket)")
        if self.occ_reduce:
            dev, n, D, W = engine.device, data.n_keys, engine.dim, data.window
            # per_pair: the negatives' gradient rows are (gn, center) pairs
            # (gnc below), so occurrence rows cover centers + run positions only
            rows = data.batch_size + data.run_len if self.per_pair else n
            self.ograd = torch.empty((rows, D), dtype=torch.float32, device=dev)
            self.gnc = (torch.empty((max(1, n - rows), 2), dtype=torch.float32, device=dev)
                        if self.per_pair else None)
            self.otail = torch.empty((max(1, (data.tiles - 1) * 2 * W), D), dtype=torch.float32,
                                     device=dev)
            # per_pair: g+ of every (center, offset) pair (k_w2v_pp -> k_w2v_ppctx)
            self.gpair = (torch.empty(data.batch_size * 2 * W, dtype=torch.float32, device=dev)
                          if self.per_pair else None)
            self.ord = [torch.empty(n, dtype=torch.int32, device=dev)
                        for _ in range(engine.depth)]
            # one GPU: the reduce runs the optimizer update of every key whose
            # gradient row is one item (k_w2v_oreduce with the table), and
            # the apply kernel then only the keys it summed over several
            # items (uhot, written by k_w2v_osort); SS_W2V_FUSE=0: off
            # (compact bf16 rows too: updated in fp32, stored with stochastic
            # rounding)
            # (the masked apply of the rest needs the wide-row vector apply:
            # with SS_PULL_VEC=0 the fuse is off, not an error mid-round)
            tab = engine.table
            self.fuse = (engine.fast1 and os.environ.get("SS_W2V_FUSE", "1") != "0" and
                         tab is not None and
                         bool(hip().apply_masked_ok(tab.dt, tab.opt.native())))
            self.uhot = ([torch.zeros(engine.max_keys * engine.world, dtype=torch.uint8,
                                      device=dev) for _ in range(engine.depth)]
                         if self.fuse else None)
            self.items = [torch.empty((n, 4), dtype=torch.int32, device=dev)
                          for _ in range(engine.depth)]
            self._post_route = self._osort
            self._out = torch.zeros_like(self._acc)
            self.loss_sum, self.pair_sum = self._out[0], self._out[1]

    def _zero_acc(self) -> None:
        if self._out is self._acc:
            self._acc.zero_()

    def _handoff(self) -> dict:
        """k_w2v_oreduce's accumulator hand-off (_acc -> _out, _acc zeroed)."""
        return {"acc": self._acc.data_ptr(), "acc_out": self._out.data_ptr(),
                "acc_n": self._acc.numel()}

    def _osort(self, dd, slot, st):
        o = dd.owner
        _, bstart, unum, ubase, P = o.bucket_view(dd.n)
        hip().w2v_osort(P, bstart, unum, ubase, o.pj.data_ptr(), o.luid.data_ptr(),
                        self.ord[slot].data_ptr(), self.items[slot].data_ptr(), st,
                        self.uhot[slot].data_ptr() if self.uhot is not None else 0)

    def _produce(self, step, slot, stream):
        kw = self._gen_kwargs(step)
        if self.window_mode:
            kw["meta"] = self.meta[slot]
        self.data.generate(step, self.rank, self.world, self.keys[slot], stream=stream, **kw)
        return self.keys[slot]

    def _fused(self, rnd):
        """Table arguments of a reduce that runs the optimizer update itself
        (one GPU), or {} (PSEngine.fuse_apply declined: the push applies)."""
        if self.uhot is None:
            return {}
        fa = self.engine.fuse_apply(rnd, snapshot=False)
        return {"t": fa["t"], "slots": fa["slots"], "op": fa["op"]} if fa else {}

    def _apply_hot(self, rnd, fa, slot, st):
        """The update of the keys the fused reduce summed over several items
        (their gradient rows are complete after it): the apply kernel over
        the round's unique keys, masked to those."""
        if not fa:
            return
        tab = self.engine.table
        sl = hip().SegList.from_device(rnd.dd.ucount.data_ptr())
        hip().apply(tab.dt, rnd.slots.data_ptr(), rnd.ugrad.data_ptr(), sl,
                    max(1, min(rnd.dd.n, rnd.dd.ucap)), fa["op"], tab.G, st, 0,
                    self.uhot[slot].data_ptr())

    def _compute(self, rnd, slot, st):
        d = self.data
        inv = rnd.inv
        B, C = d.batch_size, d.contexts
        ptr, es = inv.data_ptr(), inv.element_size()
        h = hip()
        if self.per_pair:
            h.w2v_pp(ptr, ptr + B * es, ptr + (B + d.run_len) * es, self.meta[slot].data_ptr(),
                     B, d.window, d.negatives, self.engine.dim, rnd.uvals.data_ptr(),
                     self.ograd.data_ptr(), self.gpair.data_ptr(), self._acc[0].data_ptr(),
                     self._acc[1].data_ptr(), st, self.gnc.data_ptr())
            fa = self._fused(rnd)
            h.w2v_oreduce(self.items[slot].data_ptr(), d.n_keys, self.ord[slot].data_ptr(),
                          self.ograd.data_ptr(), 0, B, d.window, self.engine.dim,
                          rnd.ugrad.data_ptr(), st, gnc=self.gnc.data_ptr(),
                          negbase=B + d.run_len, uvals=rnd.uvals.data_ptr(), **self._handoff(),
                          **fa)
            self._apply_hot(rnd, fa, slot, st)
            return
        if self.window_mode:
            occ = self.occ_reduce
            h.w2v_win(ptr, ptr + B * es, ptr + (B + d.run_len) * es, self.meta[slot].data_ptr(),
                      B, d.window, self.engine.dim, d.neg_per_pair, rnd.uvals.data_ptr(),
                      rnd.ugrad.data_ptr(), self._acc[0].data_ptr(), self._acc[1].data_ptr(),
                      st, self.ograd.data_ptr() if occ else 0, self.otail.data_ptr() if occ else 0)
            if occ:
                fa = self._fused(rnd)
                h.w2v_oreduce(self.items[slot].data_ptr(), d.n_keys, self.ord[slot].data_ptr(),
                              self.ograd.data_ptr(), self.otail.data_ptr(), B, d.window,
                              self.engine.dim, rnd.ugrad.data_ptr(), st, **self._handoff(), **fa)
                self._apply_hot(rnd, fa, slot, st)
            return
        h.w2v_sgns(ptr, ptr + B * es, ptr + B * (1 + C) * es, B, C, self.engine.dim,
                   d.neg_scale, rnd.uvals.data_ptr(), rnd.ugrad.data_ptr(),
                   self.loss_sum.data_ptr(), st, int(self.mfma_bf16))

    def samples_per_step(self) -> int:
        """Window layout: centers (words) per step, word2vec's "words/s"
        numerator; pairs layout: (center, context) pairs per step."""
        if not self.active:
            return 0
        return self.data.batch_size if self.window_mode else \
            self.data.batch_size * self.data.contexts

    def step_pairs(self) -> float:
        """Positive pairs trained in the last step (window layout: counted by
        the tile kernel; pairs layout: B x 2W).  Syncs."""
        if not self.active:
            return 0.0
        if self.window_mode:
            return float(self.pair_sum.sum().item())
        return float(self.data.batch_size * self.data.contexts)

    def mean_loss(self) -> float:
        """Mean SGNS loss per positive pair (incl. its negatives) of the last step."""
        if not self.window_mode:
            return super().mean_loss()
        n = self.step_pairs()
        return float(self.loss_sum.sum().item()) / n if n else 0.0


def window_pairs_reference(meta: np.ndarray, B: int, W: int) -> np.ndarray:
    """Valid-pair mask [B, B + 2W] of a window-layout run (ss/w2v_window.h):
    center t (run position t + W) pairs with run position q."""
    m = meta.astype(np.int64)
    c = m[W:W + B][:, None]
    q = m[None, :]
    d = np.arange(B + 2 * W)[None, :] - (np.arange(B)[:, None] + W)
    return ((c >= 0) & (q >= 0) & ((c >> 4) == (q >> 4)) & (d != 0) & (np.abs(d) <= (c & 15)))


def sgns_window_reference(V: np.ndarray, U: np.ndarray, N: np.ndarray, mask: np.ndarray,
                          neg_per_pair: float):
    """fp64 reference of one window tile.  V [T,D] centers, U [Q,D] window
    rows, N [S,D] shared negatives, mask [T,Q] valid pairs.  Returns (loss,
    pairs, gV, gU, gN); a center's negatives weigh n_t * neg_per_pair."""
    V, U, N = (a.astype(np.float64) for a in (V, U, N))
    sig = lambda z: 1.0 / (1.0 + np.exp(-z))  # noqa: E731
    sp = lambda z: np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z)))  # noqa: E731
    n = mask.sum(1).astype(np.float64)
    Sp = V @ U.T
    Gp = np.where(mask, sig(Sp) - 1.0, 0.0)
    Sn = V @ N.T
    cw = (n * neg_per_pair)[:, None]
    Gn = cw * sig(Sn)
    loss = np.where(mask, sp(-Sp), 0.0).sum() + (cw * sp(Sn)).sum()
    return loss, n.sum(), Gp @ U + Gn @ N, Gp.T @ V, Gn.T @ V


def sgns_pp_reference(V: np.ndarray, U: np.ndarray, N: np.ndarray, mask: np.ndarray):
    """fp64 reference of per-pair negatives.  V [B,D] centers, U [B,2W,D]
    context rows by offset slot, N [B,2W,K,D] each pair's negatives, mask
    [B,2W] valid pairs.  Returns (loss, gV, gU, gN) (zero where not valid)."""
    V, U, N = (a.astype(np.float64) for a in (V, U, N))
    sig = lambda z: 1.0 / (1.0 + np.exp(-z))  # noqa: E731
    sp = lambda z: np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z)))  # noqa: E731
    m = mask.astype(np.float64)
    s_p = np.einsum("bd,bod->bo", V, U)
    s_n = np.einsum("bd,bokd->bok", V, N)
    gp = (sig(s_p) - 1.0) * m
    gn = sig(s_n) * m[:, :, None]
    loss = (sp(-s_p) * m).sum() + (sp(s_n) * m[:, :, None]).sum()
    gV = np.einsum("bo,bod->bd", gp, U) + np.einsum("bok,bokd->bd", gn, N)
    gU = gp[:, :, None] * V[:, None, :]
    gN = gn[:, :, :, None] * V[:, None, None, :]
    return loss, gV, gU, gN


def sgns_reference(V: np.ndarray, X: np.ndarray, N: np.ndarray, neg_scale: float):
    """fp64 reference of one tile.  V [T,D] centers, X [T,C,D] contexts,
    N [S,D] shared negatives.  Returns (loss, gV [T,D], gX [T,C,D], gN [S,D])."""
    V, X, N = (a.astype(np.float64) for a in (V, X, N))
    sig = lambda z: 1.0 / (1.0 + np.exp(-z))  # noqa: E731
    sp = lambda z: np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z)))  # noqa: E731
    S = V @ N.T
    G = neg_scale * sig(S)
    pos = np.einsum("td,tcd->tc", V, X)
    gp = sig(pos) - 1.0
    loss = neg_scale * sp(S).sum() + sp(-pos).sum()
    gV = G @ N + np.einsum("tc,tcd->td", gp, X)
    gX = gp[:, :, None] * V[:, None, :]
    gN = G.T @ V
    return loss, gV, gX, gN
