"""Host (numpy) twin of the on-device synthetic CTR generator (models.hip k_gen_ctr).

Same counter-based RNG and distribution: field f owns keys [f*V, (f+1)*V);
ids are log-uniform (Zipf-like head) with a ``tail_frac`` uniform tail; labels
are Bernoulli(sigmoid(sum of per-key ground-truth weights + bias)).  Used by
CPU workers (reference-semantics CPU baseline, CPU cluster examples) and to
cross-check the device generator.
"""
from __future__ import annotations

import numpy as np

from ..utils.hashing import splitmix64

_U = np.uint64


def _u01(r: np.ndarray) -> np.ndarray:
    return (r >> _U(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def _fastrange(h: np.ndarray, n: int) -> np.ndarray:
    # exact (h * n) >> 64 for n < 2**32 with 64-bit limbs:
    # floor(h*n / 2^64) = (hi*n + ((lo*n) >> 32)) >> 32
    assert n < (1 << 32)
    hi = h >> _U(32)
    lo = h & _U(0xFFFFFFFF)
    nn = _U(n)
    with np.errstate(over="ignore"):
        return (hi * nn + ((lo * nn) >> _U(32))) >> _U(32)


def truth_weight(keys: np.ndarray, scale: float) -> np.ndarray:
    return (_u01(splitmix64(keys.astype(np.uint64) ^ _U(0x5DEECE66D))) - np.float32(0.5)) * \
        np.float32(scale)


def gen_ctr_np(seed: int, sample_base: int, B: int, F: int, V: int, tail_frac: float = 0.1,
               truth_scale: float = 1.0, truth_bias: float = -1.0):
    """Returns (keys int64 [B*F], labels float32 [B])."""
    with np.errstate(over="ignore"):
        gs = (np.arange(B, dtype=np.uint64) + _U(sample_base))[:, None]
        f = np.arange(F, dtype=np.uint64)[None, :]
        r = splitmix64(_U(seed) ^ (gs * _U(0xA24BAED4963EE407)) ^ (f << _U(40)))
        r2 = splitmix64(r)
        tail = _u01(r2) < np.float32(tail_frac)
        u = (r >> _U(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        logV = np.log(float(V) + 1.0)
        v = (np.exp(u * logV)).astype(np.int64) - 1
        head = np.clip(v, 0, V - 1).astype(np.uint64)
        tid = _fastrange(splitmix64(r2 ^ _U(0x632BE59BD9B4E019)), V)
        ids = np.where(tail, tid, head)
        keys = f * _U(V) + ids
        z = truth_weight(keys, truth_scale).sum(1, dtype=np.float32) + np.float32(truth_bias)
        p = 1.0 / (1.0 + np.exp(-z.astype(np.float64)))
        lr = _u01(splitmix64(_U(seed) ^ _U(0xBEEF) ^ (gs[:, 0] * _U(0x9E3779B97F4A7C15))))
        labels = (lr < p).astype(np.float32)
    return keys.reshape(-1).view(np.int64), labels


def lr_grad_np(w_occ: np.ndarray, labels: np.ndarray, F: int):
    """Per-occurrence LR gradient for binary features: returns (g_occ, loss_sum)."""
    z = w_occ.reshape(-1, F).sum(1, dtype=np.float64)
    p = 1.0 / (1.0 + np.exp(-z))
    y = labels.astype(np.float64)
    loss = float(np.sum(np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z))) - y * z))
    g = np.repeat((p - y).astype(np.float32), F)
    return g, loss
