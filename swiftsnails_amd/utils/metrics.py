"""Evaluation metrics for the CTR / LR models (host, numpy).

The reference has no evaluation code at all (its apps are absent from the
snapshot); these are the standard binary-classification metrics a
CTR trainer reports, used by the convergence tests ("loss
decreases; AUC above a threshold") and by ``SparseLRWorker.evaluate``.
"""
from __future__ import annotations

import numpy as np


def auc(scores, labels) -> float:
    """ROC AUC by the rank-sum (Mann-Whitney U) statistic; ties get the
    average rank, so a constant predictor scores exactly 0.5."""
    s = np.asarray(scores, dtype=np.float64).reshape(-1)
    y = np.asarray(labels).reshape(-1) > 0.5
    npos = int(y.sum())
    nneg = y.size - npos
    if npos == 0 or nneg == 0:
        return float("nan")
    order = np.argsort(s, kind="mergesort")
    ss = s[order]
    ranks = np.empty(s.size, dtype=np.float64)
    # average ranks over runs of equal scores
    edges = np.flatnonzero(np.diff(ss)) + 1
    starts = np.concatenate(([0], edges))
    ends = np.concatenate((edges, [s.size]))
    avg = (starts + ends + 1) / 2.0  # 1-based average rank of each run
    ranks[order] = np.repeat(avg, ends - starts)
    u = ranks[y].sum() - npos * (npos + 1) / 2.0
    return float(u / (npos * nneg))


def logloss(logits, labels) -> float:
    """Mean binary cross-entropy of logits z (numerically stable form)."""
    z = np.asarray(logits, dtype=np.float64).reshape(-1)
    y = np.asarray(labels, dtype=np.float64).reshape(-1)
    return float(np.mean(np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z))) - y * z))
