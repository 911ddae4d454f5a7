"""Dense logistic regression over the host PS (BASELINE config 1: 1 worker +
1 server on CPU over TCP loopback — the plumbing baseline).

The weight vector lives on the servers as D scalar keys 0..D-1 (dim 1), the
way a reference app would keep a model in the SparseTable; each step the
worker pulls all D weights (``pull_with_barrier``), computes the minibatch
gradient on the CPU (the reference's Vec math, utils/vec1.h: dot/scale/add)
and pushes it back (``push_with_barrier``).
"""
from __future__ import annotations

import numpy as np

from ..framework.cluster import BaseAlgorithm


class DenseLRData:
    """Synthetic dense binary-classification data from a hidden weight vector."""

    def __init__(self, dim: int = 64, seed: int = 7):
        self.dim = dim
        rng = np.random.default_rng(seed)
        self.w_true = rng.standard_normal(dim).astype(np.float32)
        self.seed = seed

    def batch(self, step: int, worker: int, batch: int):
        rng = np.random.default_rng((self.seed, step, worker))
        x = rng.standard_normal((batch, self.dim)).astype(np.float32)
        p = 1.0 / (1.0 + np.exp(-(x @ self.w_true)))
        y = (rng.random(batch) < p).astype(np.float32)
        return x, y


class DenseLR(BaseAlgorithm):
    def __init__(self, data: DenseLRData, steps: int = 50, batch: int = 256, worker_id: int = 0):
        super().__init__()
        self.data, self.steps, self.batch, self.worker_id = data, steps, batch, worker_id
        self.keys = np.arange(data.dim, dtype=np.uint64)
        self.losses: list[float] = []

    def parse_record(self, line: str):
        # "label f0 f1 ... f{D-1}" (text input for CPU-cluster runs)
        v = np.array(line.split(), dtype=np.float32)
        return v[1:], v[0]

    def train(self):
        for step in range(self.steps):
            x, y = self.data.batch(step, self.worker_id, self.batch)
            w = self.pull(self.keys)[:, 0]
            z = x @ w
            p = 1.0 / (1.0 + np.exp(-z))
            self.losses.append(float(np.mean(np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z))) - y * z)))
            g = (x.T @ (p - y) / self.batch).astype(np.float32)
            self.push(self.keys, g[:, None])
