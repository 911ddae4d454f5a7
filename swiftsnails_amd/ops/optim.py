"""Server-side update rules (the reference's Pull/PushAccessMethod menu).

The reference lets the application subclass ``PullAccessMethod``
(``init_param``/``get_pull_value``) and ``PushAccessMethod``
(``merge_push_value``/``apply_push_value``)
(/root/reference/src/core/parameter/sparse_access_method.h:10-48).  On the GPU
these are compiled device functors (``ss_device.h``: ``init_value`` and
``opt_apply``) selected by an enum — a fixed menu of rules fused into the
probe/apply kernels:

* init  : zero | uniform ``(u-0.5)*scale`` (word2vec convention, vec1.h:223-226) | normal
* push  : SGD | AdaGrad | FTRL-Proximal | lazy Adam (+ L1/L2, gradient scale, clip)
* merge : summation of duplicate-key gradients (done worker-side before push)

``apply_reference`` is the float32 numpy implementation of the same update,
used by the kernel numerics tests and by the CPU host table.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

OPT_KINDS = {"sgd": 0, "adagrad": 1, "ftrl": 2, "adam": 3}
# compiled initialisers (ss/optim.h init_value); "marker" is internal: the
# placeholder a tensor-code initialiser replaces (HbmTable.set_init_method)
INIT_KINDS = {"zero": 0, "uniform": 1, "normal": 2, "const": 3, "marker": 4}
INIT_MARKER_BITS = 0x7FBADBAD


def state_width(kind: str, dim: int) -> int:
    return {"sgd": 0, "adagrad": dim, "ftrl": 2 * dim, "adam": 2 * dim}[kind]


@dataclass
class InitConfig:
    kind: str = "zero"
    scale: float = 0.0
    state_init: float = 0.0  # initial optimizer-state value (e.g. AdaGrad accumulator)
    seed: int = 2015
    zero_key_bit: int = -1  # keys with this bit set start at zero (namespaced tables)

    def native(self):
        from .._native import hip

        return hip().InitParams(INIT_KINDS[self.kind], float(self.scale), float(self.state_init),
                                int(self.seed) & ((1 << 64) - 1), int(self.zero_key_bit))


@dataclass
class Optimizer:
    kind: str = "adagrad"
    lr: float = 0.05
    l1: float = 0.0
    l2: float = 0.0
    eps: float = 1e-8
    beta1: float = 0.9
    beta2: float = 0.999
    ftrl_alpha: float = 0.05
    ftrl_beta: float = 1.0
    grad_scale: float = 1.0
    clip: float = 0.0
    step: int = field(default=0, repr=False)  # Adam bias-correction counter (rounds)

    def __post_init__(self):
        if self.kind not in OPT_KINDS:
            raise ValueError(f"unknown optimizer {self.kind!r}; have {sorted(OPT_KINDS)}")

    def state_width(self, dim: int) -> int:
        return state_width(self.kind, dim)

    def bias_corrections(self):
        if self.kind != "adam":
            return 1.0, 1.0
        t = max(1, self.step)
        return 1.0 / (1.0 - self.beta1**t), 1.0 / (1.0 - self.beta2**t)

    def native(self):
        from .._native import hip

        bc1, bc2 = self.bias_corrections()
        return hip().OptParams(OPT_KINDS[self.kind], self.lr, self.l1, self.l2, self.eps,
                               self.beta1, self.beta2, bc1, bc2, self.ftrl_alpha, self.ftrl_beta,
                               self.grad_scale, self.clip)

    @classmethod
    def from_config(cls, cfg, prefix: str = "") -> "Optimizer":
        """Build from a ConfigParser-like mapping (keys: optimizer, learning_rate, ...)."""
        g = (lambda k, d: cfg.get(prefix + k, d)) if hasattr(cfg, "get") else (lambda k, d: d)
        return cls(kind=str(g("optimizer", "adagrad")), lr=float(g("learning_rate", 0.05)),
                   l1=float(g("l1", 0.0)), l2=float(g("l2", 0.0)))


def init_reference(init: InitConfig, keys: np.ndarray, dim: int, width: int) -> np.ndarray:
    """Host reference of ss::init_value (bit-exact for zero/uniform)."""
    from ..utils.hashing import as_u64, splitmix64

    keys = as_u64(keys)
    out = np.zeros((len(keys), width), dtype=np.float32)
    out[:, dim:] = np.float32(init.state_init)
    if init.kind == "zero" or dim == 0:
        return out
    zmask = None
    if init.zero_key_bit >= 0:
        zmask = ((keys >> np.uint64(init.zero_key_bit)) & np.uint64(1)).astype(bool)
    seed = np.uint64(int(init.seed) & ((1 << 64) - 1))
    with np.errstate(over="ignore"):
        kk = keys * np.uint64(0x9E3779B97F4A7C15)
        for j in range(dim):
            jj = np.uint64(j)
            r = splitmix64(seed ^ kk ^ (jj << np.uint64(48)) ^ jj)
            u = (r >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            if init.kind == "uniform":
                out[:, j] = (u - np.float32(0.5)) * np.float32(init.scale)
            else:
                u1 = np.maximum(u, np.float32(1e-7))
                r2 = splitmix64(r)
                u2 = (r2 >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
                out[:, j] = (np.sqrt(-2.0 * np.log(u1)) * np.cos(6.2831853 * u2) *
                             init.scale).astype(np.float32)
    if zmask is not None:
        out[zmask, :dim] = 0.0
    return out


def apply_reference(opt: Optimizer, rows: np.ndarray, grads: np.ndarray, dim: int) -> np.ndarray:
    """fp32 reference of ss::opt_apply over full rows [n, width] (returns new rows)."""
    rows = rows.astype(np.float32).copy()
    g = grads.astype(np.float32) * np.float32(opt.grad_scale)
    if opt.clip > 0:
        g = np.clip(g, -opt.clip, opt.clip)
    w = rows[:, :dim]
    f32 = np.float32
    if opt.kind == "sgd":
        g = g + f32(opt.l2) * w
        rows[:, :dim] = w - f32(opt.lr) * g
    elif opt.kind == "adagrad":
        g = g + f32(opt.l2) * w
        h = rows[:, dim:2 * dim] + g * g
        rows[:, dim:2 * dim] = h
        rows[:, :dim] = w - f32(opt.lr) * g / np.sqrt(h + f32(opt.eps))
    elif opt.kind == "ftrl":
        z = rows[:, dim:2 * dim]
        n = rows[:, 2 * dim:3 * dim]
        n2 = n + g * g
        sigma = (np.sqrt(n2) - np.sqrt(n)) / f32(opt.ftrl_alpha)
        z = z + g - sigma * w
        rows[:, dim:2 * dim] = z
        rows[:, 2 * dim:3 * dim] = n2
        neww = -(z - np.sign(z) * f32(opt.l1)) / ((f32(opt.ftrl_beta) + np.sqrt(n2)) /
                                                   f32(opt.ftrl_alpha) + f32(opt.l2))
        rows[:, :dim] = np.where(np.abs(z) <= opt.l1, f32(0), neww)
    elif opt.kind == "adam":
        bc1, bc2 = opt.bias_corrections()
        g = g + f32(opt.l2) * w
        m = f32(opt.beta1) * rows[:, dim:2 * dim] + f32(1 - opt.beta1) * g
        v = f32(opt.beta2) * rows[:, 2 * dim:3 * dim] + f32(1 - opt.beta2) * g * g
        rows[:, dim:2 * dim] = m
        rows[:, 2 * dim:3 * dim] = v
        rows[:, :dim] = w - f32(opt.lr) * (m * f32(bc1)) / (np.sqrt(v * f32(bc2)) + f32(opt.eps))
    return rows


__all__ = ["Optimizer", "InitConfig", "apply_reference", "init_reference", "state_width",
           "OPT_KINDS", "INIT_KINDS", "math"]
