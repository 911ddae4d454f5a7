"""CPU sparse parameter table (C++ ``ss::HostTable`` behind a Python facade).

Same semantics as the HBM table (lookup-or-init pull, optimizer push, text
checkpoint) using the same ``ss/optim.h`` init/update code; used by CPU
clusters (reference-style master/server/worker over TCP), by the CPU
multi-process tests of the collective engine, and as the reference-semantics
CPU baseline (BASELINE config 1).  Reference: SparseTable
(/root/reference/src/core/parameter/sparsetable.h:69-121).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .._native import host
from .optim import INIT_KINDS, OPT_KINDS, InitConfig, Optimizer


def _host_init(c: InitConfig):
    return host().InitParams(INIT_KINDS[c.kind], float(c.scale), float(c.state_init),
                             int(c.seed) & ((1 << 64) - 1), int(c.zero_key_bit))


def _host_opt(o: Optimizer):
    bc1, bc2 = o.bias_corrections()
    return host().OptParams(OPT_KINDS[o.kind], o.lr, o.l1, o.l2, o.eps, o.beta1, o.beta2, bc1, bc2,
                            o.ftrl_alpha, o.ftrl_beta, o.grad_scale, o.clip)


def _u64(keys) -> np.ndarray:
    if isinstance(keys, torch.Tensor):
        keys = keys.detach().cpu().numpy()
    a = np.ascontiguousarray(keys)
    return a.view(np.uint64) if a.dtype == np.int64 else a.astype(np.uint64)


def set_table_push_method(native_table, fn) -> None:
    """Install ``fn(rows, grads) -> rows`` (torch tensors) as the batch update
    rule of a native ``_ss_host.HostTable`` (also the one inside a host-mode
    server); ``None`` restores the optimizer menu."""
    if fn is None:
        native_table.set_batch_apply(None)
        return

    def batch(keys, rows, grads):
        out = fn(torch.from_numpy(rows), torch.from_numpy(grads))
        if isinstance(out, torch.Tensor):
            out = out.detach().cpu().numpy()
        return np.ascontiguousarray(out, dtype=np.float32)

    native_table.set_batch_apply(batch)


class HostTable:
    device = torch.device("cpu")
    push_fn = None
    init_fn = None
    pull_fn = None

    def __init__(self, dim: int, shard_num: int = 8, optimizer: Optional[Optimizer] = None,
                 init: Optional[InitConfig] = None, nthreads: int = 0):
        self.dim = int(dim)
        self.opt = optimizer or Optimizer()
        self.init_cfg = init or InitConfig()
        self._t = host().HostTable(self.dim, shard_num, _host_init(self.init_cfg),
                                   _host_opt(self.opt), nthreads)
        self.width = self._t.width

    def set_push_method(self, fn) -> None:
        """User-defined update rule, as ``HbmTable.set_push_method``:
        ``fn(rows [n, width], grads [n, dim]) -> new rows`` (torch CPU
        tensors) applied to every push (the reference's
        ``PushAccessMethod::apply_push_value``, batched per push call)."""
        self.push_fn = fn
        set_table_push_method(self._t, fn)

    def set_init_method(self, fn) -> None:
        """User initialiser, as ``HbmTable.set_init_method``: ``fn(keys) ->
        rows [n, width]`` for keys a pull (or push) creates."""
        self.init_fn = fn

    def set_pull_method(self, fn) -> None:
        """User pull transform, as ``HbmTable.set_pull_method``:
        ``fn(keys, rows [n, width]) -> vals [n, dim]``."""
        self.pull_fn = fn

    @property
    def custom_pull(self) -> bool:
        return self.init_fn is not None or self.pull_fn is not None

    def _create_missing(self, k: np.ndarray) -> None:
        """Run the user initialiser on the keys of ``k`` not yet stored."""
        if self.init_fn is None or len(k) == 0:
            return
        _, found = self._t.get_rows(k)
        miss = np.unique(k[found == 0])
        if len(miss):
            rows = self.init_fn(torch.from_numpy(miss.view(np.int64)))
            rows = np.ascontiguousarray(torch.as_tensor(rows, dtype=torch.float32).numpy())
            if rows.shape != (len(miss), self.width):
                raise ValueError(f"init method returned {rows.shape}, expected "
                                 f"{(len(miss), self.width)}")
            self._t.assign(miss, rows.reshape(-1))

    # same surface as HbmTable where it makes sense
    def pull_keys(self, keys) -> torch.Tensor:
        k = _u64(keys)
        self._create_missing(k)
        vals = torch.from_numpy(self._t.pull(k))
        if self.pull_fn is not None:
            rows, _ = self._t.get_rows(k)
            vals = torch.as_tensor(self.pull_fn(torch.from_numpy(k.view(np.int64)),
                                                torch.from_numpy(rows)), dtype=torch.float32)
            if vals.shape != (len(k), self.dim):
                raise ValueError(f"pull method returned {tuple(vals.shape)}, expected "
                                 f"{(len(k), self.dim)}")
        return vals

    def push_keys(self, keys, grads):
        g = grads.detach().cpu().numpy() if isinstance(grads, torch.Tensor) else np.asarray(grads)
        self._t.set_opt(_host_opt(self.opt))
        k = _u64(keys)
        self._create_missing(k)
        self._t.push(k, np.ascontiguousarray(g, dtype=np.float32).reshape(-1))

    def next_round(self):
        self.opt.step += 1

    def assign(self, keys, rows):
        r = rows.detach().cpu().numpy() if isinstance(rows, torch.Tensor) else np.asarray(rows)
        self._t.assign(_u64(keys), np.ascontiguousarray(r, dtype=np.float32).reshape(-1))

    def export(self, chunk_slots: int = 0, to_host: bool = True):
        k, r = self._t.export()
        if len(k):
            yield torch.from_numpy(k.view(np.int64)), torch.from_numpy(r)

    def size(self) -> int:
        return self._t.size()

    def check(self):
        pass

    def write_text(self, path: str, precision: int = 9, with_state: bool = False) -> int:
        return self._t.write_text(path, precision, with_state)

    def load_text(self, path: str) -> int:
        return self._t.load_text(path)

    def to_dict(self, with_state: bool = False):
        out = {}
        for k, r in self.export():
            kn, rn = k.numpy().view(np.uint64), r.numpy()
            for i in range(len(kn)):
                out[int(kn[i])] = rn[i] if with_state else rn[i, :self.dim]
        return out

    def __len__(self):
        return self.size()

    def __repr__(self):
        return f"HostTable(dim={self.dim}, width={self.width}, opt={self.opt.kind})"
