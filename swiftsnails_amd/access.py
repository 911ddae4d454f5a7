"""The reference's worker-side access API, on this framework's engines.

A SwiftSnails application trains with three objects
(/root/reference/src/core/parameter/global_param_cache.h:28-118,
global_pull_access.h:40-120, global_push_access.h:36-149):

    GlobalParamCache<Key, Val, Grad> cache;            // params + grads by key
    global_pull_access().pull_with_barrier(keys, cache);  // fill params, reset grads
    ... compute, cache.grads[key] += ... ;
    global_push_access().push_with_barrier(keys, cache);  // send grads, reset them

The same three calls work here against either data plane:

* a GPU round engine (``PSEngine``: HBM shards, RCCL rounds) — the cache holds
  device tensors ``params[n, dim]`` / ``grads[n, dim]`` aligned with its sorted
  unique ``keys``, so the compute between pull and push is tensor code;
* a host client (``BaseAlgorithm`` of the TCP cluster, ``WorkerClient``,
  ``local_train``) — anything with ``pull(keys) -> rows`` and
  ``push(keys, grads)``; the cache then holds host tensors.

The reference's per-key access (``cache.params[key]``) and its
``GradPramProcMethod`` hooks (``merge_grad``, ``update_param``,
``rewrite_param``; global_param_cache.h:6-19) are available as vectorised
methods.  Unlike the reference, an empty key set returns at once (its
``pull_with_barrier`` blocks forever on one, SURVEY §5 known defects).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch


def _as_keys(keys, device) -> torch.Tensor:
    if isinstance(keys, torch.Tensor):
        k = keys.reshape(-1).to(torch.int64)
    else:
        a = np.asarray(list(keys) if isinstance(keys, (set, frozenset)) else keys)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        k = torch.from_numpy(np.ascontiguousarray(a.astype(np.int64, copy=False)).reshape(-1))
    return k.to(device)


class GlobalParamCache:
    """One worker's parameters and gradients for its current key set."""

    def __init__(self, dim: int, device=None):
        self.dim = int(dim)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.keys = torch.empty(0, dtype=torch.int64, device=self.device)
        self.params = torch.empty((0, self.dim), dtype=torch.float32, device=self.device)
        self.grads = torch.empty((0, self.dim), dtype=torch.float32, device=self.device)

    # -- key set (global_param_cache.h:41-56 init_keys)
    def init_keys(self, keys) -> None:
        """Make the cache hold exactly the distinct ``keys`` (sorted), with
        zero params and grads."""
        k = torch.unique(_as_keys(keys, self.device))
        self.keys = k
        self.params = torch.zeros((k.numel(), self.dim), dtype=torch.float32, device=self.device)
        self.grads = torch.zeros_like(self.params)

    def __len__(self) -> int:
        return int(self.keys.numel())

    def index(self, keys) -> torch.Tensor:
        """Cache rows of ``keys`` (each must be in the cache)."""
        k = _as_keys(keys, self.device)
        if k.numel() == 0:
            return torch.empty(0, dtype=torch.int64, device=self.device)
        if len(self) == 0:
            raise KeyError("key not in the cache (pull it first)")
        pos = torch.searchsorted(self.keys, k).clamp(max=len(self) - 1)
        if not bool((self.keys[pos] == k).all()):
            raise KeyError("key not in the cache (pull it first)")
        return pos

    # -- per-key views (the reference's params[key] / grads[key])
    def param(self, key) -> torch.Tensor:
        return self.params[self.index([key])[0]]

    def grad(self, key) -> torch.Tensor:
        return self.grads[self.index([key])[0]]

    # -- GradPramProcMethod hooks (global_param_cache.h:6-19), vectorised
    def merge_grad(self, keys, grads) -> None:
        """grads[key] += g for every (key, g); duplicate keys accumulate."""
        g = torch.as_tensor(grads, dtype=torch.float32, device=self.device).reshape(-1, self.dim)
        self.grads.index_add_(0, self.index(keys), g)

    def update_param(self, fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]) -> None:
        """params = fn(params, grads) (a worker-local update, e.g. local_train)."""
        self.params = fn(self.params, self.grads).reshape(-1, self.dim).to(torch.float32)

    def rewrite_param(self, keys, values) -> None:
        v = torch.as_tensor(values, dtype=torch.float32, device=self.device).reshape(-1, self.dim)
        self.params[self.index(keys)] = v

    def reset_grads(self) -> None:
        self.grads.zero_()


class _Access:
    """Binds the access calls to an engine (GPU) or a host client."""

    def __init__(self, target):
        self.target = target

    def _is_engine(self) -> bool:
        return hasattr(self.target, "pull_dense") and hasattr(self.target, "push_keys")


class GlobalPullAccess(_Access):
    def pull_with_barrier(self, keys, cache: GlobalParamCache) -> GlobalParamCache:
        """Fill ``cache.params`` for the distinct ``keys`` (missing keys are
        created with the server's init rule) and reset ``cache.grads``
        (global_pull_access.h:92-113).  Blocks until the rows are there."""
        cache.init_keys(keys)
        if len(cache) == 0:
            return cache
        t = self.target
        if self._is_engine():
            rows = t.pull_dense(cache.keys.to(t.device))
            if rows.is_cuda:
                torch.cuda.current_stream().synchronize()
            cache.params = rows.to(cache.device).reshape(-1, cache.dim).clone()
        else:
            rows = t.pull(cache.keys.cpu().numpy().view(np.uint64))
            cache.params = torch.as_tensor(np.asarray(rows, dtype=np.float32)).reshape(
                -1, cache.dim).to(cache.device)
        cache.grads = torch.zeros_like(cache.params)
        return cache


class GlobalPushAccess(_Access):
    def push_with_barrier(self, keys, cache: GlobalParamCache) -> None:
        """Send ``cache.grads`` of ``keys`` (all cached keys when None) to
        their servers, which apply the update rule, then reset those grads
        (global_push_access.h:80-99).  Blocks until applied."""
        if len(cache) == 0:
            return
        # a key listed twice is still pushed (and its gradient counted) once
        idx = None if keys is None else torch.unique(cache.index(keys))
        k = cache.keys if idx is None else cache.keys[idx]
        g = cache.grads if idx is None else cache.grads[idx]
        if k.numel() == 0:
            return
        t = self.target
        if self._is_engine():
            t.push_keys(k.to(t.device), g.to(t.device))
            if g.is_cuda or getattr(t, "gpu", False):
                torch.cuda.current_stream().synchronize()
        else:
            t.push(k.cpu().numpy().view(np.uint64), g.cpu().numpy().astype(np.float32))
        if idx is None:
            cache.grads.zero_()
        else:
            cache.grads[idx] = 0.0


_default_target: Optional[object] = None


def set_global_target(target) -> None:
    """Register the engine / client ``global_pull_access()`` and
    ``global_push_access()`` use when called without one (the reference's
    accessors are process-wide singletons, global_pull_access.h:125-131)."""
    global _default_target
    _default_target = target


def _target(target):
    t = target if target is not None else _default_target
    if t is None:
        raise RuntimeError("no engine/client: pass one or call set_global_target()")
    return t


def global_pull_access(target=None) -> GlobalPullAccess:
    return GlobalPullAccess(_target(target))


def global_push_access(target=None) -> GlobalPushAccess:
    return GlobalPushAccess(_target(target))


__all__ = ["GlobalParamCache", "GlobalPullAccess", "GlobalPushAccess", "global_pull_access",
           "global_push_access", "set_global_target"]
