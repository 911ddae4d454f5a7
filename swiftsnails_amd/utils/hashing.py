"""Vectorised host-side key hashing (bit-identical to ``csrc/include/ss/hash.h``).

``fmix64`` reproduces the reference's ``get_hash_code`` (MurmurHash3
finalizer, /root/reference/src/utils/HashFunction.h:16-24).  numpy uint64
arithmetic wraps modulo 2**64 exactly like the C++/device code.
"""
from __future__ import annotations

import numpy as np
import torch

M64 = (1 << 64) - 1
EMPTY_KEY = M64  # u64 sentinel; as int64 this is -1
_C1 = np.uint64(0xFF51AFD7ED558CCD)
_C2 = np.uint64(0xC4CEB9FE1A85EC53)
_S33 = np.uint64(33)


def fmix64_int(x: int) -> int:
    """Scalar reference implementation on Python ints."""
    x &= M64
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


def fmix64(x) -> np.ndarray:
    """Vectorised fmix64 over uint64 (accepts int64 arrays / torch tensors)."""
    a = as_u64(x).copy()
    with np.errstate(over="ignore"):
        a ^= a >> _S33
        a *= _C1
        a ^= a >> _S33
        a *= _C2
        a ^= a >> _S33
    return a


def splitmix64(x) -> np.ndarray:
    a = as_u64(x).copy()
    with np.errstate(over="ignore"):
        a += np.uint64(0x9E3779B97F4A7C15)
        a = (a ^ (a >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        a = (a ^ (a >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        a = a ^ (a >> np.uint64(31))
    return a


def as_u64(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    a = np.asarray(x)
    if a.dtype == np.uint64:
        return a
    if a.dtype == np.int64:
        return a.view(np.uint64)
    return a.astype(np.uint64)


def u64_to_i64(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)


def keys_to_tensor(keys, device=None) -> torch.Tensor:
    """Any integer key container -> int64 tensor carrying the u64 bit pattern."""
    if isinstance(keys, torch.Tensor):
        t = keys.to(torch.int64) if keys.dtype != torch.int64 else keys
    else:
        t = torch.from_numpy(u64_to_i64(as_u64(np.asarray(keys, dtype=np.uint64)
                                               if not isinstance(keys, np.ndarray) else keys)))
    return t.to(device) if device is not None else t
