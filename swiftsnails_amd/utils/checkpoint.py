"""Checkpoints: the reference's text format plus a binary format and resume.

Reference behaviour (SURVEY §5 "Checkpoint / resume"):
* every ``param_backup_period`` push requests a server writes
  ``param_backup_root/param-<n>.txt`` (/root/reference/src/core/system/server/init.h:126-149);
* on terminate the final table goes to stdout (server/terminate.h:36);
* one line per key: ``key<TAB>value`` (sparsetable.h:49-56); a vector value is
  printed space separated (the reference's Vec prints ``Vec:\\t`` first —
  accepted on load);
* there is NO loader in the reference.

Here (works for ``HbmTable`` and ``HostTable``):
* ``save_text`` / ``load_text`` — same line format; optional `` | state``
  tail (optimizer state) makes a dump resumable bit-exactly (precision 9).
  Device compaction (K8 ``export``) -> D2H -> multi-threaded C++ formatter.
* ``save_binary`` / ``load_binary`` — header + ``u64 keys[n]`` + ``f32
  rows[n, width]``, the fast default for large tables.
* sharded checkpoints: one file per server rank
  (``<prefix>.shard<r>-of-<N>.<ext>``); ``load_sharded`` re-routes every key
  through the current router, so a job can resume on a different world size.
"""
from __future__ import annotations

import glob
import io
import json
import os
import struct
from typing import Iterable, Optional

import numpy as np
import torch

from .._native import host

MAGIC = b"SSCKPT01"


def _iter_export(table) -> Iterable[tuple[np.ndarray, np.ndarray]]:
    for k, r in table.export():
        yield (k.numpy().view(np.uint64) if isinstance(k, torch.Tensor) else k,
               r.numpy() if isinstance(r, torch.Tensor) else r)


def save_text(table, path: str, precision: int = 9, with_state: bool = False) -> int:
    """Write ``key\\tv0 v1 ...`` lines; returns the number of keys written."""
    n = 0
    h = host()
    out = open(path, "wb") if path != "-" else None
    try:
        for k, r in _iter_export(table):
            b = h.format_rows(np.ascontiguousarray(k), np.ascontiguousarray(r, dtype=np.float32),
                              table.dim, table.width, with_state, precision)
            if out is None:
                import sys

                sys.stdout.buffer.write(b)
            else:
                out.write(b)
            n += len(k)
    finally:
        if out is not None:
            out.close()
    return n


def read_text(path: str, dim: int, width: int, state_init: float = 0.0):
    with open(path, "rb") as f:
        data = f.read()
    return host().parse_rows(data, dim, width, state_init)


def _assign(table, keys: np.ndarray, rows: np.ndarray, chunk: int = 1 << 22):
    for a in range(0, len(keys), chunk):
        k = torch.from_numpy(np.ascontiguousarray(keys[a:a + chunk]).view(np.int64))
        r = torch.from_numpy(np.ascontiguousarray(rows[a:a + chunk]))
        table.assign(k, r)


def load_text(table, path: str, key_filter=None) -> int:
    keys, rows = read_text(path, table.dim, table.width, table.init_cfg.state_init)
    if key_filter is not None:
        m = key_filter(keys)
        keys, rows = keys[m], rows[m]
    _assign(table, keys, rows)
    table.check()
    return len(keys)


def save_binary(table, path: str, meta: Optional[dict] = None) -> int:
    parts_k, parts_r = [], []
    for k, r in _iter_export(table):
        parts_k.append(np.ascontiguousarray(k))
        parts_r.append(np.ascontiguousarray(r, dtype=np.float32))
    keys = np.concatenate(parts_k) if parts_k else np.zeros(0, np.uint64)
    rows = np.concatenate(parts_r) if parts_r else np.zeros((0, table.width), np.float32)
    hdr = json.dumps({"dim": table.dim, "width": table.width, "n": int(len(keys)),
                      "optimizer": table.opt.kind, "opt_step": table.opt.step,
                      **(meta or {})}).encode()
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC + struct.pack("<I", len(hdr)) + hdr)
        f.write(keys.astype("<u8").tobytes())
        f.write(rows.astype("<f4").tobytes())
    os.replace(tmp, path)
    return len(keys)


def read_binary(path: str):
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not a swiftsnails_amd binary checkpoint")
        (hl,) = struct.unpack("<I", f.read(4))
        hdr = json.loads(f.read(hl))
        n, w = hdr["n"], hdr["width"]
        off = 12 + hl
    keys = np.fromfile(path, dtype="<u8", count=n, offset=off)
    rows = np.fromfile(path, dtype="<f4", count=n * w, offset=off + 8 * n).reshape(n, w)
    return hdr, keys, rows


def load_binary(table, path: str, key_filter=None) -> int:
    hdr, keys, rows = read_binary(path)
    if hdr["width"] != table.width or hdr["dim"] != table.dim:
        raise ValueError(f"checkpoint layout dim={hdr['dim']} width={hdr['width']} != table "
                         f"dim={table.dim} width={table.width}")
    if key_filter is not None:
        m = key_filter(keys)
        keys, rows = keys[m], rows[m]
    _assign(table, keys, rows)
    table.opt.step = max(table.opt.step, int(hdr.get("opt_step", 0)))
    table.check()
    return len(keys)


# ----------------------------------------------------------------- sharded
def shard_path(prefix: str, rank: int, world: int, fmt: str = "bin") -> str:
    return f"{prefix}.shard{rank}-of-{world}.{'txt' if fmt == 'text' else 'bin'}"


def save_sharded(table, prefix: str, rank: int, world: int, fmt: str = "bin",
                 with_state: bool = True) -> str:
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    p = shard_path(prefix, rank, world, fmt)
    if fmt == "text":
        save_text(table, p, with_state=with_state)
    else:
        save_binary(table, p)
    return p


def load_sharded(table, prefix: str, owner_fn=None) -> int:
    """Load every shard file of `prefix`, keeping keys for which
    ``owner_fn(keys) -> bool mask`` is true (re-sharding on resume)."""
    files = sorted(glob.glob(prefix + ".shard*-of-*.bin")) + sorted(
        glob.glob(prefix + ".shard*-of-*.txt"))
    if not files:
        raise FileNotFoundError(f"no checkpoint shards for prefix {prefix}")
    n = 0
    for f in files:
        n += (load_binary if f.endswith(".bin") else load_text)(table, f, key_filter=owner_fn)
    return n


def owner_filter(frag_rank_map: np.ndarray, rank: int):
    """Key mask: keys the router assigns to `rank` (fmix64(key) % frag_num)."""
    from ..parallel.router import route_keys_np

    return lambda keys: route_keys_np(keys, frag_rank_map) == rank


__all__ = ["save_text", "load_text", "read_text", "save_binary", "load_binary", "read_binary",
           "save_sharded", "load_sharded", "shard_path", "owner_filter", "io"]
