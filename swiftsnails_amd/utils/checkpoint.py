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
  rows[n, width]``, the fast default for large tables.  Both stream: host
  memory is one export / load chunk regardless of the shard size (a 288 GB
  HBM shard does not have to fit in host RAM).
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
    """Write ``key\\tv0 v1 ...`` lines; returns the number of keys written.

    A file is written to ``path.tmp``, fsynced and renamed into place, so a
    crash mid-dump never leaves a truncated shard under ``path`` (which
    ``latest_checkpoint`` would otherwise count, and ``parse_rows`` would
    read with its cut-off last line defaulted).  ``path == "-"``: stdout,
    the reference's final dump (server/terminate.h:36)."""
    n = 0
    h = host()
    if path == "-":
        import sys

        for k, r in _iter_export(table):
            sys.stdout.buffer.write(h.format_rows(
                np.ascontiguousarray(k), np.ascontiguousarray(r, dtype=np.float32),
                table.dim, table.width, with_state, precision))
            n += len(k)
        sys.stdout.buffer.flush()
        return n
    tmp = path + ".tmp"
    try:
        with open(tmp, "wb") as out:
            for k, r in _iter_export(table):
                out.write(h.format_rows(np.ascontiguousarray(k),
                                        np.ascontiguousarray(r, dtype=np.float32),
                                        table.dim, table.width, with_state, precision))
                n += len(k)
            out.flush()
            os.fsync(out.fileno())
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise
    os.replace(tmp, path)
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


def iter_text(path: str, dim: int, width: int, state_init: float = 0.0,
              block_bytes: int = 64 << 20):
    """Parse a text dump in ~``block_bytes`` blocks cut at line ends."""
    h = host()
    with open(path, "rb") as f:
        tail = b""
        while True:
            b = f.read(block_bytes)
            if not b:
                break
            b = tail + b
            cut = b.rfind(b"\n")
            if cut < 0:
                tail = b
                continue
            tail = b[cut + 1:]
            yield h.parse_rows(b[:cut + 1], dim, width, state_init)
        if tail.strip():
            yield h.parse_rows(tail, dim, width, state_init)


def load_text(table, path: str, key_filter=None) -> int:
    n = 0
    for keys, rows in iter_text(path, table.dim, table.width, table.init_cfg.state_init):
        if key_filter is not None:
            m = key_filter(keys)
            keys, rows = keys[m], rows[m]
        if len(keys):
            _assign(table, keys, rows)
            n += len(keys)
    table.check()
    return n


def _header(path: str):
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not a swiftsnails_amd binary checkpoint")
        (hl,) = struct.unpack("<I", f.read(4))
        hdr = json.loads(f.read(hl))
    return hdr, 12 + hl


def save_binary(table, path: str, meta: Optional[dict] = None) -> int:
    """Stream the table to ``path`` chunk by chunk.

    Host memory stays at one export chunk (keys + rows of ``chunk_slots``
    table slots) whatever the shard size: ``n`` comes from ``table.size()``,
    so the key block and the row block are each written at their final
    offset with ``os.pwrite`` as chunks arrive.  Written to ``path.tmp`` and
    renamed, so a crash never leaves a truncated checkpoint under ``path``.
    """
    n = int(table.size())
    w = table.width
    hdr = json.dumps({"dim": table.dim, "width": w, "n": n,
                      "optimizer": table.opt.kind, "opt_step": table.opt.step,
                      **(meta or {})}).encode()
    off = 12 + len(hdr)
    tmp = path + ".tmp"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        os.pwrite(fd, MAGIC + struct.pack("<I", len(hdr)) + hdr, 0)
        m = 0
        for k, r in _iter_export(table):
            c = len(k)
            if m + c > n:
                raise RuntimeError(f"{path}: table grew while saving ({m + c} > {n} keys)")
            kb = np.ascontiguousarray(k).astype("<u8", copy=False).tobytes()
            rb = np.ascontiguousarray(r, dtype="<f4").tobytes()
            os.pwrite(fd, kb, off + 8 * m)
            os.pwrite(fd, rb, off + 8 * n + 4 * w * m)
            m += c
        if m != n:
            raise RuntimeError(f"{path}: exported {m} keys, table.size() said {n}")
        os.fsync(fd)
    except BaseException:
        os.close(fd)
        os.unlink(tmp)
        raise
    os.close(fd)
    os.replace(tmp, path)
    return n


def iter_binary(path: str, chunk: int = 1 << 22):
    """Yield ``(keys u64 [c], rows f32 [c, width])`` chunks of a binary
    checkpoint without reading the whole file."""
    hdr, off = _header(path)
    n, w = hdr["n"], hdr["width"]
    for a in range(0, n, chunk):
        c = min(chunk, n - a)
        keys = np.fromfile(path, dtype="<u8", count=c, offset=off + 8 * a)
        rows = np.fromfile(path, dtype="<f4", count=c * w,
                           offset=off + 8 * n + 4 * w * a).reshape(c, w)
        yield keys, rows


def read_binary(path: str):
    """Whole-file read (small tables / tests); ``iter_binary`` streams."""
    hdr, off = _header(path)
    n, w = hdr["n"], hdr["width"]
    keys = np.fromfile(path, dtype="<u8", count=n, offset=off)
    rows = np.fromfile(path, dtype="<f4", count=n * w, offset=off + 8 * n).reshape(n, w)
    return hdr, keys, rows


def load_binary(table, path: str, key_filter=None, chunk: int = 1 << 22) -> int:
    """Stream a binary checkpoint into ``table`` (``chunk`` keys at a time),
    keeping the keys ``key_filter`` selects."""
    hdr, _ = _header(path)
    if hdr["width"] != table.width or hdr["dim"] != table.dim:
        raise ValueError(f"checkpoint layout dim={hdr['dim']} width={hdr['width']} != table "
                         f"dim={table.dim} width={table.width}")
    n = 0
    for keys, rows in iter_binary(path, chunk):
        if key_filter is not None:
            m = key_filter(keys)
            keys, rows = keys[m], rows[m]
        if len(keys):
            _assign(table, keys, rows, chunk)
            n += len(keys)
    table.opt.step = max(table.opt.step, int(hdr.get("opt_step", 0)))
    table.check()
    return n


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


_SHARD_RE = None


def _shard_re():
    import re

    global _SHARD_RE
    if _SHARD_RE is None:
        _SHARD_RE = re.compile(r"^(.*)\.shard(\d+)-of-(\d+)\.(bin|txt)$")
    return _SHARD_RE


def shard_sets(prefix: str, fmt: Optional[str] = None) -> dict[int, dict[int, list[str]]]:
    """Shard files of ``prefix`` grouped by the world size that wrote them:
    ``{world: {rank: [paths]}}`` (a rank lists two paths when both a ``.bin``
    and a ``.txt`` exist).  ``fmt`` ("bin" / "text") keeps one format."""
    ext = None if fmt is None else ("txt" if fmt == "text" else "bin")
    out: dict[int, dict[int, list[str]]] = {}
    base = os.path.basename(prefix)
    for f in sorted(glob.glob(glob.escape(prefix) + ".shard*-of-*.*")):
        m = _shard_re().match(os.path.basename(f))
        if not m or m.group(1) != base or (ext is not None and m.group(4) != ext):
            continue
        out.setdefault(int(m.group(3)), {}).setdefault(int(m.group(2)), []).append(f)
    return out


def _complete(by_rank: dict[int, list[str]], world: int) -> bool:
    return set(by_rank) == set(range(world))


def select_shards(prefix: str, world: Optional[int] = None, fmt: Optional[str] = None) -> list[str]:
    """The files of exactly ONE complete shard set of ``prefix``: shards
    ``0..world-1`` written by one job.  Stale shards of another world size
    or format next to it are never mixed in (rows loaded later would
    overwrite newer ones).  Without ``world`` the prefix must hold a single
    complete set; several are ambiguous and raise ValueError."""
    sets = shard_sets(prefix, fmt)
    if world is not None:
        by = sets.get(int(world), {})
        if not _complete(by, int(world)):
            raise FileNotFoundError(f"no complete {world}-shard checkpoint for prefix {prefix}")
        chosen = int(world)
    else:
        complete = [w for w, by in sets.items() if _complete(by, w)]
        if not complete:
            raise FileNotFoundError(f"no complete checkpoint shard set for prefix {prefix}")
        if len(complete) > 1:
            raise ValueError(f"checkpoint prefix {prefix} holds complete shard sets of world "
                             f"sizes {sorted(complete)}; pass world= to choose one")
        chosen = complete[0]
    files = []
    for r in range(chosen):
        paths = sets[chosen][r]
        if len(paths) > 1:
            raise ValueError(f"shard {r} of {prefix} exists as {paths}; pass fmt= to choose")
        files.append(paths[0])
    return files


def load_sharded(table, prefix: str, owner_fn=None, world: Optional[int] = None,
                 fmt: Optional[str] = None) -> int:
    """Load the shard set of `prefix` (``select_shards``), keeping keys for
    which ``owner_fn(keys) -> bool mask`` is true (re-sharding on resume)."""
    n = 0
    for f in select_shards(prefix, world, fmt):
        n += (load_binary if f.endswith(".bin") else load_text)(table, f, key_filter=owner_fn)
    return n


def latest_checkpoint(root: str, stem: str = "param-") -> Optional[tuple[str, int, int, str]]:
    """Newest COMPLETE periodic backup under `root`: ``(prefix, round, world,
    fmt)`` of the highest ``<stem><round>`` with a shard set
    ``.shard<r>-of-<W>`` of one format present for every r < W.  A job that
    died while writing a backup leaves an incomplete set, which is skipped;
    shard files are renamed into place only once fully written (save_text /
    save_binary).  When one round holds complete sets of several world sizes
    or formats (a re-run at another size, or after ``checkpoint_format``
    changed), the most recently written set wins, and its format is returned
    so the load reads that set only.  None if there is none."""
    best = None
    seen = set()
    for f in glob.glob(os.path.join(root, glob.escape(stem) + "*.shard*-of-*.*")):
        m = _shard_re().match(os.path.basename(f))
        if not m or not m.group(1).startswith(stem):
            continue
        rnd_s = m.group(1)[len(stem):]
        if not rnd_s.isdigit() or m.group(1) in seen:
            continue
        seen.add(m.group(1))
        prefix = os.path.join(root, m.group(1))
        for fmt in ("bin", "text"):
            for w, by in shard_sets(prefix, fmt).items():
                if not _complete(by, w):
                    continue
                mtime = max(os.path.getmtime(p) for ps in by.values() for p in ps)
                cand = (int(rnd_s), mtime, prefix, w, fmt)
                if best is None or cand[:2] > best[:2]:
                    best = cand
    if best is None:
        return None
    return best[2], best[0], best[3], best[4]


def owner_filter(frag_rank_map: np.ndarray, rank: int):
    """Key mask: keys the router assigns to `rank` (fmix64(key) % frag_num)."""
    from ..parallel.router import route_keys_np

    return lambda keys: route_keys_np(keys, frag_rank_map) == rank


__all__ = ["save_text", "load_text", "read_text", "iter_text", "save_binary", "load_binary",
           "read_binary", "iter_binary", "latest_checkpoint", "save_sharded", "load_sharded",
           "select_shards", "shard_sets", "shard_path", "owner_filter", "io"]
