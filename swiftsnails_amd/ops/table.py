"""HBM-resident sparse parameter table (one shard per GPU).

Replaces ``SparseTable``/``SparseTableShard`` (google dense_hash_map + pthread
RW lock per shard, /root/reference/src/core/parameter/sparsetable.h:5-121) and
the server halves of ``PullAccessAgent``/``PushAccessAgent``
(sparsetable.h:123-222) with an open-addressed table in HBM driven by the
HIP kernels of ``csrc/hip/table.hip``:

* ``pull``  = lookup-or-init + row gather (K3/K4); missing keys are created
  with the configured initialiser, exactly like ``get_pull_value``.
* ``push``  = fused probe/update (K5) with the configured optimizer.
* ``export``/``assign`` = slot compaction / bulk insert (K8) used by the text
  and binary checkpoints and by ``resize``.

Slot layout: ``[row: width fp32 | pad | key u64]`` (see ss_device.h).
Sizing: ``HbmTable.plan(n_keys, dim, optimizer, load=0.7)`` gives the bytes a
shard needs; a 1B-key sparse-LR table (AdaGrad) is 1B/0.7 * 16 B ≈ 23 GB, so
it fits a single MI355X's 288 GB with room to spare.
"""
from __future__ import annotations

import math
import os
from typing import Iterator, Optional

import numpy as np
import torch

from ..utils.streams import current_raw
from .._native import hip
from .optim import InitConfig, Optimizer

EMPTY_I64 = -1  # u64 0xFFFF_FFFF_FFFF_FFFF
CTR_SHARDS = 256  # == ss::kCtrShards


def loss_buffer(device) -> torch.Tensor:
    """Sharded fp32 accumulator the fused model kernels add their loss into
    (256 shards x 128 B, ss::ctr_addf); read it with ``.sum()``."""
    return torch.zeros(CTR_SHARDS * 32, dtype=torch.float32, device=device)


def _align(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def slot_layout(width: int, layout: Optional[str] = None,
                elem: int = 4) -> tuple[int, int, int]:
    """(stride_bytes, key_offset_bytes, row_offset_bytes) of one slot;
    ``elem``: bytes per row element (4 fp32, 2 compact bf16 rows).

    ``rowfirst``: [row | key] (scalar rows: LR's 16-byte [w, h, key] slot).
    ``keyfirst``: [key | row], so the key and the parameters a pull reads sit
    together at the slot's start.  ``keyfirst_line``: the same, stride padded
    to whole 64-byte lines (a pull of key + params touches one line)."""
    layout = layout or os.environ.get("SS_TABLE_LAYOUT", "") or (
        "rowfirst" if width <= 2 else "keyfirst")
    if layout == "rowfirst":
        key_off = _align(elem * width, 8)
        stride = key_off + 8
        if width >= 4:
            stride = _align(stride, 16)
        return stride, key_off, 0
    if layout not in ("keyfirst", "keyfirst_line"):
        raise ValueError(f"slot layout {layout!r}")
    stride = _align(8 + elem * width, 16 if width >= 2 else 8)
    if layout == "keyfirst_line":
        stride = _align(stride, 64)
    # a row of whole 16-byte vectors starts 16-byte aligned (the stride's
    # padding moves in front of it: [key | pad | row], same stride), so wide
    # rows move as float4s (table.hip k_pull_rows_bk)
    row_off = 16 if (elem * width) % 16 == 0 and stride >= 16 + elem * width else 8
    return stride, 0, row_off


def default_lane_group(width: int) -> int:
    if width <= 2:
        return 1
    if width <= 32:   # FM k=8 + AdaGrad (18 floats): G=4 measured 0.75 vs 0.80 ms/step at G=16
        return 4
    if width <= 128:
        return 16
    return 64


def _stream_ptr(stream) -> int:
    if stream is None:
        return current_raw()
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _i16(u: int) -> int:
    """A 16-bit pattern as the signed value torch.int16 holds."""
    u &= 0xFFFF
    return u - 0x10000 if u >= 0x8000 else u


class TableFullError(RuntimeError):
    pass



class HbmTable:
    """One GPU shard of the sparse parameter table."""

    def __init__(self, dim: int, capacity: int, optimizer: Optional[Optimizer] = None,
                 init: Optional[InitConfig] = None, device=None, lane_group: Optional[int] = None,
                 max_load: float = 0.85, row_dtype: str = "fp32"):
        if dim < 1:
            raise ValueError("dim must be >= 1")
        if capacity < 1:
            raise ValueError("capacity must be >= 1")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.dim = int(dim)
        self.opt = optimizer or Optimizer()
        self.init_cfg = init or InitConfig()
        self.width = self.dim + self.opt.state_width(self.dim)
        # "bf16": compact rows (parameters and optimizer state in bf16, fp32
        # math, stochastically rounded updates): half the row bytes, for
        # tables that do not fit at fp32 (the 10B-key FM table)
        if row_dtype not in ("fp32", "bf16"):
            raise ValueError(f"row_dtype must be fp32 or bf16, not {row_dtype!r}")
        self.row_dtype = row_dtype
        self.bf16 = row_dtype == "bf16"
        self.elem = 2 if self.bf16 else 4
        self.stride, self.key_off, self.row_off = slot_layout(self.width, elem=self.elem)
        self.G = lane_group or int(os.environ.get("SS_TABLE_G", "0")) or \
            default_lane_group(self.width)
        self.max_load = max_load
        # bumped by every row-modifying call: a pull snapshot (pull_buckets
        # snap=) is valid for a blind-write apply only while it is unchanged
        self.version = 0
        # user-defined update rule (set_push_method), else the optimizer menu
        self.push_fn = None
        # user-defined initialiser / pull transform (set_init_method,
        # set_pull_method), else the compiled init menu and the identity
        self.init_fn = None
        self.pull_fn = None
        self._alloc(int(capacity))
        self._init_native = self.init_cfg.native()

    # -- storage ------------------------------------------------------------
    def _region_bits(self, cap: int) -> int:
        """Region count (log2) of a new allocation of ``cap`` slots: scalar
        16-byte [w | h | key] rows (sparse LR) are split into 2^rbits equal
        regions of >= 1024 slots (at most 2^16), inside which each key probes
        (ss_device.h ProbeSeq): the one-GPU engine then buckets whole regions
        per dedup workgroup and inserts without device atomics
        (table.hip k_pull_claim_bk).  0: one region (SS_TABLE_REGIONS=0, other
        layouts, tables under 64K slots)."""
        if (os.environ.get("SS_TABLE_REGIONS", "1") == "0" or self.bf16 or self.width != 2
                or self.dim != 1 or (self.stride, self.key_off, self.row_off) != (16, 8, 0)
                or cap >= (1 << 31) - (1 << 16)):
            return 0
        rb = min(16, max(0, (cap // 1024).bit_length() - 1))
        return rb if rb >= 6 else 0

    def _alloc(self, cap: int):
        self.rbits = self._region_bits(cap)
        if self.rbits:  # whole regions: capacity rounded up to a multiple of 2^rbits
            R = 1 << self.rbits
            cap = -(-cap // R) * R
        self.capacity = cap
        self.version += 1
        self.storage = torch.empty(cap * self.stride, dtype=torch.uint8, device=self.device)
        # key-independent init (zero): fill every row with the initial row up
        # front, so an insert is the key CAS alone (SS_TABLE_PREFILL=0: off)
        self.prefilled = (self.init_cfg.kind == "zero" and getattr(self, "init_fn", None) is None
                          and os.environ.get("SS_TABLE_PREFILL", "1") != "0")
        if self.prefilled:
            self.storage.zero_()
            slots = self.storage.view(cap, self.stride)
            slots[:, self.key_off:self.key_off + 8].fill_(255)  # every key word = EMPTY
            if self.width > self.dim and float(self.init_cfg.state_init) != 0.0:
                self.rows_view()[:, self.dim:].fill_(float(self.init_cfg.state_init))
        else:
            self.storage.fill_(255)  # every key word = EMPTY (rows: the 0xFF sentinel)
        # sharded counter: 256 shards x 128 B (see ss_device.h ctr_add)
        self.size_ctr = torch.zeros(CTR_SHARDS * 16, dtype=torch.int64, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._make_dt()

    def _make_dt(self):
        # a tensor-code initialiser needs the insert to write its marker row
        # (the prefilled fast path writes nothing on insert)
        self.dt = hip().DevTable(self.storage.data_ptr(), self.capacity, self.stride,
                                 self.key_off, self.dim, self.width,
                                 int(self.prefilled and self.init_fn is None), self.row_off,
                                 int(self.bf16), self.rbits)

    @staticmethod
    def plan(n_keys: int, dim: int, optimizer: Optional[Optimizer] = None,
             load: float = 0.7, row_dtype: str = "fp32") -> dict:
        opt = optimizer or Optimizer()
        width = dim + opt.state_width(dim)
        stride, _, _ = slot_layout(width, elem=2 if row_dtype == "bf16" else 4)
        cap = int(math.ceil(n_keys / load))
        return {"capacity": cap, "stride": stride, "bytes": cap * stride, "width": width}

    @classmethod
    def for_keys(cls, n_keys: int, dim: int, load: float = 0.7, **kw) -> "HbmTable":
        return cls(dim, max(16, int(math.ceil(n_keys / load))), **kw)

    @property
    def nbytes(self) -> int:
        return self.capacity * self.stride

    def set_optimizer(self, opt: Optimizer):
        if opt.state_width(self.dim) != self.width - self.dim:
            raise ValueError("optimizer state width differs from the table layout")
        self.opt = opt

    # -- hot path -----------------------------------------------------------
    def _seg(self, n: int):
        return hip().SegList.from_host([0], [int(n)])

    @staticmethod
    def segs(offsets, counts):
        """Segment list over one buffer: (offset, count) pairs in rows."""
        return hip().SegList.from_host([int(o) for o in offsets], [int(c) for c in counts])

    @staticmethod
    def dev_segs(count: torch.Tensor):
        """Single segment at offset 0 whose length is ``count[0]`` on the device."""
        return hip().SegList.from_device(count.data_ptr())

    def pull(self, keys: torch.Tensor, insert: bool = True, unique: bool = False,
             out: Optional[torch.Tensor] = None, slots: Optional[torch.Tensor] = None,
             segs=None, max_n: Optional[int] = None, stream=None):
        """Lookup-or-init (insert=True) + gather. Returns (vals[n, dim], slots[n])."""
        n = keys.numel() if max_n is None else max_n
        st = _stream_ptr(stream)
        h = hip()
        if out is None:
            out = torch.empty((keys.numel(), self.dim), dtype=torch.float32, device=self.device)
        if slots is None:
            slots = torch.empty(keys.numel(), dtype=torch.int64, device=self.device)
        sl = segs if segs is not None else self._seg(keys.numel())
        # the CAS-insert fused kernel is also correct for duplicate keys (a
        # lane reading a row another lane is initialising substitutes the
        # deterministic init value)
        if insert:
            h.pull_unique(self.dt, keys.data_ptr(), sl, n, slots.data_ptr(), out.data_ptr(),
                          self._init_native, self.size_ctr.data_ptr(), self.err.data_ptr(),
                          self.G, st)
        else:
            h.probe(self.dt, keys.data_ptr(), sl, n, slots.data_ptr(), self._init_native,
                    int(insert), self.size_ctr.data_ptr(), self.err.data_ptr(), self.G, st)
            h.gather(self.dt, slots.data_ptr(), sl, n, out.data_ptr(), self.G, st)
        if self.custom_pull and segs is None:
            self.finish_pull(slots, out)
        return out, slots

    @property
    def snapshot_ok(self) -> bool:
        """Rows are (w, h) scalar AdaGrad pairs the pull can snapshot."""
        return (self.G == 1 and self.dim == 1 and self.width == 2 and self.push_fn is None and
                not self.bf16 and
                not self.custom_pull and
                self.opt.kind == "adagrad" and self.stride % 8 == 0 and self.row_off % 8 == 0)

    # -- user-defined access methods (tensor code) ---------------------------
    @property
    def custom_pull(self) -> bool:
        return self.init_fn is not None or self.pull_fn is not None

    def set_init_method(self, fn) -> None:
        """The reference's ``PullAccessMethod::init_param`` as tensor code
        (/root/reference/src/core/parameter/sparse_access_method.h:10-28,
        called by lookup-or-init, sparsetable.h:142-149): ``fn(keys) ->
        rows`` gives the full rows [n, width] (parameters, then optimizer
        state) of keys a pull creates.  The device insert writes a NaN marker
        row; ``finish_pull`` finds the marked rows among a pull's and replaces
        them.  ``None`` restores the compiled initialiser."""
        was = self.init_fn
        self.init_fn = fn
        self._init_native = (InitConfig("marker", state_init=self.init_cfg.state_init).native()
                             if fn is not None else self.init_cfg.native())
        if fn is not None and was is None and self.prefilled:
            # empty rows hold the prefilled initial row; a concurrent reader
            # of a key being inserted must see the 0xFF "not written yet"
            # pattern instead (table.hip fresh_or)
            empty = self.keys_view() == EMPTY_I64
            rv = self.rows_view()
            fill = torch.tensor(-1, dtype=torch.int16 if self.bf16 else torch.int32,
                                device=self.device).view(rv.dtype)
            rv[empty] = fill
        self._make_dt()
        self.version += 1

    def set_pull_method(self, fn) -> None:
        """The reference's ``PullAccessMethod::get_pull_value`` as tensor
        code: ``fn(keys, rows) -> vals`` maps the stored rows [n, width] to the
        values [n, dim] a pull returns (e.g. a weight derived from optimizer
        state).  ``None`` returns the parameters as stored."""
        self.pull_fn = fn
        self.version += 1

    def keys_view(self) -> torch.Tensor:
        """[capacity] int64 view of every slot's key word (strided)."""
        return self.storage.view(torch.int64).view(self.capacity, self.stride // 8)[
            :, self.key_off // 8]

    def finish_pull(self, slots: torch.Tensor, out: torch.Tensor, n=None) -> None:
        """Apply the tensor-code initialiser / pull transform to the rows a
        pull just produced: ``slots`` [n] (resolved slots, -1 = none), ``out``
        [n, dim] (the pulled values, rewritten).  ``n``: a host count or a
        device count tensor (synced).  On the current stream."""
        if not self.custom_pull:
            return
        if n is None:
            n = slots.numel()
        elif isinstance(n, torch.Tensor):
            n = int(n.reshape(-1).sum().item())
        if n == 0:
            return
        s = slots.reshape(-1)[:n]
        ok = s >= 0
        s = s[ok]
        rv = self.rows_view()
        raw = rv[s]
        rows = raw.to(torch.float32)
        keys = self.keys_view()[s]
        if self.init_fn is not None:
            from .optim import INIT_MARKER_BITS

            if self.bf16:  # a compact row keeps the marker's top 16 bits
                new = raw[:, 0].view(torch.int16) == _i16(INIT_MARKER_BITS >> 16)
            else:
                new = raw[:, 0].view(torch.int32) == INIT_MARKER_BITS
            if bool(new.any()):
                r = torch.as_tensor(self.init_fn(keys[new]), dtype=torch.float32,
                                    device=self.device)
                if r.shape != (int(new.sum()), self.width):
                    raise ValueError(f"init method returned {tuple(r.shape)}, expected "
                                     f"{(int(new.sum()), self.width)}")
                rv[s[new]] = r.to(rv.dtype)
                rows[new] = r
        vals = rows[:, :self.dim]
        if self.pull_fn is not None:
            vals = torch.as_tensor(self.pull_fn(keys, rows), dtype=torch.float32,
                                   device=self.device)
            if vals.shape != (s.numel(), self.dim):
                raise ValueError(f"pull method returned {tuple(vals.shape)}, expected "
                                 f"{(s.numel(), self.dim)}")
        o = out.reshape(-1, self.dim)[:n]
        o[ok] = vals

    # -- user-defined update rule -------------------------------------------
    def set_push_method(self, fn) -> None:
        """Replace the optimizer menu by ``fn(rows, grads) -> new_rows``, the
        reference's ``PushAccessMethod::apply_push_value`` as tensor code
        (/root/reference/src/core/parameter/sparse_access_method.h:30-48):
        ``rows`` [n, width] are the pushed keys' full rows (parameters, then
        the optimizer state columns of ``optimizer.state_width(dim)``),
        ``grads`` [n, dim] their merged gradients; the returned rows are
        stored back.  Runs as torch ops on the gathered rows (two random row
        passes instead of the fused update kernel).  ``None`` restores the
        built-in rule."""
        self.push_fn = fn
        self.version += 1

    def rows_view(self) -> torch.Tensor:
        """[capacity, width] float32 view of every slot's row (strided)."""
        dt = torch.bfloat16 if self.bf16 else torch.float32
        rows = self.storage.view(dt).view(self.capacity, self.stride // self.elem)
        r0 = self.row_off // self.elem
        return rows[:, r0:r0 + self.width]

    def apply_custom(self, slots: torch.Tensor, grads: torch.Tensor, stream=None) -> None:
        """Apply ``push_fn`` at resolved ``slots`` (unique; -1 = skipped)."""
        if stream is None:
            st = torch.cuda.current_stream()
        elif isinstance(stream, int):
            st = torch.cuda.ExternalStream(stream, device=self.device)
        else:
            st = stream
        with torch.cuda.stream(st):
            s = slots.reshape(-1)
            g = grads.reshape(s.numel(), self.dim)
            ok = s >= 0
            s, g = s[ok], g[ok]
            if s.numel() == 0:
                return
            rv = self.rows_view()
            new = self.push_fn(rv[s].to(torch.float32), g.to(torch.float32))
            new = torch.as_tensor(new, dtype=torch.float32, device=self.device)
            if new.shape != (s.numel(), self.width):
                raise ValueError(f"push method returned {tuple(new.shape)}, "
                                 f"expected {(s.numel(), self.width)}")
            rv[s] = new.to(rv.dtype)
            self.version += 1

    def pull_buckets(self, view, out: torch.Tensor, slots: torch.Tensor, stream=None,
                     snap: Optional[torch.Tensor] = None):
        """Unique-key lookup-or-init + gather straight from a bucketed dedup
        (``Deduper.bucket_view()``): rows land at their compact unique ids.  ``snap`` ([ucap, 2] float32,
        ``snapshot_ok`` tables): also write each key's (w, h) there, for a
        ``push_slots(snap=)`` that needs no random row read."""
        bkeys, bstart, unum, ubase, P = view
        if snap is not None and not self.snapshot_ok:
            raise ValueError("pull snapshot needs scalar AdaGrad rows (dim 1, G 1)")
        hip().pull_unique_bk(self.dt, bkeys, bstart, unum, ubase, P, slots.data_ptr(),
                             out.data_ptr(), self._init_native, self.size_ctr.data_ptr(),
                             self.err.data_ptr(), self.G, _stream_ptr(stream),
                             0 if snap is None else snap.data_ptr())
        return out, slots

    def lookup_slots(self, keys: torch.Tensor, insert: bool = False, segs=None,
                     max_n: Optional[int] = None, stream=None) -> torch.Tensor:
        slots = torch.empty(keys.numel(), dtype=torch.int64, device=self.device)
        sl = segs if segs is not None else self._seg(keys.numel())
        hip().probe(self.dt, keys.data_ptr(), sl, keys.numel() if max_n is None else max_n,
                    slots.data_ptr(), self._init_native, int(insert), self.size_ctr.data_ptr(),
                    self.err.data_ptr(), self.G, _stream_ptr(stream))
        return slots

    def push_slots(self, slots: torch.Tensor, grads: torch.Tensor, segs=None,
                   max_n: Optional[int] = None, stream=None,
                   snap: Optional[torch.Tensor] = None):
        """Apply the optimizer at resolved slots (keys in one call must be unique).
        ``snap``: the (w, h) rows ``pull_buckets(snap=)`` read, updated and
        stored blind — the caller guarantees no row changed since (same
        ``version``)."""
        if self.push_fn is not None:
            if segs is not None:
                raise ValueError("push_slots with a custom push method takes whole slot lists")
            n = slots.numel() if max_n is None else max_n
            self.apply_custom(slots[:n], grads.reshape(-1, self.dim)[:n], stream)
            return
        sl = segs if segs is not None else self._seg(slots.numel())
        self.version += 1
        hip().apply(self.dt, slots.data_ptr(), grads.data_ptr(), sl,
                    slots.numel() if max_n is None else max_n, self.opt.native(), self.G,
                    _stream_ptr(stream), 0 if snap is None else snap.data_ptr())

    def push(self, keys: torch.Tensor, grads: torch.Tensor, stream=None):
        """push by key: keys missing from the table are created first (the
        reference CHECK-fails instead, sparsetable.h:184)."""
        slots = self.lookup_slots(keys, insert=True, stream=stream)
        if self.init_fn is not None:  # keys this push created: the user's rows first
            self.finish_pull(slots, torch.empty((slots.numel(), self.dim), device=self.device))
        self.push_slots(slots, grads.reshape(-1, self.dim).contiguous(), stream=stream)

    def next_round(self):
        """Advance per-round optimizer state (Adam bias correction)."""
        self.opt.step += 1

    # -- maintenance --------------------------------------------------------
    def size(self) -> int:
        return int(self.size_ctr.sum().item())

    def load_factor(self) -> float:
        return self.size() / self.capacity

    def probe_histogram(self, nbins: int = 32):
        """Distance of every stored key from its home slot (linear probing),
        binned; the last bin counts ``>= nbins-1``.  Scans the whole shard."""
        hist = torch.empty(nbins, dtype=torch.int64, device=self.device)
        hip().probe_hist(self.dt, hist.data_ptr(), nbins, _stream_ptr(None))
        return hist.cpu().numpy()

    def region_occupancy(self) -> dict:
        """Occupied slots per probe region of a region table (keys probe only
        inside the region their hash names, so the fullest region, not the
        table's load, is what fills first): max / mean / p99 / min over the
        2^rbits regions and the fullest region's fill fraction.  Reads every
        slot's key word (a device pass over the shard)."""
        if not self.rbits:
            return {}
        R = 1 << self.rbits
        rlen = self.capacity // R
        kw = self.storage.view(torch.int64).view(self.capacity, self.stride // 8)[
            :, self.key_off // 8]
        occ = (kw != -1).view(R, rlen).sum(1, dtype=torch.int64).float()
        q = torch.quantile(occ, torch.tensor([0.5, 0.99], device=occ.device))
        return {"regions": R, "region_slots": rlen, "max": int(occ.max()),
                "mean": float(occ.mean()), "p50": float(q[0]), "p99": float(q[1]),
                "min": int(occ.min()), "max_fill": float(occ.max()) / rlen}

    def stats(self) -> dict:
        """Observability snapshot: size, load factor, mean/max probe length."""
        import numpy as np

        h = self.probe_histogram(64)
        n = int(h.sum())
        d = np.arange(len(h))
        return {"size": self.size(), "capacity": self.capacity,
                "load_factor": self.size() / self.capacity,
                "probe_mean": float((h * d).sum() / n) if n else 0.0,
                "probe_p99": int(np.searchsorted(np.cumsum(h), 0.99 * n)) if n else 0,
                "probe_max_bin": int(np.nonzero(h)[0].max()) if n else 0,
                "hbm_bytes": int(self.storage.numel() * self.storage.element_size())}

    def check(self):
        e = int(self.err.item())
        if e & 1:
            if self.rbits:  # keys probe only inside the region their hash names
                raise TableFullError(
                    f"table region full: a key's probe region ({self.capacity >> self.rbits} "
                    f"slots, one of {1 << self.rbits}) has no empty slot; table size "
                    f"{self.size()} of {self.capacity} (load {self.size() / self.capacity:.3f}) "
                    "— the keys of that region were not inserted; size the shard for a lower load")
            raise TableFullError(f"table full: capacity {self.capacity}, size {self.size()}")
        if e & 2:
            raise ValueError("key 0xFFFFFFFFFFFFFFFF is reserved (empty-slot sentinel)")
        if e & 4:
            raise RuntimeError("a claimed slot was taken by another key before its commit (a "
                               "direct table insert between a claimed pull and its push)")

    def assign(self, keys: torch.Tensor, rows: torch.Tensor, stream=None):
        """Insert-or-overwrite full rows (params + optimizer state)."""
        keys = keys.to(self.device, torch.int64).contiguous()
        rows = rows.to(self.device, torch.float32).reshape(-1, self.width).contiguous()
        if rows.shape[0] != keys.numel():
            raise ValueError("rows/keys length mismatch")
        self.version += 1
        hip().assign(self.dt, keys.data_ptr(), rows.data_ptr(), keys.numel(),
                     self.size_ctr.data_ptr(), self.err.data_ptr(), self.G, _stream_ptr(stream))

    def export(self, chunk_slots: int = 1 << 24, to_host: bool = True
               ) -> Iterator[tuple[torch.Tensor, torch.Tensor]]:
        """Yield (keys int64, rows float32 [m, width]) for all occupied slots."""
        h = hip()
        st = _stream_ptr(None)
        cursor = torch.zeros(1, dtype=torch.int64, device=self.device)
        kbuf = torch.empty(min(chunk_slots, self.capacity), dtype=torch.int64, device=self.device)
        rbuf = torch.empty((min(chunk_slots, self.capacity), self.width), dtype=torch.float32,
                           device=self.device)
        for s0 in range(0, self.capacity, chunk_slots):
            n = min(chunk_slots, self.capacity - s0)
            cursor.zero_()
            h.export_slots(self.dt, s0, n, kbuf.data_ptr(), rbuf.data_ptr(), cursor.data_ptr(), st)
            m = int(cursor.item())
            if m:
                k, r = kbuf[:m], rbuf[:m]
                yield (k.cpu(), r.cpu()) if to_host else (k.clone(), r.clone())

    def resize(self, new_capacity: int):
        """Rehash into a new allocation (capacity planning / growth)."""
        if new_capacity < self.size():
            raise ValueError("new capacity smaller than the number of keys")
        chunks = list(self.export(to_host=False))
        old = self.storage
        self._alloc(int(new_capacity))
        del old
        for k, r in chunks:
            self.assign(k, r)
        self.check()

    def maybe_grow(self, incoming: int = 0, factor: float = 2.0) -> bool:
        if self.size() + incoming > self.max_load * self.capacity:
            self.resize(int(max(self.capacity * factor, (self.size() + incoming) / 0.5)))
            return True
        return False

    # -- dense views (tests / small tables) --------------------------------
    def to_dict(self, with_state: bool = False) -> dict[int, np.ndarray]:
        out = {}
        for k, r in self.export():
            kn = k.numpy().view(np.uint64)
            rn = r.numpy()
            for i in range(len(kn)):
                out[int(kn[i])] = rn[i] if with_state else rn[i, :self.dim]
        return out

    def __len__(self):
        return self.size()

    def __repr__(self):
        return (f"HbmTable(dim={self.dim}, width={self.width}, capacity={self.capacity}, "
                f"stride={self.stride}B, opt={self.opt.kind}, device={self.device})")
