"""Worker-side key dedup + routing (K1/K2) with preallocated scratch.

Replaces the caller-side ``std::unordered_set`` and ``arrange_local_vals``
grouping of ``pull_with_barrier``/``push_with_barrier``
(/root/reference/src/core/parameter/global_pull_access.h:40-72,
global_push_access.h:80-99).  Output layout is the alltoallv send layout:

* ``ukeys[nranks * ucap]``: unique keys, destination ``r`` owns
  ``[r*ucap, r*ucap + ucount[r])``;
* ``inv[n]``: occurrence -> unique id (index into rows laid out the same way);
* ``ugrad[nranks * ucap, gdim]``: zeroed gradient rows for the unique keys.

Two device implementations:

* ``bucket`` (default, bdedup.hip): partition occurrences by hash into
  ~1024-occurrence buckets whose ids encode the destination, dedup each
  bucket in LDS — no device-scope atomics; the partition (``pj``, ``luid``)
  is also the plan of the duplicate-merging gradient reduction (``reduce``);
* ``hash`` (dedup.hip): one global scratch hash table, a CAS per occurrence.

``dedup_reference`` is the host implementation used on CPU and by the tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..utils.hashing import fmix64
from ..utils.logging import get_logger
from .table import _stream_ptr

log = get_logger("swiftsnails.dedup")

INVALID = 0xFFFFFFFF


def _next_pow2(x: int) -> int:
    return 1 << max(4, (int(x) - 1).bit_length())


@dataclass
class DedupResult:
    ukeys: torch.Tensor       # int64 [nranks*ucap]
    ucount: torch.Tensor      # int64 [nranks] (device)
    inv: torch.Tensor         # int32 [n] (uint32 bit pattern; INVALID for bad keys)
    ugrad: Optional[torch.Tensor]
    ucap: int
    nranks: int
    n: int
    owner: object = None      # the Deduper (bucket mode: reduce plan lives there)
    lay: int = 0              # bucket-layout size (>= n; N>1 engines: max_keys)
    rbits: int = 0            # > 0: buckets hold whole regions of a 2^rbits-region table


class Deduper:
    """Device dedup/route with scratch sized for up to ``max_n`` keys per call."""

    def __init__(self, max_n: int, nranks: int = 1, frag_map: Optional[torch.Tensor] = None,
                 gdim: int = 1, device=None, with_grad: bool = True, zero_grad: bool = True,
                 mode: Optional[str] = None, record_layout: bool = False,
                 record_group: bool = False):
        from .._native import hip

        self.mode = mode or os.environ.get("SS_DEDUP", "bucket")
        if self.mode not in ("bucket", "hash"):
            raise ValueError(f"dedup mode {self.mode!r}")
        # zero_grad=False: the model's backward writes every unique row itself
        # (e.g. the segmented reduction of segreduce.hip), skip zeroing here.
        self.zero_grad = zero_grad
        # bucket mode: False skips the inverse-index pass; consumers then read
        # luid[pos_of[j]] themselves (the LR forward does, fused)
        self.materialize_inv = True
        # bucket mode: False skips the scatter's bucket-of-occurrence array
        # (BdIndex.bkt) when no consumer resolves uid(j) through it (the LR
        # forward in its one-gather mode reads occ[pos_of[j]] instead)
        self.need_bkt = True
        # bucket mode: False skips writing the contiguous send segment (ukeys)
        # when nothing reads it (the colocated 1-GPU engine pulls per bucket)
        self.need_ukeys = True
        # bucket mode, N>1 engines: lay the buckets out as a call of lay_n
        # keys whatever the call's n (every rank the same Pd buckets per
        # destination: the servers merge bucket k of all sources, server.hip)
        self.lay_n: Optional[int] = None
        # need_pos=False: no consumer reads the j -> bucket-position map
        # (pos_of), so the scatter skips writing it
        self.need_pos = True
        # bucket mode: per unique key, whether it occurs once in the batch
        # (``usingle``, compact unique ids) — lets the LR reduce store instead
        # of accumulate with LDS atomics.  Allocated by track_singletons().
        self.usingle = None
        # bucket mode, N>1 xGMI engines: each bucket's unique keys grouped by
        # the server's sub-bucket (msub > 1), with the offsets in ``usub``
        # ([P][msub], sent with the keys: the server reads its exact ranges)
        self.msub, self.usub = 1, None
        # bucket mode, one rank: bucket whole regions of a region table with
        # 2^rbits regions (ops/table.py _region_bits) when the call's layout
        # allows it (the kernel reports the bits it used: DedupResult.rbits)
        self.rbits = 0
        # bucket mode, N>1 record exchange (enable_records): no dedup — every
        # occurrence's key goes into ukeys at its send-segment position
        # (destination d from d * ucap), its occurrence index into ``spj``;
        # pos_of maps j to that position (the rows come back there)
        self.spj = None

        self.h = hip()
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.max_n = int(max_n)
        self.nranks = int(nranks)
        self.gdim = int(gdim)
        self.ucap = self.max_n
        # load <= 0.67 even if every key is unique; ~0.35 for CTR batches
        self.scap = _next_pow2(self.max_n + self.max_n // 2 + 1)
        self.nblocks = self.h.dedup_blocks(max(1, self.max_n))
        d = self.device
        if frag_map is None:
            frag_map = torch.zeros(1, dtype=torch.int32)
        # the layout argument every bucket helper takes: the destinations the
        # buckets are sized for, plus (record_layout: N>1 record exchange,
        # enable_records) the record-layout bit — smaller source buckets, so
        # that N sources' records fill one server bucket (bdedup.hip)
        self.record_layout = bool(record_layout)
        # ... record_group (N>1): the unique layout's fuller source buckets,
        # each bucket's records then grouped by the servers' sub-bucket after
        # the scatter (bdedup.hip k_rec_group; split_for_servers(m > 1))
        self.record_group = bool(record_layout and record_group)
        self.ndest = effective_ndest(frag_map, self.nranks) | (
            self.h.bd_record_layout_bit() if self.record_layout else 0) | (
            self.h.bd_record_group_bit() if self.record_group else 0)
        self.gkeys = self.gspj = None  # grouped records: the scatter's staging
        self.frag_map = frag_map.to(d, torch.int32).contiguous()
        m = max(1, self.max_n)
        if self.mode == "bucket" and m > self.h.bd_max_keys():
            # above ~45M keys per call the bucket-count cap would push more
            # than ~2800 occurrences into a bucket's 4096-slot LDS table
            log.warning("dedup: %d keys per call exceed the bucketed dedup's %d; "
                        "using the scratch-hash dedup", m, self.h.bd_max_keys())
            self.mode = "hash"
        if self.mode == "hash":
            self.skeys = torch.empty(self.scap, dtype=torch.int64, device=d)
            self._dirty = True
            self.stag = torch.empty(self.scap, dtype=torch.int32, device=d)
            self.blk_cnt = torch.empty(self.h.dedup_cnt_words(m, self.nranks),
                                       dtype=torch.int32, device=d)
            self.slot_of = torch.empty(self.max_n, dtype=torch.int32, device=d)
        else:
            # word 0 of the scratch is the sticky overflow flag (zeroed once)
            self.scratch = torch.zeros(self.h.bd_scratch_words(m, self.nranks, self.ndest),
                                       dtype=torch.int32, device=d)
            self.pj = torch.empty(m, dtype=torch.int32, device=d)      # bucket order -> j
            self.pos_of = torch.empty(m, dtype=torch.int32, device=d)  # j -> bucket order
            self.bkt = torch.empty(m, dtype=torch.int32, device=d)     # j -> bucket
            self.luid = torch.empty(m, dtype=torch.int32, device=d)    # bucket-local ids
            self.bkeys = torch.empty(m, dtype=torch.int64, device=d)   # staged unique keys
            # (key, sample) records in bucket order, 16 B each (scatter -> dedup)
            self.rec = torch.empty((m, 4), dtype=torch.int32, device=d)
            self._last_n = 0
            # SS_BD_DEBUG=1: per-bucket phase timestamps of the dedup kernel
            self.dbg = (torch.zeros(8 * self.h.bd_buckets(m, self.nranks, self.ndest),
                                    dtype=torch.int64,
                                    device=d) if os.environ.get("SS_BD_DEBUG") else None)
        self.inv = torch.empty(self.max_n, dtype=torch.int32, device=d)
        self.ukeys = torch.empty(self.nranks * self.ucap, dtype=torch.int64, device=d)
        self.ucount = torch.zeros(self.nranks, dtype=torch.int64, device=d)
        self.ugrad = (torch.empty((self.nranks * self.ucap, self.gdim), dtype=torch.float32,
                                  device=d) if with_grad else None)

    def __call__(self, keys: torch.Tensor, stream=None) -> DedupResult:
        n = keys.numel()
        if n > self.max_n:
            raise ValueError(f"dedup: {n} keys > capacity {self.max_n}")
        st = _stream_ptr(stream)
        ug = self.ugrad.data_ptr() if (self.ugrad is not None and self.zero_grad) else 0
        if self.mode == "bucket":
            self._last_n = n
            used = self.h.bd_dedup(keys.data_ptr(), n, self.frag_map.data_ptr(), self.frag_map.numel(),
                            self.nranks, self.ucap, self.scratch.data_ptr(), self.pj.data_ptr(),
                            self.pos_of.data_ptr() if self.need_pos else 0,
                            self.bkt.data_ptr() if self.need_bkt else 0,
                            self.luid.data_ptr(),
                            self.bkeys.data_ptr(), self.ucount.data_ptr(),
                            self.ukeys.data_ptr(), ug, self.gdim,
                            self.inv.data_ptr() if self.materialize_inv else 0,
                            int(self.need_ukeys or bool(ug)), st,
                            self.dbg.data_ptr() if self.dbg is not None else 0,
                            self.rec.data_ptr(),
                            self.usingle.data_ptr() if self.usingle is not None else 0,
                            self.ndest, self.lay_n or 0, self.msub,
                            self.usub.data_ptr() if self.usub is not None else 0,
                            self.rbits, self.spj.data_ptr() if self.spj is not None else 0,
                            self.gkeys.data_ptr() if self.gkeys is not None else 0,
                            self.gspj.data_ptr() if self.gspj is not None else 0)
            return DedupResult(self.ukeys, self.ucount, self.inv[:n], self.ugrad, self.ucap,
                               self.nranks, n, self, self._lay(n), int(used or 0))
        # the scratch is all-EMPTY between calls: the finish kernel resets the
        # slots its winners claimed, so no per-round 0xFF memset is needed
        if self._dirty:
            self.skeys.fill_(-1)
            self._dirty = False
        self.h.dedup_route(keys.data_ptr(), n, self.skeys.data_ptr(), self.stag.data_ptr(),
                           self.scap, self.slot_of.data_ptr(), self.frag_map.data_ptr(),
                           self.frag_map.numel(), self.nranks, self.ucap, self.ucount.data_ptr(),
                           self.ukeys.data_ptr(), ug, self.gdim,
                           self.blk_cnt.data_ptr(), self.inv.data_ptr(), st)
        return DedupResult(self.ukeys, self.ucount, self.inv[:n], self.ugrad, self.ucap,
                           self.nranks, n, self, n)

    def _lay(self, n: int) -> int:
        """Layout size of a call of n keys (what every bucket-layout helper
        takes instead of n)."""
        return max(int(self.lay_n or 0), int(n))

    def run_tables(self, Pd: int):
        """(ubase, unum) of the LAST call as int32 views of [nranks * Pd]:
        destination d's bucket runs at [d*Pd, (d+1)*Pd) — what a source
        sends each server with its keys (N>1, server.hip)."""
        if self.mode != "bucket":
            raise RuntimeError("run_tables needs mode='bucket'")
        P, _, o_un, o_ub = self.h.bd_offsets(self._lay(self._last_n), self.nranks, self.ndest)
        if P != Pd * self.nranks:
            raise RuntimeError(f"run_tables: {P} buckets, expected {Pd} x {self.nranks}")
        return self.scratch[o_ub:o_ub + P], self.scratch[o_un:o_un + P]

    def split_for_servers(self, m: int) -> None:
        """Group each bucket's unique keys by the servers' sub-bucket (one
        of ``m``, server.hip) and record the groups' offsets (bucket mode,
        N>1 engines with a fixed ``lay_n``)."""
        if m <= 1:
            self.msub, self.usub = 1, None
            return
        if self.mode != "bucket" or not self.lay_n:
            raise RuntimeError("split_for_servers needs mode='bucket' and lay_n")
        P = self.h.bd_buckets(self.lay_n, self.nranks, self.ndest)
        self.msub = int(m)
        self.usub = torch.zeros(P * self.msub, dtype=torch.int32, device=self.device)

    def sub_table(self, Pd: int) -> torch.Tensor:
        """int32 [nranks * Pd * msub]: destination d's sub-bucket offsets at
        [d*Pd*msub, (d+1)*Pd*msub) (after split_for_servers)."""
        if self.usub is None or self.usub.numel() != self.nranks * Pd * self.msub:
            raise RuntimeError("sub_table: split_for_servers(m) with this layout first")
        return self.usub

    def enable_records(self) -> None:
        """Route every occurrence instead of the unique keys (bucket mode,
        N>1 engines with a fixed ``lay_n``; sub-buckets with record_group,
        each bucket's records grouped by them): ukeys holds the
        occurrences' keys at their send-segment positions, ``spj`` their
        occurrence indices, ``ucount`` the records per destination, and the
        run tables the records per bucket (the servers dedup them)."""
        if self.mode != "bucket" or not self.lay_n or not self.record_layout or (
                self.msub != 1 and not self.record_group):
            raise RuntimeError("enable_records needs mode='bucket', lay_n and "
                               "Deduper(record_layout=True); sub-buckets only with record_group")
        if self.spj is None:
            self.spj = torch.empty(self.nranks * self.ucap, dtype=torch.int32,
                                   device=self.device)
        if self.msub > 1 and self.gkeys is None:
            self.gkeys = torch.empty(self.nranks * self.ucap, dtype=torch.int64,
                                     device=self.device)
            self.gspj = torch.empty(self.nranks * self.ucap, dtype=torch.int32,
                                    device=self.device)
        self.need_pos = True
        self.need_bkt = False
        self.materialize_inv = False

    def track_singletons(self) -> None:
        """Have the dedup flag the unique keys that occur once (bucket mode)."""
        if self.mode == "bucket" and self.usingle is None:
            self.usingle = torch.zeros(self.nranks * self.ucap, dtype=torch.uint8,
                                       device=self.device)

    def reduce(self, n: int, gs: torch.Tensor, F: int, ugrad: torch.Tensor,
               xval: Optional[torch.Tensor] = None, stream=None):
        """K7 for scalar rows, for the LAST call's partition (bucket mode):
        ugrad[uid] = sum over occurrences j of uid of gs[j // F] * xval[j]
        (per-sample gradient times feature value; no zero-fill needed)."""
        if self.mode != "bucket" or self.gdim != 1:
            raise RuntimeError("Deduper.reduce needs mode='bucket' and gdim=1")
        self.h.bd_reduce(self._lay(n), self.nranks, self.scratch.data_ptr(), self.pj.data_ptr(),
                         self.luid.data_ptr(), gs.data_ptr(),
                         xval.data_ptr() if xval is not None else 0, F, ugrad.data_ptr(),
                         _stream_ptr(stream), 0,
                         self.usingle.data_ptr() if self.usingle is not None else 0,
                         ndest=self.ndest)

    def fill_occ(self, n: int, uvals: torch.Tensor, occ: torch.Tensor, stream=None):
        """Scalar rows of the LAST call by occurrence position:
        ``occ[p] = uvals[uid]`` of the occurrence at bucket position p (0
        where it has none), so a consumer reads ``occ[pos_of[j]]``."""
        if self.mode != "bucket":
            raise RuntimeError("fill_occ needs mode='bucket'")
        self.h.bd_fill_occ(self._lay(n), self.nranks, self.scratch.data_ptr(),
                           self.luid.data_ptr(), uvals.data_ptr(), occ.data_ptr(), 0,
                           _stream_ptr(stream), self.ndest, 0)

    def index_ptrs(self, n: Optional[int] = None):
        """(pos_of, luid, bkt, ubase) device pointers of the last call: the
        kernels' BdIndex, uid(j) = ubase[bkt[j]] + luid[pos_of[j]]."""
        if self.mode != "bucket":
            raise RuntimeError("index_ptrs needs mode='bucket'")
        n = self._last_n if n is None else n
        ub = self.scratch.data_ptr() + 4 * self.h.bd_ubase_offset(max(1, self._lay(n)),
                                                                  self.nranks, self.ndest)
        return [self.pos_of.data_ptr(), self.luid.data_ptr(), self.bkt.data_ptr(), ub]

    def bucket_view(self, n: Optional[int] = None):
        """(bkeys, bstart, unum, ubase, P) of the last call: bucket b's unique
        keys are bkeys[bstart[b] : bstart[b] + unum[b]] with unique ids from
        ubase[b] (device pointers; bucket mode)."""
        if self.mode != "bucket":
            raise RuntimeError("bucket_view needs mode='bucket'")
        n = self._last_n if n is None else n
        P, o_bs, o_un, o_ub = self.h.bd_offsets(max(1, self._lay(n)), self.nranks, self.ndest)
        b0 = self.scratch.data_ptr()
        return (self.bkeys.data_ptr(), b0 + 4 * o_bs, b0 + 4 * o_un, b0 + 4 * o_ub, P)

    def check(self):
        """Raise if any bucket overflowed its LDS table (sticky; syncs).  The
        overflowing occurrences got no unique id, so their forward rows and
        gradients were dropped: the engine calls this at every check point
        (PSEngine.check: end of bench, backups, PSContext.finish)."""
        if self.mode == "bucket" and int(self.scratch[0].item()) != 0:
            raise DedupOverflowError("bucketed dedup: an LDS bucket table overflowed "
                                     "(pathological key distribution); use SS_DEDUP=hash")


class DedupOverflowError(RuntimeError):
    pass


def effective_ndest(frag_map, nranks: int) -> int:
    """Destinations the bucketed dedup sizes its buckets for: the fragment
    count over the largest per-rank fragment count (ranks hosting no shard,
    and uneven fragment maps, receive proportionally fewer / more keys),
    rounded with 5% slack so an even-ish map (1024 fragments over 3 servers)
    counts all its servers."""
    fm = np.asarray(frag_map.cpu() if isinstance(frag_map, torch.Tensor) else frag_map,
                    dtype=np.int64).reshape(-1)
    if fm.size == 0:
        return 1
    biggest = int(np.bincount(fm).max())
    return max(1, min(int(nranks), int(fm.size * 1.05 / biggest)))


class CpuDeduper:
    """Host implementation with the same output layout (CPU engine / tests)."""

    def __init__(self, max_n: int, nranks: int = 1, frag_map: Optional[torch.Tensor] = None,
                 gdim: int = 1, device=None, with_grad: bool = True, zero_grad: bool = True):
        self.max_n, self.nranks, self.gdim = int(max_n), int(nranks), int(gdim)
        self.ucap = self.max_n
        self.frag_map = (frag_map.cpu().numpy().astype(np.int64) if frag_map is not None
                         else np.zeros(1, dtype=np.int64))
        self.with_grad = with_grad

    def __call__(self, keys: torch.Tensor, stream=None) -> DedupResult:
        n = keys.numel()
        if n > self.max_n:
            raise ValueError(f"dedup: {n} keys > capacity {self.max_n}")
        uk, uc, inv = dedup_reference(keys.cpu().numpy(), self.nranks, self.frag_map, self.ucap)
        ug = (torch.zeros((self.nranks * self.ucap, self.gdim), dtype=torch.float32)
              if self.with_grad else None)
        return DedupResult(torch.from_numpy(uk.view(np.int64)), torch.from_numpy(uc),
                           torch.from_numpy(inv.astype(np.int32)), ug, self.ucap, self.nranks, n,
                           None, n)


def dedup_reference(keys, nranks: int = 1, frag_map: Optional[np.ndarray] = None,
                    ucap: Optional[int] = None):
    """Host reference: returns (ukeys [nranks*ucap] u64, ucount [nranks], inv [n]).

    Unique keys inside a destination segment are sorted ascending (the device
    kernel's order is arbitrary; compare as sets + inverse consistency)."""
    k = np.asarray(keys)
    k = k.view(np.uint64) if k.dtype == np.int64 else k.astype(np.uint64)
    n = len(k)
    ucap = ucap or max(n, 1)
    uniq, inv0 = np.unique(k, return_inverse=True)
    if nranks == 1 or frag_map is None:
        dest = np.zeros(len(uniq), dtype=np.int64)
    else:
        dest = frag_map[(fmix64(uniq) % np.uint64(len(frag_map))).astype(np.int64)].astype(
            np.int64)
    ukeys = np.full(nranks * ucap, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    ucount = np.zeros(nranks, dtype=np.int64)
    uid = np.empty(len(uniq), dtype=np.int64)
    for r in range(nranks):
        idx = np.nonzero(dest == r)[0]
        ucount[r] = len(idx)
        ukeys[r * ucap:r * ucap + len(idx)] = uniq[idx]
        uid[idx] = r * ucap + np.arange(len(idx))
    inv = uid[inv0] if n else np.zeros(0, dtype=np.int64)
    return ukeys, ucount, inv
