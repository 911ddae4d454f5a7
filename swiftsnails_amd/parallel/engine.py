"""Collective pull/push round engine (the MI355X replacement of Transfer + the
global pull/push access objects, /root/reference/src/core/parameter/
global_pull_access.h:40-120 and global_push_access.h:36-149).

A round is lockstep across ranks and split in three stages:

    route (route stream): dedup + route keys into per-rank segments (bucketed
                          LDS dedup, every rank on the same bucket layout);
                          [N>1] keys + per-bucket runs to the servers
    pull  (main stream, or the pull stream with pull-ahead): [N>1] server
                          merge of all sources' keys (ONE lookup per distinct
                          key) -> rows back
    push  (main stream) : [N>1] grads out -> server merge + ONE optimizer
                          update per distinct key

Route of step i+1 runs on its own stream while step i computes; with
pull-ahead (N>1 default; FM and word2vec at N=1) round i+1 is pulled while
round i computes (staleness exactly 1).  Route buffers are a ring of
``depth`` slots.

The device-count paths — one GPU (no exchange) and N>1 over the xGMI
mailboxes — issue each stage as ONE call into the C++ round engine
(``csrc/hip/round_engine.cpp``: stream waits, kernels, puts / waits, the
ring's events).  Host-count transports (RCCL, gloo, the CPU engine that
tests the multi-rank logic) are the ``HostRounds`` mixin
(``engine_host.py``).  Split roles (S servers + W workers) fall out of the
same code: non-server ranks own no table, non-worker ranks route an empty
key set, every rank enters every round.  The N>1 device set-up
(``engine_dist.py``) and the read-only lookup / control calls
(``engine_ctl.py``) are mixins of PSEngine.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops.dedup import CpuDeduper, DedupResult, Deduper
from ..utils.streams import current, current_raw, use_stream
from ..utils.tracing import Metrics, Tracer
from .engine_ctl import EngineControl
from .engine_dist import DeviceSetup, _ServerSlot  # noqa: F401 (re-export)
from .engine_host import HostRounds
from .router import HashFrag
from .transport import CountsHandle, LoopbackTransport, Transport

ROUTE, PULL, FREE = 0, 1, 2  # RoundEngine event kinds


@dataclass
class Routed:
    """A batch whose keys are deduplicated and routed (stage 1 of a round)."""
    dd: DedupResult
    slot: int                               # ring slot of the route buffers
    counts: Optional[CountsHandle] = None   # host-count transports: counts (async)
    ready: bool = False                     # GPU: the slot's route event is recorded
    tag: int = 0                            # hipGraph capture it was recorded in


@dataclass
class Round:
    dd: DedupResult
    uvals: torch.Tensor                   # [N*ucap, dim] pulled rows, unique-key order
    slot: int = 0
    slots: Optional[torch.Tensor] = None  # GPU world-1 path: table slots of ukeys
    scounts: Optional[np.ndarray] = None  # keys this rank sent to each server
    rcounts: Optional[np.ndarray] = None  # keys this rank received from each worker
    pushed: bool = False
    stats: dict = field(default_factory=dict)
    ready: bool = False                   # pull-ahead: the slot's pull event is recorded
    tag: int = 0
    snap: Optional[torch.Tensor] = None   # world-1: (w, h) rows as pulled (blind apply)
    snap_version: int = -1                # table.version the snapshot is valid for
    applied: bool = False                 # the model's kernel already ran K5 (fuse_apply)
    slot32: bool = False                  # world-1: `slots` holds 4-byte indices (first half)
    deferred: bool = False                # world-1 claimed pull: new keys' slots not written yet
    occ_filled: bool = False              # world-1 claimed pull also filled claim_occ
    server: Optional[object] = None       # CPU N>1: (unique keys, inverse) of the server merge
    # record exchange: this rank's own records' rows (cached, cap rows; the
    # rest stay in the vals arena) and, set by the model before the push,
    # (gs, spj, F, xval) pointers its server merge reads their gradients from
    own_vals: Optional[torch.Tensor] = None
    own_grad: Optional[tuple] = None

    @property
    def inv(self) -> torch.Tensor:
        return self.dd.inv

    @property
    def ugrad(self) -> torch.Tensor:
        return self.dd.ugrad


def _hip():
    from .._native import hip

    return hip()



class PSEngine(HostRounds, DeviceSetup, EngineControl):
    """Worker+server round engine for one rank.

    table           : this rank's shard (``HbmTable``/``HostTable``) or None when not a server
    transport       : data-plane transport (xGMI mailboxes / RCCL / gloo)
    count_transport : transport of the route-stage exchanges (host-count paths)
    pull_transport  : transport of the pulled-ahead keys/rows exchanges
    max_keys        : max key occurrences per pull on this rank (agrees across
                      ranks: it fixes the common bucket layout)
    server_ranks    : ranks that host a shard (default: all — colocated mode)
    frag_num        : number of hash fragments (reference config ``frag_num``)
    depth           : route-buffer ring depth

    A ``Round`` aliases engine-owned buffers of its ring slot: it is valid
    until that slot is routed again (``depth`` routes later).

    exchange        : what an N>1 xGMI round ships for dim-1 rows —
                      ``"unique"`` (each source's unique keys; per-unique
                      rows and gradients, the worker merges its occurrences)
                      or ``"records"`` (every occurrence: no worker dedup or
                      merge, the servers dedup and merge what they receive;
                      ``Round.uvals`` / ``ugrad`` are then per occurrence at
                      its send-segment position).  Records halve the
                      per-rank kernel work at N <= 2 but double the link
                      bytes (docs/PERFORMANCE.md): not the default.
    streams_of      : another engine of this rank whose route and server
                      streams this one reuses (two candidate engines of one
                      job that never run at the same time — bench.py's
                      exchange calibration: a process gets GPU_MAX_HW_QUEUES
                      = 4 hardware queues, and a fifth stream shares one with
                      a busy stream, serialising what should overlap:
                      records at one rank 0.98 vs 0.80 ms/step)"""

    def __init__(self, table, transport: Optional[Transport], max_keys: int, dim: int,
                 frag_num: int = 0, server_ranks: Optional[Sequence[int]] = None, device=None,
                 count_transport: Optional[Transport] = None, depth: Optional[int] = None,
                 pull_transport: Optional[Transport] = None, zero_grad: bool = True,
                 exchange: str = "unique", streams_of: Optional["PSEngine"] = None):
        self.t = transport or LoopbackTransport()
        self.ct = count_transport or self.t
        self.pt = pull_transport or self.ct
        self.rank, self.world = self.t.rank, self.t.world
        self.table, self.dim = table, int(dim)
        if device is None:
            device = table.device if table is not None else (
                torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                else torch.device("cpu"))
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.server_ranks = list(server_ranks) if server_ranks is not None else list(
            range(self.world))
        if (table is not None) != (self.rank in self.server_ranks):
            raise ValueError("a rank owns a table iff it is listed in server_ranks")
        frag_num = frag_num or max(1024, 8 * len(self.server_ranks))
        self.router = HashFrag(len(self.server_ranks), frag_num)
        self.frag_map = self.router.rank_map(self.server_ranks)
        # SS_ENGINE_GENERAL=1|rccl|xgmi runs a 1-GPU job through the N>1 path;
        # so does a 1-rank engine handed an N>1 data plane (a size-1 mailbox
        # arena or communicator)
        self.fast1 = (self.gpu and self.world == 1 and isinstance(self.t, LoopbackTransport)
                      and os.environ.get("SS_ENGINE_GENERAL", "0") == "0")
        self.dist = not self.fast1
        from .xgmi import XgmiTransport

        self.xg = self.t if isinstance(self.t, XgmiTransport) else None
        # record exchange (N>1 over the mailboxes, scalar rows): chosen by the
        # caller for a model whose compute handles per-occurrence rows
        # (SparseLRWorker; bench.py / the launcher pass SS_XCHG).  The
        # engine's dedupers (and its lookup's) take the record bucket layout
        if exchange not in ("unique", "records"):
            raise ValueError(f"exchange must be unique or records, not {exchange!r}")
        self.records = bool(exchange == "records" and self.gpu and self.dist and
                            self.xg is not None and int(dim) == 1)
        # N>1 on GPU: segment strides a multiple of 64 rows (aligned peer stores)
        self.max_keys = int(max_keys) if not (self.gpu and self.dist) else \
            -(-int(max_keys) // 64) * 64
        # ring depth 4 (measured 1.008 vs 1.018 ms/step for 3, LR on one
        # GPU); 3 when a fourth slot would take more than 1/8 of the device.
        # One GPU, scalar LR rows: 8 — the route stream then runs further
        # ahead of the main stream (bench 0.774-0.780 vs 0.785-0.794 ms/step
        # with 3584-key buckets; word2vec 0.089 vs 0.091, FM unchanged: 4);
        # N>1 keeps 4 (every slot is a set of IPC-mapped mailboxes)
        if depth is None and os.environ.get("SS_ENGINE_DEPTH") is None:
            fast = (self.gpu and self.world == 1 and isinstance(self.t, LoopbackTransport)
                    and os.environ.get("SS_ENGINE_GENERAL", "0") == "0")
            depth = 8 if fast and getattr(table, "snapshot_ok", False) else 4
            budget = torch.cuda.mem_get_info(self.device)[1] // 8 if self.gpu else 0
            while self.gpu and depth > 3 and \
                    depth * self.slot_bytes(self.world, max_keys, dim) > budget:
                depth = 4 if depth > 4 else 3
        self.depth = max(1, int(depth if depth is not None else
                                os.environ.get("SS_ENGINE_DEPTH", "4")))
        # observability: occurrences routed, unique keys exchanged,
        # distinct keys the servers merged them into, exchange payload bytes
        self.metrics = Metrics()
        self.tracer = Tracer(enabled=False)
        fm = torch.from_numpy(self.frag_map.astype(np.int32))
        dd_cls = Deduper if self.gpu else CpuDeduper
        # N>1 records, SS_REC_GROUP=1: the unique layout's source buckets,
        # each bucket's records grouped by the servers' sub-bucket after the
        # scatter (bdedup.hip k_rec_group).  Measured slower than the small
        # record buckets (3584 / N records, no sub-buckets; default): 2 ranks
        # on one GPU 2.18 vs 1.75 ms, 4 ranks 4.54 vs 3.96, 8 ranks 8.83 vs
        # 8.86 (profiles/raw/r6_rec_group_ab.txt) — the regroup's per-record
        # pos_of stores land in random order
        self.rec_group = bool(self.records and self.world > 1 and
                              os.environ.get("SS_REC_GROUP", "0") == "1")
        rl = {"record_layout": True, "record_group": self.rec_group} if self.records else {}
        self.dedupers = [dd_cls(self.max_keys, nranks=self.world, frag_map=fm, gdim=self.dim,
                                device=self.device, zero_grad=zero_grad, **rl)
                         for _ in range(self.depth)]
        N, cap, d, dev = self.world, self.max_keys, self.dim, self.device
        self.uvals = [torch.empty((N * cap, d), dtype=torch.float32, device=dev)
                      for _ in range(self.depth)]
        self.displs = [r * cap for r in range(N)]
        self.rounds, self._next_slot = 0, 0
        self.snapshot, self.pull_ahead, self.pull_stream = False, False, None
        self.capture_tag: Optional[int] = None
        self._dix = (self.device.index or 0) if self.gpu else -1
        self.native = None
        self._streams_of = streams_of
        if self.gpu:
            self.route_stream = (streams_of.route_stream if streams_of is not None
                                 else self._make_route_stream(dev))
            # + one slot past the ring: the N>1 read-only lookup's round
            # (PSEngine.lookup) never touches a ring slot the pipeline holds
            self.native = _hip().RoundEngine(self.depth + 1, self._dix)
            self._pins = [torch.zeros(2 * N, dtype=torch.int64, pin_memory=True)
                          for _ in range(self.depth)]
        # claimed pulls whose slots no kernel has written yet (pulled, merge not
        # issued): a further pull first commits them (pull A, pull B, push A,
        # push B must not claim a slot twice), and the ring slot of the last
        # claimed round, whose push a pull off the main stream waits for
        self._claimed: list = []
        self._deferred_slot: Optional[int] = None
        self.claim = False
        # set by a caller whose every pulled round is pushed through the
        # fused snapshot merge (SparseLRWorker): only its pulls claim; and
        # its occurrence-position parameter buffer, which a claimed pull
        # fills itself (k_bd_fill_occ fused into k_pull_claim_bk)
        self.claim_rounds = False
        self.claim_occ: Optional[torch.Tensor] = None
        if self.fast1:
            # pull snapshots for the blind-write apply (scalar AdaGrad rows)
            self.snapshot = bool(getattr(table, "snapshot_ok", False))
            # ... whose slot indices the pull stores as 4 bytes when the shard
            # has fewer than 2^31 slots (the fused merge reads them back):
            # 42 MB less traffic per step at the bench shape (SS_SLOT32=0: 8)
            self.slot32 = bool(self.snapshot and table.stride == 16 and table.G == 1 and
                               table.capacity < (1 << 31) and
                               os.environ.get("SS_SLOT32", "1") != "0")
            self.slots = [torch.empty(cap, dtype=torch.int64, device=dev)
                          for _ in range(self.depth)]
            self._snaps = [torch.empty((cap, 2), dtype=torch.float32, device=dev)
                           for _ in range(self.depth)] if self.snapshot else None
            if table is not None:  # the pull reads the dedup's staging: no send segment
                for dd in self.dedupers:
                    dd.need_ukeys = False
            # claimed pulls (region tables, table.hip k_pull_claim_bk): the
            # dedup buckets whole table regions, the bucket's pull claims new
            # keys' slots in LDS (no device-scope CAS, nothing written), and
            # the fused merge stores [w | h | key] per slot (SS_CLAIM=0: off)
            self.claim = bool(self.slot32 and getattr(table, "rbits", 0) and
                              os.environ.get("SS_CLAIM", "1") != "0")
            if self.claim:
                for dd in self.dedupers:
                    if getattr(dd, "mode", None) == "bucket":
                        dd.rbits = table.rbits
        elif self.gpu:
            self._init_dist_gpu()
        else:
            self.rkeys = torch.empty(N * cap, dtype=torch.int64)
            self.rvals = torch.zeros((N * cap, d), dtype=torch.float32)
            self.rgrads = torch.empty((N * cap, d), dtype=torch.float32)
        self._streams_of = None  # the streams are taken; keep no reference to that engine
        # pull-ahead (SURVEY X3 bounded staleness): rounds i+1 .. i+L are
        # pulled on the pull stream while round i computes, L = SS_STALENESS
        # (default 1; at most depth - 2: rounds i .. i+L pulled or pulling and
        # i+L+1 routing fill the ring); a pulled-ahead round misses at most
        # L rounds' updates (its pull waits for the push L+1 rounds back).
        # SS_STALENESS=ring: one round ahead, bounded by the ring depth only;
        # SS_STALENESS=0: synchronous rounds always.  Models opt in (FM,
        # word2vec: enable_pull_ahead); sparse LR runs synchronous rounds
        # (the servers' snapshot blind-store update) unless the bench /
        # launcher calibration (SS_PULL_AHEAD=auto, PipelinedWorker.
        # calibrate_pull_ahead) measures pull-ahead faster on the live world.
        # SS_PULL_AHEAD=1 / 0 forces it on / off for every model at N>1
        st_env = os.environ.get("SS_STALENESS", "1")
        ring = st_env == "ring"
        k = 1 if ring else max(0, int(st_env))
        self.lookahead = max(1, min(k, self.depth - 2)) if k > 0 else 0
        self.staleness = 0 if ring else self.lookahead  # bound the pull waits for
        if self.dist and self.depth >= 3 and self.lookahead > 0 and \
                os.environ.get("SS_PULL_AHEAD", "auto") == "1":
            self.pull_ahead = True
            if self.gpu and not self.shared_device:
                self.pull_stream = torch.cuda.Stream(device=self.device)

    def _make_route_stream(self, dev) -> torch.cuda.Stream:
        """The route stream; SS_ROUTE_CUS=n: restricted to n of the device's
        CUs (a CU-masked HIP stream), so the dedup's large workgroups leave
        the remaining CUs to the main stream's latency-bound table kernels."""
        n = int(os.environ.get("SS_ROUTE_CUS", "0") or 0)
        if n <= 0:
            return torch.cuda.Stream(device=dev)
        ptr = _hip().cu_stream(dev.index or 0, n, 0)
        return torch.cuda.ExternalStream(ptr, device=dev)

    def last_route_matches(self) -> bool:
        """The last routed round ran the keys-in as a route issued now would
        (N>1 xGMI: on the route stream for synchronous rounds with
        SS_SRV_AHEAD, else in the pull); a hipGraph capture must start from
        such a round (PipelinedWorker.enable_graph)."""
        last = getattr(self, "_route_srv", None)
        return last is None or last == (getattr(self, "srv_ahead", False) and not self.pull_ahead)

    @property
    def shared_device(self) -> bool:
        """Several ranks of this job run on this rank's GPU (one-GPU
        rehearsals of an N-rank job).  Their processes' streams then share
        the device's hardware queues: 8 processes x 3 streams measured
        2.5x slower than x 2 (HWS oversubscription; GPU_MAX_HW_QUEUES=2
        restores it), so a pulled-ahead round then runs on the route stream
        instead of a third stream of its own."""
        xg = getattr(self, "xg", None)
        return bool(xg is not None and getattr(xg, "devices", self.world) < self.world)

    @staticmethod
    def slot_bytes(world: int, max_keys: int, dim: int) -> int:
        """Device bytes of one route-ring slot (pulled rows, send keys +
        gradient rows + dedup scratch, and for N>1 the server merge)."""
        rows = world * max_keys
        return rows * (4 * dim + 8 + 4 * dim + (32 if world > 1 else 0)) + 40 * max_keys

    # ------------------------------------------------------------ plumbing
    def main_stream(self) -> torch.cuda.Stream:
        return current(self._dix)

    def raw_stream(self) -> int:
        """hipStream_t of the caller's current stream on this engine's device
        (0 on the CPU engine)."""
        return current_raw(self._dix) if self.gpu else 0

    @property
    def _tag(self) -> int:
        return self.capture_tag or 0

    def _wait_ev(self, kind: int, obj, stream: int) -> None:
        """``stream`` waits for the object's route / pull event if it was
        recorded in the current capture (eager: eagerly); an event of an
        earlier capture or of the eager priming has completed already."""
        if obj.ready:
            self.native.wait(kind, obj.slot, stream, self._tag)

    def _release(self, slot: int) -> None:
        if self.gpu:
            self.native.record(FREE, slot, self.raw_stream(), self._tag)

    def trace(self, name: str, stream=None):
        """A tracer phase range (roctx + host and device time); a no-op when
        the tracer is off and inside a hipGraph capture."""
        t = self.tracer
        if not t.enabled or self.capture_tag is not None:
            return contextlib.nullcontext()
        return t.gpu_range(name, stream) if self.gpu else t.range(name)

    # ------------------------------------------------------------ stage 1
    def route(self, keys: Optional[torch.Tensor] = None, produce=None, post=None) -> Routed:
        """Dedup + route a batch on the route stream (non-blocking on GPU):
        ``keys`` produced on the current stream, or ``produce(stream)``
        writing them on the route stream; ``post(dd, slot, stream_ptr)`` runs
        right after the dedup (planning that depends on the key layout)."""
        slot = self._next_slot
        self._next_slot = (slot + 1) % self.depth
        dd_fn = self.dedupers[slot]
        if not self.gpu:
            with self.trace("route"):
                keys = (produce(None) if produce is not None else keys).reshape(-1)
                dd = dd_fn(keys.to(self.device))
                return Routed(dd, slot, self.ct.exchange_counts_async(dd.ucount))
        rs, tag = self.route_stream, self._tag
        # the previous user of this slot is done (same capture only)
        self.native.wait(FREE, slot, rs.cuda_stream, tag)
        if keys is not None and self.capture_tag is None:
            rs.wait_stream(self.main_stream())  # keys were produced on the main stream
        with use_stream(rs), self.trace("route", rs):
            keys = (produce(rs) if produce is not None else keys).reshape(-1)
            if keys.device != self.device:
                keys = keys.to(self.device)
            dd = dd_fn(keys, stream=rs)
            if post is not None:
                post(dd, slot, rs.cuda_stream)
            counts = None
            if self.xg:
                ub, un = dd.owner.run_tables(self.Pd)
                us = dd.owner.sub_table(self.Pd).data_ptr() if dd.owner.msub > 1 else 0
                # synchronous rounds: the keys in + the server's distinct-key
                # merge on the route stream, a round ahead, off the main
                # stream's chain (SS_SRV_AHEAD=0: at the head of the pull).
                # Pulled-ahead rounds keep them in the pull, already off the
                # main stream (on the route stream they lengthened its chain:
                # word2vec N>1 0.107 -> 0.117 ms/step)
                tab = self.table is not None
                ahead = self.srv_ahead and not self.pull_ahead
                self._route_srv = ahead
                self.native.route_end(slot, tag, rs.cuda_stream, dd.ukeys.data_ptr(),
                                      dd.ucount.data_ptr(), ub.data_ptr(), un.data_ptr(), us,
                                      ahead, tab, self.rkeys[slot].data_ptr(),
                                      self.rmeta[slot][0].data_ptr(),
                                      self.rmeta[slot][1].data_ptr(),
                                      self.srv_err.data_ptr() if tab else 0)
            else:
                if self.dist:
                    counts = self._route_counts(dd, slot, rs)
                self.native.record(ROUTE, slot, rs.cuda_stream, tag)
        return Routed(dd, slot, counts, True, tag)

    # ------------------------------------------------------------ stage 2
    def pull(self, keys_or_routed) -> Round:
        r = keys_or_routed if isinstance(keys_or_routed, Routed) else self.route(keys_or_routed)
        with self.trace("pull"):
            if self.gpu:
                self._wait_ev(ROUTE, r, self.raw_stream())
            return self._pull_stage(r, self.uvals[r.slot], self.raw_stream() if self.gpu else None,
                                    ahead=False)

    def pull_ahead_round(self, r: Routed) -> Round:
        """Stage 2 on the pull (or route) stream (pull-ahead): the Round's
        rows are ready at its pull event; ``begin(rnd)`` makes the main
        stream wait for them.  The CPU engine pulls right away (the same
        collective order: round i+L's pull before round i's push)."""
        if not self.gpu:
            with self.trace("pull"):
                return self._pull_stage(r, self.uvals[r.slot], None, ahead=True)
        ps = self.pull_stream or self.route_stream
        st = ps.cuda_stream
        if ps is not self.route_stream:
            self._wait_ev(ROUTE, r, st)
        if self._claimed:  # committed on the main stream, after their pulls
            self._commit_claimed(self.raw_stream())
            ps.wait_stream(self.main_stream())
        if self._deferred_slot is not None:
            # the table holds the last claimed pull's new keys only after that
            # round's push: a pull off the main stream waits for it
            self.native.wait(FREE, self._deferred_slot, st, self._tag)
            self._deferred_slot = None
        # staleness bound: round i+1 waits for round i-1's push (k slots back)
        k = self.staleness
        if 0 < k < self.depth - 1:
            self.native.wait(FREE, (r.slot - k - 1) % self.depth, st, self._tag)
        with use_stream(ps), self.trace("pull", ps):
            rnd = self._pull_stage(r, self.uvals[r.slot], st, ahead=True)
            if not rnd.ready:
                self.native.record(PULL, r.slot, st, self._tag)
        rnd.ready, rnd.tag = True, self._tag
        return rnd

    def _pull_stage(self, r: Routed, uv: torch.Tensor, st, ahead: bool) -> Round:
        """The pull of a routed round on stream ``st`` (its waits done);
        a returned Round with ``ready`` set has its pull event recorded."""
        dd, slot, tab = r.dd, r.slot, self.table
        if self.fast1:
            self._commit_claimed(st)
            own = dd.owner
            snap = (self._snaps[slot] if (not ahead and self.snapshot and tab.snapshot_ok)
                    else None)
            native = getattr(own, "mode", None) == "bucket" and not tab.custom_pull
            s32 = claim = False
            if native:
                v = own.bucket_view(dd.n)
                s32 = self.slot32 and snap is not None
                # a claimed pull: synchronous rounds only (the table is written
                # by this round's merge, before the next pull on this stream)
                claim = bool(s32 and self.claim and self.claim_rounds and dd.rbits and
                             dd.rbits == tab.rbits)
                occ = self.claim_occ if claim else None
                self.native.pull_fast(slot, self._tag, st, False, -1, ahead, tab.dt,
                                      tab._init_native, tab.size_ctr.data_ptr(),
                                      tab.err.data_ptr(), tab.G, list(v[:4]), v[4], uv.data_ptr(),
                                      self.slots[slot].data_ptr(),
                                      snap.data_ptr() if snap is not None else 0, int(s32), claim,
                                      own.luid.data_ptr() if occ is not None else 0,
                                      occ.data_ptr() if occ is not None else 0)
                if claim:
                    self._deferred_slot = slot
            elif getattr(own, "mode", None) == "bucket":
                tab.pull_buckets(own.bucket_view(dd.n), uv, self.slots[slot], stream=st, snap=snap)
            else:
                tab.pull(dd.ukeys, insert=True, unique=True, out=uv, slots=self.slots[slot],
                         segs=tab.dev_segs(dd.ucount), max_n=max(1, min(dd.n, dd.ucap)), stream=st)
            if tab.custom_pull:  # user init / pull methods (tensor code; syncs)
                tab.finish_pull(self.slots[slot], uv, n=dd.ucount)
            self.metrics.add(occurrences=dd.n)
            rnd = Round(dd, uv, slot, slots=self.slots[slot], snap=snap,
                        snap_version=tab.version, ready=native and ahead, tag=self._tag,
                        slot32=native and s32, deferred=claim,
                        occ_filled=bool(claim and self.claim_occ is not None))
            if claim:
                self._claimed.append(rnd)
            return rnd
        if not (self.xg and self.gpu):
            return self._pull_counts(r, uv, self.pt if ahead else self.t, st)
        # N>1 over the mailboxes: one call (keys wait, server merge + lookup,
        # rows back, counters); a tensor-code pull hook splits it in two
        S = self.srv[slot] if self.srv is not None else None
        if S is not None:
            S.snap_valid = S.snap is not None and not self.pull_ahead and tab.snapshot_ok
        acc = self.metrics.device_block(("unique_sent", "unique_recv", "a2a_bytes"), self.device)
        sx = self.metrics.device_block(("server_unique",), self.device) if S is not None else None
        m = [acc.data_ptr(), S.ucount.data_ptr() if S else 0, sx.data_ptr() if S else 0]
        custom = S is not None and tab.custom_pull
        # a claimed server pull (sync snapshot rounds, region buckets): its
        # merge in this round's push stores the new keys' slots
        claim = bool(S is not None and S.snap_valid and not custom and self.claim and
                     self.claim_rounds and dd.rbits and dd.rbits == tab.rbits)
        if claim:
            self._deferred_slot = slot
        svals = self.svals.data_ptr() if S is not None else 0
        ss = self._srv_stream(custom)
        ov = self.own_vals[slot] if getattr(self, "own_vals", None) is not None else None
        self.native.pull_xgmi(slot, self._tag, st, False, -1, ahead and not custom, S is not None,
                              tab.dt if S else self._nodt, tab._init_native if S else self._noip,
                              tab.size_ctr.data_ptr() if S else 0, tab.err.data_ptr() if S else 0,
                              tab.G if S else 1, self.rkeys[slot].data_ptr(),
                              self.rmeta[slot][0].data_ptr(), self.rmeta[slot][1].data_ptr(),
                              self.srv_err.data_ptr() if S else 0, svals,
                              self.rvals.data_ptr(), bool(S and S.snap_valid),
                              dd.ucount.data_ptr(), m, custom, claim, True, ss,
                              ov.data_ptr() if ov is not None else 0)
        if custom:
            tab.finish_pull(S.slots, self.svals, n=S.ucount)
            self.native.pull_xgmi_finish(slot, self._tag, st, ahead, svals, self.rvals.data_ptr(),
                                         dd.ucount.data_ptr(), m)
        self.metrics.add(occurrences=dd.n)
        return Round(dd, self.uvals[slot], slot, ready=ahead, tag=self._tag, own_vals=ov)

    def enable_pull_ahead(self, on: bool = True, pull_stream: bool = False,
                          force: bool = False) -> bool:
        """Opt into pull-ahead (staleness ``lookahead``) where supported.
        ``pull_stream`` (one GPU; SS_PULL_STREAM=0/1 overrides): the lookup
        on its own stream instead of behind the dedup on the route stream —
        pays when it would hold up the next dedup (word2vec 0.128 -> 0.125
        ms/step), not when the main stream is the longer one (FM 0.655 ->
        0.685).  N>1 always pulls on its own stream.  ``force``: the
        calibration's switch (ignores SS_PULL_AHEAD=auto's model default).
        Switching off takes effect for the next pull; rounds already pulled
        drain (PipelinedWorker.set_pull_ahead)."""
        env = os.environ.get("SS_PULL_AHEAD", "auto")
        if on and (self.gpu or self.dist) and self.depth >= 3 and self.lookahead > 0 and \
                (env != "0" or force):
            self.pull_ahead = True
            want = os.environ.get("SS_PULL_STREAM", "1" if pull_stream else "0") != "0"
            if self.gpu and self.pull_stream is None and (self.dist or want) and \
                    not self.shared_device:
                self.pull_stream = torch.cuda.Stream(device=self.device)
        elif not on:
            self.pull_ahead = False
        return self.pull_ahead

    def begin(self, rnd: Round) -> None:
        if self.gpu:
            self._wait_ev(PULL, rnd, self.raw_stream())

    # ------------------------------------------------------------ stage 3
    def _server_update_kind(self) -> Optional[str]:
        """How the server merge applies the update: fused into the merge for
        scalar AdaGrad rows ("scalar") and for wider rows ("rows": lane c of
        a key's lane group updates coordinate c); None: merged rows first,
        then the apply kernel (other scalar rules) or a tensor-code rule."""
        tab = self.table
        if tab is None or tab.push_fn is not None:
            return None
        if self.dim > 1:
            return "rows"
        if (tab.opt.kind == "adagrad" and tab.width == 2 and tab.G == 1 and
                not getattr(tab, "bf16", False)):
            return "scalar"
        return None

    def _srv_stream(self, host_side: bool) -> int:
        """hipStream_t of the server stream for this stage, 0 for none.  A
        stage with tensor-code hooks (a user pull method, a merged-rows push
        the caller applies) runs on the caller's stream; the server stream is
        then retired for good (the main stream first waits for it), so no
        server update can reorder against a lookup."""
        ss = getattr(self, "server_stream", None)
        if ss is None:
            return 0
        if host_side:
            torch.cuda.current_stream(self.device).wait_stream(ss)
            self.server_stream = None
            return 0
        return ss.cuda_stream

    def fuse_apply(self, rnd: Round, snapshot: bool = True) -> Optional[dict]:
        """Arguments that let a model's gradient-merge kernel run the optimizer
        update itself (``bd_reduce(..., **args)`` / ``bd_reduce_fm``), or
        None.  One GPU; ``snapshot``: scalar AdaGrad rows from the pull's
        still-valid (w, h) snapshot (blind store).  Marks the round applied."""
        tab = self.table
        if not (self.fast1 and not rnd.applied and rnd.slots is not None
                and getattr(tab, "push_fn", None) is None):
            return None
        if snapshot and not (rnd.snap is not None and rnd.snap_version == tab.version):
            return None
        if rnd.deferred and not snapshot:
            return None  # a claimed pull is committed by the snapshot merge only
        rnd.applied = True
        tab.version += 1
        args = {"t": tab.dt, "slots": rnd.slots.data_ptr(), "op": tab.opt.native(),
                "slot32": int(rnd.slot32)}
        if snapshot:
            args["snap"] = rnd.snap.data_ptr()
        if rnd.deferred:  # the merge stores whole [w | h | key] slots
            args["bkeys"] = rnd.dd.owner.bkeys.data_ptr()
            self._claimed = [x for x in self._claimed if x is not rnd]
            rnd.deferred = False
        return args

    def _commit(self, rnd: Round, stream: Optional[int] = None) -> None:
        """Write the keys (and the initial rows, i.e. its snapshot) of a
        claimed pull that no fused merge committed — its snapshot went stale
        before the push, or another pull comes first (k_commit_claims)."""
        if not rnd.deferred:
            return
        v = rnd.dd.owner.bucket_view(rnd.dd.n)
        _hip().commit_claims(self.table.dt, v[0], v[1], v[2], v[3], v[4], rnd.slots.data_ptr(),
                             rnd.snap.data_ptr(),
                             self.raw_stream() if stream is None else stream,
                             self.table.err.data_ptr())
        rnd.deferred = False
        self._claimed = [x for x in self._claimed if x is not rnd]

    def _commit_claimed(self, stream) -> None:
        for rnd in list(self._claimed):
            self._commit(rnd, stream)

    def push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        with self.trace("push"):
            self._push(rnd, grads)

    def _push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        g = rnd.ugrad if grads is None else grads
        tab, slot = self.table, rnd.slot
        if self.fast1:
            if not rnd.applied:
                self._commit(rnd)
            if not rnd.applied and tab.push_fn is not None:
                n = int(rnd.dd.ucount.sum())  # a tensor rule: host-sized (syncs)
                sl = rnd.slots
                if rnd.slot32:  # the pull stored 4-byte slot indices
                    sl = sl.view(torch.int32)[:sl.numel()].to(torch.int64)
                tab.apply_custom(sl[:n], g[:n])
                self._release(slot)
            else:
                apply = not rnd.applied
                snap = rnd.snap if (apply and rnd.snap is not None and
                                    rnd.snap_version == tab.version) else None
                if apply:
                    tab.version += 1
                # a 4-byte-slot pull: the apply kernel reads them as such
                self.native.push_fast(slot, self._tag, self.raw_stream(), apply, tab.dt,
                                      tab.opt.native(), tab.G, rnd.slots.data_ptr(), g.data_ptr(),
                                      rnd.dd.ucount.data_ptr(),
                                      max(1, min(rnd.dd.n, rnd.dd.ucap)),
                                      snap.data_ptr() if snap is not None else 0,
                                      int(bool(rnd.slot32)))
            tab.next_round()
        elif self.xg and self.gpu:
            kind = self._server_update_kind()
            S = self.srv[slot] if self.srv is not None else None
            merged_only = S is not None and kind is None
            ss = self._srv_stream(merged_only)
            self.native.push_xgmi(slot, self._tag, self.raw_stream(), g.data_ptr(),
                                  rnd.dd.ucount.data_ptr(), S is not None, kind is not None,
                                  tab.dt if S else self._nodt, tab.opt.native() if S else self._noop,
                                  self.rgrads[slot].data_ptr(), kind == "scalar",
                                  bool(S and S.snap_valid),
                                  self.sgrad.data_ptr() if merged_only else 0, not merged_only,
                                  ss, self.gstage.data_ptr()
                                  if S is not None and getattr(self, "gstage", None) is not None
                                  else 0, list(rnd.own_grad) if rnd.own_grad and S is not None
                                  else [])
            if merged_only:
                self._apply_merged(slot)
                self._release(slot)
            if tab is not None:
                tab.version += 1
                tab.next_round()
        else:
            self._push_counts(rnd, g)
            if tab is not None:
                tab.next_round()
            self._release(slot)
        rnd.pushed = True
        self.rounds += 1
