"""Collective pull/push round engine (the MI355X replacement of Transfer + the
global pull/push access objects).

Reference call stacks being replaced:

* ``GlobalPullAccess::pull_with_barrier``
  (/root/reference/src/core/parameter/global_pull_access.h:40-120): group keys
  per server, one ``WORKER_PULL_REQUEST`` per server, server
  ``get_pull_value`` per key (server/init.h:48-72), callback writes the
  worker cache and resets grads, ``StateBarrier`` counts responses.
* ``GlobalPushAccess::push_with_barrier`` (global_push_access.h:36-149):
  group (key, grad) per server, server ``apply_push_value`` (server/init.h:115-149).

A round is lockstep across ranks and split in three stages:

    route (route stream): dedup + route keys into per-rank segments (bucketed
                          LDS dedup); [N>1] counts all-to-all + async D2H
    pull  (main stream, or the pull stream with pull-ahead): [N>1] wait
                          counts; keys a2av -> server probe/init/gather ->
                          values a2av back
    push  (main stream) : grads a2av -> server apply, one launch per source
                          rank in rank order (duplicate keys never race)

``route`` of step i+1 is enqueued before ``pull`` of step i, on its own HIP
stream and its own RCCL communicator, so key generation, dedup and the count
exchange overlap the previous step's compute, and the one host
synchronisation per round (the counts RCCL needs on the host) is already
satisfied when ``pull`` asks for it.  With pull-ahead (N>1 default; FM and
word2vec at N=1) round i+1 is pulled on a third stream and communicator
while round i computes (staleness 1).  Route buffers are a ring of depth 4.
On one GPU (world 1) no host synchronisation happens at all: the unique-key
count stays on the device and every kernel reads it there; scalar AdaGrad
rows are snapshotted by the pull and updated inside the model's gradient
merge (``fuse_apply``).

Split roles (S servers + W workers) fall out of the same code: non-server
ranks own no table and receive nothing (the router never maps to them);
non-worker ranks route an empty key set — every rank still enters the
collectives, which is what makes the round lockstep.

The same engine runs on CPU (``HostTable`` shards, host dedup, gloo
transport) — that is how the multi-rank logic is tested without GPUs.
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
from ..utils.tracing import Tracer
from .router import HashFrag
from .transport import CountsHandle, LoopbackTransport, Transport


@dataclass
class Routed:
    """A batch whose keys are deduplicated and routed (stage 1 of a round)."""
    dd: DedupResult
    slot: int                               # ring slot of the route buffers
    counts: Optional[CountsHandle] = None   # N>1: host counts (async)
    ready: Optional[torch.cuda.Event] = None  # route-stream completion (GPU)
    tag: Optional[int] = None               # hipGraph capture the event belongs to


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
    ready: Optional[object] = None        # pull-ahead: route-stream event of the pulled rows
    tag: Optional[int] = None             # hipGraph capture of `ready`
    snap: Optional[torch.Tensor] = None   # world-1: (w, h) rows as pulled (blind apply)
    snap_version: int = -1                # table.version the snapshot is valid for
    applied: bool = False                 # the model's kernel already ran K5 (fuse_apply)
    occ_filled: bool = False              # the pull also wrote the occurrence parameters

    @property
    def inv(self) -> torch.Tensor:
        return self.dd.inv

    @property
    def ugrad(self) -> torch.Tensor:
        return self.dd.ugrad


def _hip():
    from .._native import hip

    return hip()


def _stream():
    return current_raw()


class PSEngine:
    """Worker+server round engine for one rank.

    table           : this rank's shard (``HbmTable``/``HostTable``) or None when not a server
    transport       : data-plane transport (RCCL on MI355X)
    count_transport : transport for the route-stage count exchange (a second
                      RCCL communicator on GPU; defaults to ``transport``)
    max_keys        : max key occurrences per pull on this rank
    server_ranks    : ranks that host a shard (default: all — colocated mode)
    frag_num        : number of hash fragments (reference config ``frag_num``)
    depth           : route-buffer ring depth (2 = one batch of lookahead)

    A ``Round`` aliases engine-owned buffers of its ring slot: it is valid
    until that slot is routed again (``depth`` routes later).
    """

    def __init__(self, table, transport: Optional[Transport], max_keys: int, dim: int,
                 frag_num: int = 0, server_ranks: Optional[Sequence[int]] = None, device=None,
                 count_transport: Optional[Transport] = None, depth: Optional[int] = None,
                 pull_transport: Optional[Transport] = None,
                 zero_grad: bool = True):
        self.t = transport or LoopbackTransport()
        self.ct = count_transport or self.t
        # pull-ahead collectives get their own communicator (one stream per
        # communicator: RCCL operations of one communicator must not run
        # concurrently on two streams)
        self.pt = pull_transport or self.ct
        self.rank, self.world = self.t.rank, self.t.world
        self.table = table
        self.dim = int(dim)
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
        self.max_keys = int(max_keys)
        # ring depth 4 by default: with one batch of lookahead, routing round
        # i+1 reuses the buffers of round i-3 (long pushed) instead of waiting
        # on round i-1's push (a cross-queue event on the critical path); 3 is
        # the minimum for pull-ahead, 4 measured 1.008 vs 1.018 ms/step (LR,
        # one GPU).  Every slot holds N*max_keys-row buffers (slot_bytes), so
        # the default drops to 3 when a fourth slot would take more than 1/8
        # of the device's memory (wide rows at large N)
        if depth is None and os.environ.get("SS_ENGINE_DEPTH") is None:
            depth = 4
            # (HIP's total memory: torch's device-property query can read a
            # device count of 0 off the main thread, where the in-process
            # rehearsal builds its engines)
            if self.gpu and 4 * self.slot_bytes(self.world, max_keys, dim) > \
                    torch.cuda.mem_get_info(self.device)[1] // 8:
                depth = 3
        self.depth = max(1, int(depth if depth is not None else
                                os.environ.get("SS_ENGINE_DEPTH", "4")))
        dd_cls = Deduper if self.gpu else CpuDeduper
        fm = torch.from_numpy(self.frag_map.astype(np.int32))
        self.dedupers = [dd_cls(self.max_keys, nranks=self.world, frag_map=fm, gdim=self.dim,
                                device=self.device, zero_grad=zero_grad) for _ in range(self.depth)]
        N, cap, d = self.world, self.max_keys, self.dim
        dev = self.device
        self.uvals = [torch.empty((N * cap, d), dtype=torch.float32, device=dev)
                      for _ in range(self.depth)]
        # observability: occurrences routed, unique keys exchanged,
        # alltoallv payload bytes (host-known counts; world-1 keeps counts on
        # the device and only counts occurrences)
        from ..utils.tracing import Metrics

        self.metrics = Metrics()
        # per-phase roctx ranges + HIP-event device times (route / pull /
        # push, and the model's compute); a disabled tracer unless the job
        # sets `trace: 1` (framework/gpu.py hands its tracer over)
        self.tracer = Tracer(enabled=False)
        # SS_ENGINE_GENERAL=1 runs a 1-GPU job through the N>1 code path
        # (send segments, count exchange, server-side segment pull/apply): the
        # per-rank cost of the multi-GPU pipeline without the network
        self.fast1 = (self.gpu and self.world == 1 and
                      os.environ.get("SS_ENGINE_GENERAL", "0") == "0")
        if self.fast1:
            self.slots = [torch.empty(cap, dtype=torch.int64, device=dev)
                          for _ in range(self.depth)]
            # pull snapshots for the blind-write apply (scalar AdaGrad rows,
            # pull and push of a round adjacent in table order: Round.snap);
            # SS_PULL_SNAPSHOT=0 turns them off
            self.snapshot = (os.environ.get("SS_PULL_SNAPSHOT", "1") != "0" and
                             getattr(table, "snapshot_ok", False))
            self._snaps = [torch.empty((cap, 2), dtype=torch.float32, device=dev)
                           if self.snapshot else None for _ in range(self.depth)]
            # SS_FUSE_APPLY=0: the model's merge kernel writes ugrad and
            # k_apply runs separately even when fuse_apply() could fuse them
            self.fuse_apply_on = os.environ.get("SS_FUSE_APPLY", "1") != "0"
            # the colocated pull reads the bucketed dedup's staging directly:
            # no contiguous send segment is needed
            if table is not None and table.insert_mode == "cas":
                for dd in self.dedupers:
                    dd.need_ukeys = False
        else:
            # server-side receive buffers: one fixed segment per source rank.
            # rslots must survive from pull to push of the same round -> ring.
            self.rkeys = torch.empty(N * cap, dtype=torch.int64, device=dev)
            self.rvals = torch.zeros((N * cap, d), dtype=torch.float32, device=dev)
            self.rgrads = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
            if self.gpu:
                self.rslots = [torch.empty(N * cap, dtype=torch.int64, device=dev)
                               for _ in range(self.depth)]
        if self.gpu:
            # SS_ROUTE_PRIORITY=1 gives the route chain (data -> dedup -> counts)
            # dispatch priority; measured no gain on 1 GPU (186 vs 189 M/s), off
            prio = -1 if os.environ.get("SS_ROUTE_PRIORITY", "0") != "0" else 0
            self.route_stream = torch.cuda.Stream(device=dev, priority=prio)
            # SS_ROUTE_CUS=k: the route stream's kernels may use only k CUs (a
            # CU-masked stream), leaving the memory system to the main stream's
            # critical chain while the route stage, which has slack, runs longer.
            # Measured slower for every k (0.97 -> 1.17-1.20 ms/step): off
            route_cus = int(os.environ.get("SS_ROUTE_CUS", "0") or 0)
            if route_cus > 0:
                ptr = _hip().cu_mask_stream(dev.index or 0, route_cus)
                self.route_stream = torch.cuda.ExternalStream(ptr, device=dev)
            self._free = [None] * self.depth  # main-stream event: slot buffers released
            self._free_tag = [None] * self.depth
            self._pins = [torch.zeros(2 * N, dtype=torch.int64, pin_memory=True)
                          for _ in range(self.depth)]
        self.displs = [r * cap for r in range(N)]
        self.rounds = 0
        self._next_slot = 0
        # pull-ahead (N>1 on GPU): round i+1's pull (keys a2av, server lookup,
        # rows a2av) runs on the route stream with the count communicator
        # while round i computes and pushes on the main stream — bounded
        # staleness 1, the asynchronous-PS semantics of the reference
        # (SURVEY X3).  Needs ring depth >= 3 (rounds i, i+1, i+2 in flight).
        self.pull_ahead = (self.gpu and not self.fast1 and self.depth >= 3 and
                           os.environ.get("SS_PULL_AHEAD", "1") != "0")
        # on one GPU pull-ahead moves the table lookup onto the route stream;
        # a model whose route stream is light (FM, word2vec) opts in with
        # enable_pull_ahead(), sparse LR (route stream already the longer one)
        # does not
        # a third stream for the pulled-ahead round: its collectives wait on the
        # network while the route stream dedups and the main stream computes
        self.pull_stream = (torch.cuda.Stream(device=self.device)
                            if self.pull_ahead and self.pt is not self.ct else None)
        # pull-ahead staleness bound (_bound_staleness): a pulled-ahead round
        # misses at most this many rounds' updates; SS_STALENESS=ring: only the
        # ring depth bounds it
        st_env = os.environ.get("SS_STALENESS", "1")
        self.staleness = 0 if st_env == "ring" else max(1, int(st_env))
        # device index for the cheap current-stream lookups (utils/streams.py)
        # and per-slot events, reused round after round (a slot's event is
        # re-recorded only after the waits on its previous record were enqueued)
        self._dix = (self.device.index or 0) if self.gpu else -1
        if self.gpu:
            self._ev_route = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_pull = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_free = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_grad = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_gate = [torch.cuda.Event() for _ in range(self.depth)]
        # gate_next_pull(): the next pulled-ahead round waits for this event
        self._pull_gate = None
        # push on the pull stream (N>1 with a pull stream, SS_PUSH_STREAM=pull):
        # round i's gradient all-to-all-v and server apply are enqueued on the
        # pull stream right behind round i+1's pull (the worker calls
        # pull_ahead_round(i+1) before push(i)).  The main stream is then left
        # with the model's forward + merge, the pull stream carries lookup +
        # apply, and pull(i+2) still sees apply(i) (same stream): the same
        # staleness-1 schedule with the apply off the compute chain.  Measured
        # (N>1 path on one GPU, three A/B pairs) 1.049-1.053 -> 1.058-1.103
        # ms/step: every stream shares the chip's memory system, and the route
        # stream's dedup, which the next pull waits for, stays the chain; off
        self.push_on_pull = (self.pull_stream is not None and
                             os.environ.get("SS_PUSH_STREAM", "main") == "pull")
        # occurrence-space unique ids (enable_osi): the model indexes rows
        # with the dedup's own inverse (bstart[b] + l), see ops/dedup.py
        self.osi = False
        # occ_buf (set by a model, one GPU): the bucketed snapshot pull also
        # writes each occurrence's parameter at its bucket position into it
        # (table.pull_buckets(occ=), fused with Deduper.fill_occ)
        self.occ_buf: Optional[torch.Tensor] = None
        # hipGraph capture in progress (models/base.py enable_graph): an id
        # per captured step.  Inside a capture the route stream forks from the
        # capturing stream, and events of other captures are not waited on —
        # graph replays run one after the other, so what they order is done
        self.capture_tag: Optional[int] = None

    @staticmethod
    def slot_bytes(world: int, max_keys: int, dim: int) -> int:
        """Device bytes of one route-ring slot: pulled rows, the deduper's
        send keys + gradient rows (+ its ~40 B/key scratch) and, for N>1,
        the resolved server slots — each sized ``world * max_keys`` rows
        (a destination segment must hold every unique key of a batch).
        At N=8 and 10.2M keys per batch: 2.4 GB for LR rows (dim 1), 7.6 GB
        for FM rows (dim 9)."""
        rows = world * max_keys
        return rows * (4 * dim + 8 + 4 * dim + (8 if world > 1 else 0)) + 40 * max_keys

    def _wait(self, stream, ev, tag) -> None:
        if ev is not None and tag == self.capture_tag:
            stream.wait_event(ev)

    def main_stream(self) -> torch.cuda.Stream:
        """The caller's current stream on this engine's device."""
        return current(self._dix)

    def raw_stream(self) -> int:
        """hipStream_t of the caller's current stream on this engine's device."""
        return current_raw(self._dix)

    def trace(self, name: str, stream=None):
        """A phase range of the tracer: roctx + host time, plus the device
        time between two HIP events on ``stream`` (GPU).  A no-op when the
        tracer is off and inside a hipGraph capture."""
        t = self.tracer
        if not t.enabled or self.capture_tag is not None:
            return contextlib.nullcontext()
        return t.gpu_range(name, stream) if self.gpu else t.range(name)

    def enable_osi(self) -> bool:
        """Switch the dedupers to occurrence-space unique ids (bucketed dedup
        with CAS inserts on GPU only): the dedup kernel writes the inverse
        index itself and the model's rows live at bstart[b] + l — in the
        pulled buffer on one GPU, in a per-slot buffer the received rows are
        unplaced into for N>1.  Returns whether it is on.

        Off unless SS_OSI=1: measured on MI355X (sparse LR, 10.2M keys/step)
        the forward gets 192 -> 123 us, but the dedup's random 4-B inverse
        stores cost more (217 -> 350 us): 1.26 vs 1.18 ms/step."""
        ok = (self.gpu and all(getattr(d, "mode", None) == "bucket" for d in self.dedupers)
              and (self.table is None or self.table.insert_mode == "cas")
              and os.environ.get("SS_OSI", "0") != "0")
        if not ok:
            return False
        for d in self.dedupers:
            d.osi = True
        if not self.fast1:
            self.uvals_osi = [torch.empty((self.max_keys, self.dim), dtype=torch.float32,
                                          device=self.device) for _ in range(self.depth)]
        self.osi = True
        return True

    def _rows_for_model(self, dd: DedupResult, uv: torch.Tensor, slot: int) -> torch.Tensor:
        """N>1 with osi: compact received rows -> occurrence-space rows."""
        if not self.osi or self.fast1:
            return uv
        out = self.uvals_osi[slot]
        dd.owner.unplace(dd.n, uv, out)
        return out

    # ------------------------------------------------------------ stage 1
    def route(self, keys: Optional[torch.Tensor] = None, produce=None, post=None) -> Routed:
        """Dedup + route a batch on the route stream (non-blocking on GPU).

        Either pass ``keys`` (produced on the current stream), or a
        ``produce(stream)`` callable that writes and returns the keys on the
        route stream (e.g. the synthetic data generator).  ``post(dd, slot,
        stream_ptr)`` runs right after dedup on the route stream (model-side
        planning that only depends on the key layout)."""
        slot = self._next_slot
        self._next_slot = (slot + 1) % self.depth
        dd_fn = self.dedupers[slot]
        if not self.gpu:
            with self.trace("route"):
                if produce is not None:
                    keys = produce(None)
                keys = keys.reshape(-1).to(self.device)
                dd = dd_fn(keys)
                counts = None if self.world == 1 and self.fast1 else \
                    self.ct.exchange_counts_async(dd.ucount)
            return Routed(dd, slot, counts)
        rs = self.route_stream
        # previous user of this slot is done (inside a capture only if it ran
        # in the same capture: an earlier replay has completed anyway)
        if self._free[slot] is not None:
            self._wait(rs, self._free[slot], self._free_tag[slot])
        if keys is not None and self.capture_tag is None:
            rs.wait_stream(self.main_stream())  # keys were produced on the main stream
        with use_stream(rs), self.trace("route", rs):
            if produce is not None:
                keys = produce(rs)
            keys = keys.reshape(-1)
            if keys.device != self.device:
                keys = keys.to(self.device)
            dd = dd_fn(keys, stream=rs)
            if post is not None:
                post(dd, slot, rs.cuda_stream)
            counts = None
            if not self.fast1:
                counts = self.ct.exchange_counts_async(dd.ucount, pinned=self._pins[slot],
                                                       stream=rs)
            ev = self._ev_route[slot]
            ev.record(rs)
        return Routed(dd, slot, counts, ev, self.capture_tag)

    # ------------------------------------------------------------ stage 2
    def _server_pull(self, rcounts: np.ndarray, slot: int) -> None:
        tab, D = self.table, self.displs
        nrecv = int(rcounts.sum())
        if tab is None or nrecv == 0:
            return
        if self.gpu:
            tab.pull(self.rkeys, insert=True, unique=False, out=self.rvals,
                     slots=self.rslots[slot], segs=tab.segs(D, rcounts), max_n=nrecv)
        else:
            for s in range(self.world):
                c = int(rcounts[s])
                if c:
                    self.rvals[D[s]:D[s] + c] = tab.pull_keys(self.rkeys[D[s]:D[s] + c])

    def pull(self, keys_or_routed) -> Round:
        r = keys_or_routed if isinstance(keys_or_routed, Routed) else self.route(keys_or_routed)
        with self.trace("pull"):
            return self._pull(r)

    def _pull(self, r: Routed) -> Round:
        dd, slot = r.dd, r.slot
        if self.gpu:
            self._wait(self.main_stream(), r.ready, r.tag)
        tab = self.table
        uv = self.uvals[slot]
        if self.fast1:
            own = dd.owner
            snap = None
            occ = None
            if getattr(own, "mode", None) == "bucket" and tab.insert_mode == "cas":
                if self.snapshot and not self.osi:
                    snap = self._snaps[slot]
                    if self.occ_buf is not None and tab.stride == 16:
                        occ = self.occ_buf
                tab.pull_buckets(own.bucket_view(dd.n), uv, self.slots[slot], osi=self.osi,
                                 snap=snap, luid=own.luid if occ is not None else None, occ=occ)
            else:
                tab.pull(dd.ukeys, insert=True, unique=True, out=uv, slots=self.slots[slot],
                         segs=tab.dev_segs(dd.ucount), max_n=max(1, min(dd.n, dd.ucap)))
            self.metrics.add(occurrences=dd.n)
            return Round(dd, uv, slot, slots=self.slots[slot], snap=snap,
                         snap_version=tab.version, occ_filled=occ is not None)
        scounts, rcounts = r.counts.wait()
        D = self.displs
        self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
        self._server_pull(rcounts, slot)
        self.t.alltoallv(self.rvals, rcounts, D, uv, scounts, D, self.dim)
        uv = self._rows_for_model(dd, uv, slot)
        sent, recv = int(scounts.sum()), int(rcounts.sum())
        # pull: keys out + rows back; push (next): grad rows out
        self.metrics.add(occurrences=dd.n, unique_sent=sent, unique_recv=recv,
                         a2a_bytes=8 * (sent + recv) + 4 * self.dim * (2 * sent + 2 * recv))
        return Round(dd, uv, slot, scounts=scounts, rcounts=rcounts,
                     stats={"sent": sent, "recv": recv})

    def pull_ahead_round(self, r: Routed) -> Round:
        """Stage 2 of a round on the route stream (pull-ahead mode): returns a
        Round whose rows are ready at ``rnd.ready``; ``begin(rnd)`` makes the
        current (main) stream wait for them."""
        dd, slot = r.dd, r.slot
        if self.fast1:
            # one GPU: the pull waits for this round's dedup only, on its own
            # stream (SS_PULL_STREAM=1), so the route stream goes on with the
            # next round's dedup meanwhile; or right behind the dedup on the
            # route stream
            uv, tab = self.uvals[slot], self.table
            rs = self.pull_stream or self.route_stream
            if rs is not self.route_stream:
                self._wait(rs, r.ready, r.tag)
            self._bound_staleness(rs, slot)
            self._take_gate(rs)
            with use_stream(rs), self.trace("pull", rs):
                own = dd.owner
                if getattr(own, "mode", None) == "bucket" and tab.insert_mode == "cas":
                    tab.pull_buckets(own.bucket_view(dd.n), uv, self.slots[slot], osi=self.osi,
                                     stream=rs)
                else:
                    tab.pull(dd.ukeys, insert=True, unique=True, out=uv, slots=self.slots[slot],
                             segs=tab.dev_segs(dd.ucount), max_n=max(1, min(dd.n, dd.ucap)))
                ev = self._ev_pull[slot]
                ev.record(rs)
            self.metrics.add(occurrences=dd.n)
            return Round(dd, uv, slot, slots=self.slots[slot], ready=ev, tag=self.capture_tag)
        scounts, rcounts = r.counts.wait()  # host: the route stage enqueued earlier
        D, uv = self.displs, self.uvals[slot]
        ps = self.pull_stream or self.route_stream
        if ps is not self.route_stream:
            self._wait(ps, r.ready, r.tag)
        self._bound_staleness(ps, slot)
        self._take_gate(ps)
        with use_stream(ps), self.trace("pull", ps):
            self.pt.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
            self._server_pull(rcounts, slot)
            self.pt.alltoallv(self.rvals, rcounts, D, uv, scounts, D, self.dim)
            uv = self._rows_for_model(dd, uv, slot)
            ev = self._ev_pull[slot]
            ev.record(ps)
        sent, recv = int(scounts.sum()), int(rcounts.sum())
        self.metrics.add(occurrences=dd.n, unique_sent=sent, unique_recv=recv,
                         a2a_bytes=8 * (sent + recv) + 4 * self.dim * (2 * sent + 2 * recv))
        return Round(dd, uv, slot, scounts=scounts, rcounts=rcounts,
                     stats={"sent": sent, "recv": recv}, ready=ev, tag=self.capture_tag)

    def gate_next_pull(self, slot: int) -> None:
        """Make the next ``pull_ahead_round`` wait for the work enqueued so
        far on the current stream (a model calls this inside its compute, after
        the kernels the lookup should not run beside).  Used by FM's
        SS_FM_PULL_GATE experiment (lookup behind the forward, whose gathers
        it slows 84 -> 215 us: the step measured slower, the lookup then
        crowds the merge and the update)."""
        if not self.gpu:
            return
        ev = self._ev_gate[slot]
        ev.record(self.main_stream())
        self._pull_gate = (ev, self.capture_tag)

    def _take_gate(self, stream) -> None:
        if self._pull_gate is not None:
            ev, tag = self._pull_gate
            self._pull_gate = None
            self._wait(stream, ev, tag)

    def _bound_staleness(self, stream, slot: int) -> None:
        """Pull-ahead of round i+1 (ring slot ``slot``): wait until round
        i-1's push has been applied, two slots back in the ring (staleness k:
        round i-k's).  Round i+1 then reads every update but round i's —
        staleness exactly 1.  Without
        the wait a side stream that runs ahead of the main stream (the host
        enqueues rounds before the device has finished earlier ones) can pull
        before round i-1 is applied as well: measured on FM (one GPU, pull on
        its own stream) the loss stuck at 0.69 instead of 0.60."""
        k = self.staleness
        if k <= 0 or k + 1 >= self.depth:
            return  # SS_STALENESS=ring: bounded by the ring depth only
        prev = (slot - k - 1) % self.depth
        if self._free[prev] is not None:
            self._wait(stream, self._free[prev], self._free_tag[prev])

    def enable_pull_ahead(self, on: bool = True, pull_stream: bool = False) -> bool:
        """Opt into pull-ahead (staleness 1) where the engine supports it.
        ``pull_stream`` (one GPU; SS_PULL_STREAM=0/1 overrides): run the
        pulled-ahead lookup on its own stream instead of behind the dedup on
        the route stream — pays when the lookup would otherwise hold up the
        next round's dedup (word2vec, 0.128 -> 0.125 ms/step), not when the
        main stream is the longer one anyway (FM, 0.655 -> 0.685)."""
        if on and self.gpu and self.depth >= 3 and \
                os.environ.get("SS_PULL_AHEAD", "1") != "0":
            self.pull_ahead = True
            want = os.environ.get("SS_PULL_STREAM", "1" if pull_stream else "0") != "0"
            if self.fast1 and self.pull_stream is None and want:
                self.pull_stream = torch.cuda.Stream(device=self.device)
        elif not on:
            self.pull_ahead = False
        return self.pull_ahead

    def begin(self, rnd: Round) -> None:
        if rnd.ready is not None:
            self._wait(self.main_stream(), rnd.ready, rnd.tag)

    # ------------------------------------------------------------ stage 3
    def _server_apply(self, rcounts: np.ndarray, slot: int, resolved: bool) -> None:
        """Apply received grads, one source rank at a time in rank order, so
        duplicate keys from different workers never race (no lost updates)."""
        tab, D = self.table, self.displs
        if tab is None:
            return
        for s in range(self.world):
            c = int(rcounts[s])
            if not c:
                continue
            if self.gpu:
                sl = tab.segs([D[s]], [c])
                rsl = self.rslots[slot]
                if not resolved:
                    _hip().probe(tab.dt, self.rkeys.data_ptr(), sl, c, rsl.data_ptr(),
                                 tab._init_native, 1, tab.size_ctr.data_ptr(),
                                 tab.err.data_ptr(), tab.G, _stream())
                if tab.push_fn is not None:
                    tab.apply_custom(rsl[D[s]:D[s] + c], self.rgrads[D[s]:D[s] + c])
                else:
                    tab.push_slots(rsl, self.rgrads, segs=sl, max_n=c)
            else:
                tab.push_keys(self.rkeys[D[s]:D[s] + c], self.rgrads[D[s]:D[s] + c])
        tab.next_round()

    def _release(self, slot: int):
        if self.gpu:
            ev = self._ev_free[slot]
            ev.record(self.main_stream())
            self._free[slot] = ev
            self._free_tag[slot] = self.capture_tag

    def fuse_apply(self, rnd: Round, snapshot: bool = True) -> Optional[dict]:
        """Arguments that let a model's gradient-merge kernel run the optimizer
        update itself (``bd_reduce(..., **args)`` / ``bd_reduce_fm``), or
        None.  One GPU, compact unique ids; ``snapshot``: scalar AdaGrad rows
        updated from the pull's still-valid (w, h) snapshot (blind store),
        else a read-modify-write of the row.  The round is marked applied and
        ``push`` only does the bookkeeping."""
        tab = self.table
        if not (self.fast1 and self.fuse_apply_on and not self.osi and not rnd.applied
                and rnd.slots is not None and getattr(tab, "push_fn", None) is None):
            return None
        if snapshot and not (rnd.snap is not None and rnd.snap_version == tab.version):
            return None
        rnd.applied = True
        tab.version += 1
        args = {"t": tab.dt, "slots": rnd.slots.data_ptr(), "op": tab.opt.native()}
        if snapshot:
            args["snap"] = rnd.snap.data_ptr()
        return args

    def push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        with self.trace("push", self.pull_stream if self.push_on_pull else None):
            self._push(rnd, grads)

    def _push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        g = rnd.ugrad if grads is None else grads
        tab = self.table
        if self.fast1 and rnd.applied:
            tab.next_round()
        elif self.fast1 and getattr(tab, "push_fn", None) is not None:
            # user-defined update rule: compact unique ids 0..ucount-1 (syncs)
            if self.osi:
                raise NotImplementedError("a custom push method needs compact unique ids")
            n = int(rnd.dd.ucount.sum())
            tab.apply_custom(rnd.slots[:n], g[:n])
            tab.next_round()
        elif self.fast1:
            if self.osi:
                tab.push_buckets(rnd.dd.owner.bucket_view(rnd.dd.n), rnd.slots, g)
            else:
                # the pull's (w, h) snapshot replaces the random row read when
                # no row changed since that pull (this round is the next push)
                snap = rnd.snap if (rnd.snap is not None and
                                    rnd.snap_version == tab.version) else None
                tab.push_slots(rnd.slots, g, segs=tab.dev_segs(rnd.dd.ucount),
                               max_n=max(1, min(rnd.dd.n, rnd.dd.ucap)), snap=snap)
            tab.next_round()
        elif self.push_on_pull:
            D, ps = self.displs, self.pull_stream
            ev = self._ev_grad[rnd.slot]
            ev.record(self.main_stream())  # the merged gradients
            ps.wait_event(ev)
            with use_stream(ps):
                self.pt.alltoallv(g, rnd.scounts, D, self.rgrads, rnd.rcounts, D, self.dim)
                self._server_apply(rnd.rcounts, rnd.slot, resolved=True)
                self._release(rnd.slot)  # the slot is free once the apply has read it
            rnd.pushed = True
            self.rounds += 1
            return
        else:
            D = self.displs
            self.t.alltoallv(g, rnd.scounts, D, self.rgrads, rnd.rcounts, D, self.dim)
            self._server_apply(rnd.rcounts, rnd.slot, resolved=True)
        self._release(rnd.slot)
        rnd.pushed = True
        self.rounds += 1

    # ------------------------------------------------------- occurrence API
    def gather(self, rnd: Round, n: Optional[int] = None) -> torch.Tensor:
        """Rows in occurrence order ([n, dim]) from a pulled round."""
        n = rnd.dd.n if n is None else n
        if self.gpu:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
            _hip().gather_rows(rnd.uvals.data_ptr(), rnd.inv.data_ptr(), n, self.dim,
                               out.data_ptr(), _stream())
            return out
        return rnd.uvals[rnd.inv[:n].long()]

    def accumulate(self, rnd: Round, grads: torch.Tensor) -> None:
        """Add per-occurrence gradients into the round's unique-key rows
        (the reference's merge_push_value, sparse_access_method.h:39-40)."""
        grads = grads.reshape(rnd.dd.n, self.dim).contiguous()
        if self.osi and not self.fast1:
            # the push sends compact rows; osi ids index occurrence space
            raise NotImplementedError("accumulate() with occurrence-space ids needs world 1")
        if self.gpu:
            _hip().scatter_add_rows(grads.data_ptr(), rnd.inv.data_ptr(), rnd.dd.n, self.dim,
                                    rnd.ugrad.data_ptr(), _stream())
        else:
            rnd.ugrad.index_add_(0, rnd.inv.long(), grads.to(rnd.ugrad.dtype))

    def pull_dense(self, keys: torch.Tensor) -> torch.Tensor:
        """pull_with_barrier in occurrence order: rows for `keys` ([n, dim])."""
        rnd = self.pull(keys)
        out = self.gather(rnd, keys.numel())
        self._release(rnd.slot)
        return out

    def push_keys(self, keys: torch.Tensor, grads: torch.Tensor) -> None:
        """Stand-alone push of per-occurrence gradients (no pull this round).

        Duplicate keys are merged (summed) on the worker first.  Keys unknown
        to the server are created with the initialiser before the update (the
        reference CHECK-fails, sparsetable.h:184)."""
        keys = keys.reshape(-1)
        # this path merges into zeroed rows and probes the send segment: force
        # both on the deduper that routes it (a model may have switched them off)
        own = self.dedupers[self._next_slot]
        saved = (getattr(own, "zero_grad", True), getattr(own, "need_ukeys", True),
                 getattr(own, "osi", False))
        own.zero_grad, own.need_ukeys = True, True
        if hasattr(own, "osi"):
            own.osi = False  # compact ids: the merge + probe below use the send segment
        try:
            r = self.route(keys)
        finally:
            own.zero_grad, own.need_ukeys = saved[:2]
            if hasattr(own, "osi"):
                own.osi = saved[2]
        if self.gpu:
            self._wait(self.main_stream(), r.ready, r.tag)
        dd = r.dd
        rnd = Round(dd, self.uvals[r.slot], r.slot)
        self.accumulate(rnd, grads.to(self.device))
        tab = self.table
        if self.fast1:
            sl = tab.dev_segs(dd.ucount)
            n = max(1, min(dd.n, dd.ucap))
            s = self.slots[r.slot]
            _hip().probe(tab.dt, dd.ukeys.data_ptr(), sl, n, s.data_ptr(), tab._init_native, 1,
                         tab.size_ctr.data_ptr(), tab.err.data_ptr(), tab.G, _stream())
            if tab.push_fn is not None:
                u = int(dd.ucount.sum())
                tab.apply_custom(s[:u], dd.ugrad[:u])
            else:
                tab.push_slots(s, dd.ugrad, segs=sl, max_n=n)
            tab.next_round()
        else:
            scounts, rcounts = r.counts.wait()
            D = self.displs
            self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
            self.t.alltoallv(dd.ugrad, scounts, D, self.rgrads, rcounts, D, self.dim)
            self._server_apply(rcounts, r.slot, resolved=False)
        self._release(r.slot)
        self.rounds += 1

    def barrier(self):
        self.t.barrier()

    def check(self) -> None:
        """Raise on a sticky device-side error of this rank (syncs): a dedup
        bucket whose LDS table overflowed (its occurrences got no unique id,
        so their rows and gradients were dropped) or a full / misused table.
        Called at the check points that must not pass silently: the end of
        bench.py, every periodic backup and PSContext.finish."""
        for d in self.dedupers:
            chk = getattr(d, "check", None)
            if chk is not None:
                chk()
        chk = getattr(self.table, "check", None) if self.table is not None else None
        if chk is not None:
            chk()
