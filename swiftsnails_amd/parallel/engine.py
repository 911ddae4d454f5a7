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
                          LDS dedup, every rank on the same bucket layout);
                          [N>1] counts + per-bucket runs to the servers
    pull  (main stream, or the pull stream with pull-ahead): [N>1] keys out ->
                          server merge of all sources' keys (server.hip: ONE
                          lookup per distinct key) -> rows back
    push  (main stream) : [N>1] grads out -> server merge of all sources'
                          gradients + ONE optimizer update per distinct key

``route`` of step i+1 is enqueued before ``pull`` of step i on its own HIP
stream, so key generation, dedup and the count exchange overlap the previous
step's compute.  With pull-ahead (N>1 default; FM and word2vec at N=1) round
i+1 is pulled while round i computes (staleness exactly 1).  Route buffers
are a ring of ``depth`` slots.  On one GPU (world 1) no host synchronisation
happens at all: the unique-key count stays on the device, scalar AdaGrad rows
are snapshotted by the pull and updated inside the model's gradient merge
(``fuse_apply``).

Split roles (S servers + W workers) fall out of the same code: non-server
ranks own no table and receive nothing (the router never maps to them);
non-worker ranks route an empty key set — every rank still enters the
collectives, which is what makes the round lockstep.

The same engine runs on CPU (``HostTable`` shards, host dedup, gloo
transport) — that is how the multi-rank logic is tested without GPUs; the
host server merges duplicate keys across sources exactly like the device one.
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
    ready: Optional[object] = None        # pull-ahead: event of the pulled rows
    tag: Optional[int] = None             # hipGraph capture of `ready`
    snap: Optional[torch.Tensor] = None   # world-1: (w, h) rows as pulled (blind apply)
    snap_version: int = -1                # table.version the snapshot is valid for
    applied: bool = False                 # the model's kernel already ran K5 (fuse_apply)
    server: Optional[object] = None       # CPU N>1: (unique keys, inverse) of the server merge

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


class _ServerSlot:
    """Device buffers of one ring slot's server-side merge (N>1, GPU): the
    bucket layout of the distinct keys received from all sources and what
    survives from the pull to the push of the round."""

    def __init__(self, rows: int, P: int, dim: int, dev, snapshot: bool):
        u32 = torch.int32
        self.cnt = torch.zeros(P + 1, dtype=u32, device=dev)  # + the arrival counter
        self.bstart = torch.empty(P + 1, dtype=u32, device=dev)
        self.ubase = torch.empty(P, dtype=u32, device=dev)
        self.unum = torch.empty(P, dtype=u32, device=dev)
        self.ucount = torch.zeros(1, dtype=torch.int64, device=dev)
        self.pj = torch.empty(rows, dtype=u32, device=dev)
        self.luid = torch.empty(rows, dtype=u32, device=dev)
        self.bkeys = torch.empty(rows, dtype=torch.int64, device=dev)
        self.slots = torch.empty(rows, dtype=torch.int64, device=dev)
        self.snap = torch.empty((rows, 2), dtype=torch.float32, device=dev) if snapshot else None
        self.snap_valid = False

    def view(self, P: int):
        return (self.bkeys.data_ptr(), self.bstart.data_ptr(), self.unum.data_ptr(),
                self.ubase.data_ptr(), P)


class PSEngine:
    """Worker+server round engine for one rank.

    table           : this rank's shard (``HbmTable``/``HostTable``) or None when not a server
    transport       : data-plane transport (RCCL on MI355X)
    count_transport : transport of the route-stage exchanges (counts, bucket
                      runs); defaults to ``transport``
    pull_transport  : transport of the pulled-ahead keys/rows exchanges
    max_keys        : max key occurrences per pull on this rank (must agree
                      across ranks: it fixes the common bucket layout)
    server_ranks    : ranks that host a shard (default: all — colocated mode)
    frag_num        : number of hash fragments (reference config ``frag_num``)
    depth           : route-buffer ring depth

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
        # SS_ENGINE_GENERAL=1 (or rccl) runs a 1-GPU job through the N>1 code
        # path: the per-rank cost of the multi-GPU pipeline without the network
        self.fast1 = (self.gpu and self.world == 1 and
                      os.environ.get("SS_ENGINE_GENERAL", "0") == "0")
        self.dist = not self.fast1
        # the xGMI mailbox transport (device-side counts) or a host-count one
        from .xgmi import XgmiTransport

        self.xg = self.t if isinstance(self.t, XgmiTransport) else None
        # N>1 on GPU: segment strides a multiple of 64 rows (aligned peer stores)
        self.max_keys = int(max_keys) if not (self.gpu and self.dist) else \
            -(-int(max_keys) // 64) * 64
        # ring depth 4 by default: with one batch of lookahead, routing round
        # i+1 reuses the buffers of round i-3 (long pushed) instead of waiting
        # on round i-1's push; 4 measured 1.008 vs 1.018 ms/step for 3 (LR,
        # one GPU).  Drops to 3 when a fourth slot would take more than 1/8 of
        # the device's memory (wide rows at large N)
        if depth is None and os.environ.get("SS_ENGINE_DEPTH") is None:
            depth = 4
            if self.gpu and 4 * self.slot_bytes(self.world, max_keys, dim) > \
                    torch.cuda.mem_get_info(self.device)[1] // 8:
                depth = 3
        self.depth = max(1, int(depth if depth is not None else
                                os.environ.get("SS_ENGINE_DEPTH", "4")))
        from ..utils.tracing import Metrics

        # observability: occurrences routed, unique keys exchanged,
        # distinct keys the servers merged them into, alltoallv payload bytes
        self.metrics = Metrics()
        self.tracer = Tracer(enabled=False)
        fm = torch.from_numpy(self.frag_map.astype(np.int32))
        dd_cls = Deduper if self.gpu else CpuDeduper
        self.dedupers = [dd_cls(self.max_keys, nranks=self.world, frag_map=fm, gdim=self.dim,
                                device=self.device, zero_grad=zero_grad) for _ in range(self.depth)]
        N, cap, d = self.world, self.max_keys, self.dim
        dev = self.device
        self.uvals = [torch.empty((N * cap, d), dtype=torch.float32, device=dev)
                      for _ in range(self.depth)]
        self.displs = [r * cap for r in range(N)]
        self.rounds = 0
        self._next_slot = 0
        self.snapshot = False
        self.pull_ahead = False
        self.pull_stream = None
        self.capture_tag: Optional[int] = None
        self._dix = (self.device.index or 0) if self.gpu else -1
        if self.gpu:
            self.route_stream = torch.cuda.Stream(device=dev)
            self._free = [None] * self.depth  # main-stream event: slot buffers released
            self._free_tag = [None] * self.depth
            self._pins = [torch.zeros(2 * N, dtype=torch.int64, pin_memory=True)
                          for _ in range(self.depth)]
            self._ev_route = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_pull = [torch.cuda.Event() for _ in range(self.depth)]
            self._ev_free = [torch.cuda.Event() for _ in range(self.depth)]
        if self.fast1:
            self.slots = [torch.empty(cap, dtype=torch.int64, device=dev)
                          for _ in range(self.depth)]
            # pull snapshots for the blind-write apply (scalar AdaGrad rows,
            # pull and push of a round adjacent in table order: Round.snap)
            self.snapshot = bool(getattr(table, "snapshot_ok", False))
            self._snaps = [torch.empty((cap, 2), dtype=torch.float32, device=dev)
                           for _ in range(self.depth)] if self.snapshot else None
            # the colocated pull reads the bucketed dedup's staging directly:
            # no contiguous send segment is needed
            if table is not None:
                for dd in self.dedupers:
                    dd.need_ukeys = False
        elif self.gpu:
            self._init_dist_gpu()
        else:
            self.rkeys = torch.empty(N * cap, dtype=torch.int64)
            self.rvals = torch.zeros((N * cap, d), dtype=torch.float32)
            self.rgrads = torch.empty((N * cap, d), dtype=torch.float32)
        # pull-ahead (N>1 on GPU): round i+1's pull (keys a2av, server merge +
        # lookup, rows a2av) runs on the pull stream while round i computes
        # and pushes on the main stream — bounded staleness 1, the
        # asynchronous-PS semantics of the reference.  Needs ring
        # depth >= 3 (rounds i, i+1, i+2 in flight)
        if self.gpu and self.dist and self.depth >= 3 and \
                os.environ.get("SS_PULL_AHEAD", "1") != "0":
            self.pull_ahead = True
            self.pull_stream = torch.cuda.Stream(device=self.device)
        # pull-ahead staleness bound (_bound_staleness): a pulled-ahead round
        # misses at most this many rounds' updates; SS_STALENESS=ring: only the
        # ring depth bounds it
        st_env = os.environ.get("SS_STALENESS", "1")
        self.staleness = 0 if st_env == "ring" else max(1, int(st_env))

    # ------------------------------------------------------------ N>1 (GPU)
    def _init_dist_gpu(self) -> None:
        """Receive buffers and the server-merge slots of the N>1 device path.
        Every rank lays its buckets out as a call of ``max_keys`` keys (the
        common layout the servers merge), and sends each destination its
        per-bucket runs with the keys."""
        N, cap, d, dev = self.world, self.max_keys, self.dim, self.device
        h = _hip()
        for dd in self.dedupers:
            dd.lay_n = cap
        self.Pd = h.bd_buckets(cap, N, self.dedupers[0].ndest) // N
        self.sub = h.srv_sub_buckets(N)
        self.Ps = self.Pd * self.sub
        # every rank's max_keys must agree (it fixes Pd); one int all-reduce
        # at start-up turns a mismatch into an error instead of wrong routing
        mk = torch.tensor([cap, -cap], dtype=torch.int64, device=dev)
        self._agree(mk)
        if int(mk[0]) != cap or int(-mk[1]) != cap:
            raise ValueError("PSEngine: max_keys differs across ranks (the N>1 bucket layout "
                             "is a function of it)")
        rows = N * cap
        self.rvals = torch.zeros((rows, d), dtype=torch.float32, device=dev)
        if self.xg:
            # the receive buffers are the arena's mailboxes: keys + the bucket
            # runs (bases, sizes) per source, rows back, gradients
            Pd = self.Pd
            self.xg.setup({"keys": (self.depth, [cap * 8, Pd * 4, Pd * 4]),
                           "vals": (self.depth, [cap * 4 * d]),
                           "grads": (self.depth, [cap * 4 * d])})
            self.rkeys = [self.xg.region("keys", 0, q, torch.int64) for q in range(self.depth)]
            self.rmeta = [(self.xg.region("keys", 1, q, torch.int32),
                           self.xg.region("keys", 2, q, torch.int32)) for q in range(self.depth)]
            self.uvals = [self.xg.region("vals", 0, q, torch.float32, d)
                          for q in range(self.depth)]
            self.rgrads = [self.xg.region("grads", 0, q, torch.float32, d)
                           for q in range(self.depth)]
        else:
            self.rkeys = [torch.empty(rows, dtype=torch.int64, device=dev)] * self.depth
            # per slot: the received bucket runs ([N][Pd] bases, then sizes)
            meta = [torch.zeros(2 * N * self.Pd, dtype=torch.int32, device=dev)
                    for _ in range(self.depth)]
            self.rmeta = [(m[:N * self.Pd], m[N * self.Pd:]) for m in meta]
            self.rgrads = [torch.empty((rows, d), dtype=torch.float32, device=dev)] * self.depth
        self.srv = None
        if self.table is not None:
            self.svals = torch.empty((rows, d), dtype=torch.float32, device=dev)
            self.sgrad = torch.empty((rows, d), dtype=torch.float32, device=dev)
            self.srv_err = torch.zeros(1, dtype=torch.int32, device=dev)
            # a snapshot pull + blind-store update is exact only if nothing
            # writes the rows between a round's pull and its push: without
            # pull-ahead (decided after this; re-checked per round)
            snap_ok = bool(getattr(self.table, "snapshot_ok", False))
            self.srv = [_ServerSlot(rows, self.Ps, d, dev, snap_ok) for _ in range(self.depth)]

    def _agree(self, t: torch.Tensor) -> None:
        """min-all-reduce of a small int64 tensor over the data transport."""
        if self.world == 1:
            return
        self.t.allreduce_(t, "min")
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()

    @staticmethod
    def slot_bytes(world: int, max_keys: int, dim: int) -> int:
        """Device bytes of one route-ring slot: pulled rows, the deduper's
        send keys + gradient rows (+ its ~40 B/key scratch) and, for N>1, the
        server merge of the slot (~32 B per received key)."""
        rows = world * max_keys
        return rows * (4 * dim + 8 + 4 * dim + (32 if world > 1 else 0)) + 40 * max_keys

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
                counts = self.ct.exchange_counts_async(dd.ucount)
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
            if self.dist:
                # the keys with the per-bucket runs of every destination's
                # segment (fixed size: Pd bases + Pd sizes per peer)
                ub, un = dd.owner.run_tables(self.Pd)
                Pd, N = self.Pd, self.world
                dsp = [r * Pd for r in range(N)]
                if self.xg:
                    self.xg.put("keys", slot, [(dd.ukeys, self.displs, dd.ucount, None),
                                               (ub, dsp, None, Pd), (un, dsp, None, Pd)],
                                stream=rs)
                else:
                    counts = self.ct.exchange_counts_async(dd.ucount, pinned=self._pins[slot],
                                                           stream=rs)
                    mb, mn = self.rmeta[slot]
                    fixed = [Pd] * N
                    self.ct.alltoallv(ub, fixed, dsp, mb, fixed, dsp, 1)
                    self.ct.alltoallv(un, fixed, dsp, mn, fixed, dsp, 1)
            ev = self._ev_route[slot]
            ev.record(rs)
        return Routed(dd, slot, counts, ev, self.capture_tag)

    # ------------------------------------------------------------ stage 2
    def _server_pull_gpu(self, slot: int, stream) -> None:
        """Merge the keys of all sources (one entry per distinct key), look
        them up / create them, fill the response rows per received key."""
        tab = self.table
        if tab is None:
            return
        h, S, N = _hip(), self.srv[slot], self.world
        st = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        mb, mn = self.rmeta[slot]
        h.srv_dedup(self.rkeys[slot].data_ptr(), mb.data_ptr(), mn.data_ptr(),
                    self.max_keys, N, self.Pd, self.sub, self.rank, S.cnt.data_ptr(),
                    S.bstart.data_ptr(), S.pj.data_ptr(), S.luid.data_ptr(), S.bkeys.data_ptr(),
                    S.ubase.data_ptr(), S.unum.data_ptr(), S.ucount.data_ptr(),
                    self.srv_err.data_ptr(), st)
        # a snapshot is exact when no update lands between this pull and the
        # round's push: the pull and push alternate (no pull-ahead)
        S.snap_valid = S.snap is not None and not self.pull_ahead and tab.snapshot_ok
        tab.pull_buckets(S.view(self.Ps), self.svals, S.slots, stream=st,
                         snap=S.snap if S.snap_valid else None)
        if tab.custom_pull:  # user init / pull methods (tensor code; syncs)
            tab.finish_pull(S.slots, self.svals, n=S.ucount)
        h.srv_fill(self.Ps, S.bstart.data_ptr(), S.ubase.data_ptr(), S.unum.data_ptr(),
                   S.pj.data_ptr(), S.luid.data_ptr(), self.svals.data_ptr(),
                   self.rvals.data_ptr(), self.dim, st)
        if not self.xg:  # (xgmi: counted by the vals wait, no launch of its own)
            sacc = self.metrics.device_block(("server_unique",), self.device)
            sacc.add_(S.ucount)  # (one tiny kernel, no sync)

    def _server_pull_cpu(self, rcounts: np.ndarray):
        """Host server: distinct keys of all sources, looked up once."""
        tab, D = self.table, self.displs
        if tab is None or int(rcounts.sum()) == 0:
            return None
        idx = np.concatenate([np.arange(D[s], D[s] + int(rcounts[s]))
                              for s in range(self.world)])
        keys = self.rkeys[torch.from_numpy(idx)]
        uk, inv = torch.unique(keys, return_inverse=True)
        self.rvals[torch.from_numpy(idx)] = tab.pull_keys(uk)[inv]
        self.metrics.add(server_unique=int(uk.numel()))
        return (idx, uk, inv)

    def _pull_xgmi(self, r: Routed, stream) -> Round:
        """Keys in (put by every source at route time), server merge +
        lookup, rows back over the mailboxes; nothing leaves the device."""
        dd, slot, xg = r.dd, r.slot, self.xg
        nb = 4 * self.Pd
        xg.wait("keys", slot, stream, fixed_parts=[(1, nb), (2, nb)])
        self._server_pull_gpu(slot, stream)
        rc = xg.counts("keys", 0, slot)
        xg.put("vals", slot, [(self.rvals, self.displs, rc, None, self.dim)], stream=stream)
        acc = self.metrics.device_block(("unique_sent", "unique_recv", "a2a_bytes"), self.device)
        sx = None
        if self.table is not None:
            sx = self.metrics.device_block(("server_unique",), self.device)
        xg.wait("vals", slot, stream,
                metrics=(dd.ucount, rc, acc, self.srv[slot].ucount if sx is not None else None, sx),
                bytes_per_key=8.0 + 8.0 * self.dim)
        self.metrics.add(occurrences=dd.n)
        return Round(dd, self.uvals[slot], slot)

    def _pull_exchange(self, r: Routed, uv: torch.Tensor, tr: Transport, stream):
        """Keys out, server merge + lookup, rows back (N>1; host counts)."""
        if self.xg and self.gpu:
            return self._pull_xgmi(r, stream)
        dd, slot = r.dd, r.slot
        scounts, rcounts = r.counts.wait()
        D = self.displs
        tr.alltoallv(dd.ukeys, scounts, D, self.rkeys[slot] if self.gpu else self.rkeys,
                     rcounts, D, 1)
        server = None
        if self.gpu:
            self._server_pull_gpu(slot, stream)
        else:
            server = self._server_pull_cpu(rcounts)
        tr.alltoallv(self.rvals, rcounts, D, uv, scounts, D, self.dim)
        sent, recv = int(scounts.sum()), int(rcounts.sum())
        # pull: keys out + rows back; push (next): grad rows out
        self.metrics.add(occurrences=dd.n, unique_sent=sent, unique_recv=recv,
                         a2a_bytes=8 * (sent + recv) + 4 * self.dim * (2 * sent + 2 * recv))
        return Round(dd, uv, slot, scounts=scounts, rcounts=rcounts,
                     stats={"sent": sent, "recv": recv}, server=server)

    def pull(self, keys_or_routed) -> Round:
        r = keys_or_routed if isinstance(keys_or_routed, Routed) else self.route(keys_or_routed)
        with self.trace("pull"):
            return self._pull(r)

    def _pull(self, r: Routed) -> Round:
        dd, slot = r.dd, r.slot
        if self.gpu:
            self._wait(self.main_stream(), r.ready, r.tag)
        uv = self.uvals[slot]
        if not self.fast1:
            return self._pull_exchange(r, uv, self.t, self.main_stream() if self.gpu else None)
        tab = self.table
        snap = None
        own = dd.owner
        if getattr(own, "mode", None) == "bucket":
            if self.snapshot and tab.snapshot_ok:
                snap = self._snaps[slot]
            tab.pull_buckets(own.bucket_view(dd.n), uv, self.slots[slot], snap=snap)
        else:
            tab.pull(dd.ukeys, insert=True, unique=True, out=uv, slots=self.slots[slot],
                     segs=tab.dev_segs(dd.ucount), max_n=max(1, min(dd.n, dd.ucap)))
        if tab.custom_pull:  # user init / pull methods (tensor code; syncs)
            tab.finish_pull(self.slots[slot], uv, n=dd.ucount)
        self.metrics.add(occurrences=dd.n)
        return Round(dd, uv, slot, slots=self.slots[slot], snap=snap,
                     snap_version=tab.version)

    def pull_ahead_round(self, r: Routed) -> Round:
        """Stage 2 of a round on the pull (or route) stream (pull-ahead
        mode): returns a Round whose rows are ready at ``rnd.ready``;
        ``begin(rnd)`` makes the current (main) stream wait for them."""
        dd, slot = r.dd, r.slot
        ps = self.pull_stream or self.route_stream
        if ps is not self.route_stream:
            self._wait(ps, r.ready, r.tag)
        self._bound_staleness(ps, slot)
        with use_stream(ps), self.trace("pull", ps):
            if self.fast1:
                # one GPU: the pull waits for this round's dedup only
                uv, tab, own = self.uvals[slot], self.table, dd.owner
                if getattr(own, "mode", None) == "bucket":
                    tab.pull_buckets(own.bucket_view(dd.n), uv, self.slots[slot], stream=ps)
                else:
                    tab.pull(dd.ukeys, insert=True, unique=True, out=uv, slots=self.slots[slot],
                             segs=tab.dev_segs(dd.ucount), max_n=max(1, min(dd.n, dd.ucap)))
                if tab.custom_pull:
                    tab.finish_pull(self.slots[slot], uv, n=dd.ucount)
                self.metrics.add(occurrences=dd.n)
                rnd = Round(dd, uv, slot, slots=self.slots[slot])
            else:
                rnd = self._pull_exchange(r, self.uvals[slot], self.pt, ps)
            ev = self._ev_pull[slot]
            ev.record(ps)
        rnd.ready, rnd.tag = ev, self.capture_tag
        return rnd

    def _bound_staleness(self, stream, slot: int) -> None:
        """Pull-ahead of round i+1 (ring slot ``slot``): wait until round
        i-1's push has been applied, two slots back in the ring (staleness k:
        round i-k's).  Round i+1 then reads every update but round i's —
        staleness exactly 1.  Without the wait a side stream that runs ahead
        of the main stream can pull before round i-1 is applied as well:
        measured on FM (one GPU, pull on its own stream) the loss stuck at
        0.69 instead of 0.60."""
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
    def _server_push_gpu(self, slot: int) -> None:
        """Merge the gradients all sources pushed for each distinct key and
        update every such row once (fused for scalar AdaGrad rows)."""
        tab = self.table
        if tab is None:
            return
        h, S, st = _hip(), self.srv[slot], _stream()
        args = (self.Ps, S.bstart.data_ptr(), S.ubase.data_ptr(), S.unum.data_ptr(),
                S.pj.data_ptr(), S.luid.data_ptr(), self.rgrads[slot].data_ptr())
        fused = (self.dim == 1 and tab.push_fn is None and tab.opt.kind == "adagrad" and
                 tab.width == 2 and tab.G == 1 and not getattr(tab, "bf16", False))
        if fused:
            h.srv_merge(*args, 0, 1, tab.dt, S.slots.data_ptr(),
                        S.snap.data_ptr() if S.snap_valid else 0, tab.opt.native(), st)
        elif self.dim > 1 and tab.push_fn is None:
            # rows: the merged gradient row goes straight into the update
            h.srv_merge(*args, 0, self.dim, tab.dt, S.slots.data_ptr(), 0, tab.opt.native(), st)
        else:
            h.srv_merge(*args, self.sgrad.data_ptr(), self.dim, st=st)
            if tab.push_fn is not None:
                u = int(S.ucount.item())  # a tensor rule runs on host-sized tensors
                tab.apply_custom(S.slots[:u], self.sgrad[:u])
            else:
                tab.push_slots(S.slots, self.sgrad, segs=tab.dev_segs(S.ucount),
                               max_n=self.world * self.max_keys)
        tab.version += 1

    def _server_push_cpu(self, rnd: Round) -> None:
        tab = self.table
        if tab is None or rnd.server is None:
            return
        idx, uk, inv = rnd.server
        g = torch.zeros((uk.numel(), self.dim), dtype=torch.float32)
        g.index_add_(0, inv, self.rgrads[torch.from_numpy(idx)])
        tab.push_keys(uk, g)

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
        if not (self.fast1 and not rnd.applied and rnd.slots is not None
                and getattr(tab, "push_fn", None) is None):
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
        with self.trace("push"):
            self._push(rnd, grads)

    def _push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        g = rnd.ugrad if grads is None else grads
        tab = self.table
        if self.fast1:
            if rnd.applied:
                pass
            elif getattr(tab, "push_fn", None) is not None:
                # user-defined update rule: compact unique ids 0..ucount-1 (syncs)
                n = int(rnd.dd.ucount.sum())
                tab.apply_custom(rnd.slots[:n], g[:n])
            else:
                # the pull's (w, h) snapshot replaces the random row read when
                # no row changed since that pull (this round is the next push)
                snap = rnd.snap if (rnd.snap is not None and
                                    rnd.snap_version == tab.version) else None
                tab.push_slots(rnd.slots, g, segs=tab.dev_segs(rnd.dd.ucount),
                               max_n=max(1, min(rnd.dd.n, rnd.dd.ucap)), snap=snap)
            tab.next_round()
        else:
            D = self.displs
            if self.xg and self.gpu:
                self.xg.put("grads", rnd.slot, [(g, D, rnd.dd.ucount, None, self.dim)],
                            stream=self.main_stream())
                self.xg.wait("grads", rnd.slot, self.main_stream())
            else:
                self.t.alltoallv(g, rnd.scounts, D,
                                 self.rgrads[rnd.slot] if self.gpu else self.rgrads,
                                 rnd.rcounts, D, self.dim)
            if self.gpu:
                self._server_push_gpu(rnd.slot)
            else:
                self._server_push_cpu(rnd)
            if tab is not None:
                tab.next_round()
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
                 getattr(own, "materialize_inv", True))
        own.zero_grad, own.need_ukeys, own.materialize_inv = True, True, True
        try:
            r = self.route(keys)
        finally:
            own.zero_grad, own.need_ukeys, own.materialize_inv = saved
        if self.gpu:
            self._wait(self.main_stream(), r.ready, r.tag)
        dd = r.dd
        if self.fast1:
            rnd = Round(dd, self.uvals[r.slot], r.slot)
            self.accumulate(rnd, grads.to(self.device))
            tab = self.table
            sl = tab.dev_segs(dd.ucount)
            n = max(1, min(dd.n, dd.ucap))
            s = self.slots[r.slot]
            _hip().probe(tab.dt, dd.ukeys.data_ptr(), sl, n, s.data_ptr(), tab._init_native, 1,
                         tab.size_ctr.data_ptr(), tab.err.data_ptr(), tab.G, _stream())
            if tab.init_fn is not None:  # keys this push created: the user's rows first
                tab.finish_pull(s, self.uvals[r.slot], n=dd.ucount)
            if tab.push_fn is not None:
                u = int(dd.ucount.sum())
                tab.apply_custom(s[:u], dd.ugrad[:u])
            else:
                tab.push_slots(s, dd.ugrad, segs=sl, max_n=n)
            tab.next_round()
            self._release(r.slot)
            self.rounds += 1
            return
        # N>1: the pull half creates missing keys on their servers (the rows
        # it returns are not needed), the push half merges and applies
        rnd = self._pull_exchange(r, self.uvals[r.slot], self.t,
                                  self.main_stream() if self.gpu else None)
        self.accumulate(rnd, grads.to(self.device))
        self._push(rnd)

    def barrier(self):
        self.t.barrier()

    def all_done(self, local_done: bool) -> bool:
        """Collective termination check: True once every rank reports done.
        Every rank calls it at the same rounds (syncs); a rank that finished
        early keeps serving rounds with an empty key set until then — the
        reference's master waiting for WORKER_FINISH_WORK from every worker
        before telling the servers to stop (master/terminate.h:44-62)."""
        if self.world == 1:
            return bool(local_done)
        dev = self.device if (self.gpu and not hasattr(self.t, "aux")) else "cpu"
        flag = torch.tensor([1 if local_done else 0], dtype=torch.int64, device=dev)
        self.t.allreduce_(flag, "min")
        return int(flag.item()) == 1

    def check(self) -> None:
        """Raise on a sticky device-side error of this rank (syncs): a dedup
        bucket whose LDS table overflowed (its occurrences got no unique id,
        so their rows and gradients were dropped), a server-merge bucket that
        overflowed, or a full / misused table.  Called at the check points
        that must not pass silently: the end of bench.py, every periodic
        backup and PSContext.finish."""
        for d in self.dedupers:
            chk = getattr(d, "check", None)
            if chk is not None:
                chk()
        if getattr(self, "srv", None) is not None and int(self.srv_err.item()) != 0:
            from ..ops.dedup import DedupOverflowError

            raise DedupOverflowError("server merge: a bucket of received keys overflowed its "
                                     "LDS table")
        chk = getattr(self.table, "check", None) if self.table is not None else None
        if chk is not None:
            chk()
        if self.xg is not None:
            self.xg.check()  # a peer that never arrived / a corrupt count
