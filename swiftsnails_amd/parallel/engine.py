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

Here a round is lockstep across ranks:

    pull:  dedup+route (1 kernel + inverse) -> [N>1] counts a2a -> keys a2av
           -> server probe/init/gather -> values a2av back
    push:  grads a2av -> server apply, one launch per source rank in rank order

On one GPU (world 1) the round needs no host synchronisation at all: the
unique-key count stays on the device and every kernel reads it there.

Split roles (S servers + W workers) fall out of the same code: non-server
ranks own no table and receive nothing (the router never maps to them);
non-worker ranks call ``pull``/``push`` with an empty key set — every rank
still enters the collective, which is what makes the round lockstep.

The same engine runs on CPU (``HostTable`` shards, host dedup, gloo
transport) — that is how the multi-rank logic is tested without GPUs.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops.dedup import CpuDeduper, DedupResult, Deduper
from .router import HashFrag
from .transport import LoopbackTransport, Transport


@dataclass
class Round:
    dd: DedupResult
    uvals: torch.Tensor                   # [N*ucap, dim] pulled rows, unique-key order
    slots: Optional[torch.Tensor] = None  # GPU world-1 path: table slots of ukeys
    scounts: Optional[np.ndarray] = None  # keys this rank sent to each server
    rcounts: Optional[np.ndarray] = None  # keys this rank received from each worker
    pushed: bool = False
    stats: dict = field(default_factory=dict)

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
    return torch.cuda.current_stream().cuda_stream


class PSEngine:
    """Worker+server round engine for one rank.

    table         : this rank's shard (``HbmTable``/``HostTable``) or None when not a server
    transport     : data-plane transport (RCCL on MI355X)
    max_keys      : max key occurrences per pull on this rank
    server_ranks  : ranks that host a shard (default: all — colocated mode)
    frag_num      : number of hash fragments (reference config ``frag_num``)

    A ``Round`` aliases engine-owned buffers: it is valid until the next pull.
    """

    def __init__(self, table, transport: Optional[Transport], max_keys: int, dim: int,
                 frag_num: int = 0, server_ranks: Optional[Sequence[int]] = None, device=None):
        self.t = transport or LoopbackTransport()
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
        dd_cls = Deduper if self.gpu else CpuDeduper
        self.dedup = dd_cls(self.max_keys, nranks=self.world,
                            frag_map=torch.from_numpy(self.frag_map.astype(np.int32)),
                            gdim=self.dim, device=self.device)
        N, cap, d = self.world, self.max_keys, self.dim
        dev = self.device
        self.uvals = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
        self.fast1 = self.gpu and self.world == 1
        if self.fast1:
            self.slots = torch.empty(cap, dtype=torch.int64, device=dev)
        else:
            # server-side receive buffers: one fixed segment per source rank
            self.rkeys = torch.empty(N * cap, dtype=torch.int64, device=dev)
            self.rvals = torch.zeros((N * cap, d), dtype=torch.float32, device=dev)
            self.rgrads = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
            if self.gpu:
                self.rslots = torch.empty(N * cap, dtype=torch.int64, device=dev)
        self.displs = [r * cap for r in range(N)]
        self.rounds = 0

    # ----------------------------------------------------------- server side
    def _server_pull(self, rcounts: np.ndarray) -> None:
        tab, D = self.table, self.displs
        nrecv = int(rcounts.sum())
        if tab is None or nrecv == 0:
            return
        if self.gpu:
            tab.pull(self.rkeys, insert=True, unique=False, out=self.rvals, slots=self.rslots,
                     segs=tab.segs(D, rcounts), max_n=nrecv)
        else:
            for s in range(self.world):
                c = int(rcounts[s])
                if c:
                    self.rvals[D[s]:D[s] + c] = tab.pull_keys(self.rkeys[D[s]:D[s] + c])

    def _server_apply(self, rcounts: np.ndarray, resolved: bool) -> None:
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
                if not resolved:
                    h = _hip()
                    h.probe(tab.dt, self.rkeys.data_ptr(), sl, c, self.rslots.data_ptr(),
                            tab._init_native, 1, tab.size_ctr.data_ptr(), tab.err.data_ptr(),
                            tab.G, _stream())
                tab.push_slots(self.rslots, self.rgrads, segs=sl, max_n=c)
            else:
                tab.push_keys(self.rkeys[D[s]:D[s] + c], self.rgrads[D[s]:D[s] + c])
        tab.next_round()

    # ------------------------------------------------------------------ pull
    def pull(self, keys: torch.Tensor) -> Round:
        keys = keys.reshape(-1)
        if keys.device != self.device:
            keys = keys.to(self.device)
        dd = self.dedup(keys)
        tab = self.table
        if self.fast1:
            tab.pull(dd.ukeys, insert=True, unique=True, out=self.uvals, slots=self.slots,
                     segs=tab.dev_segs(dd.ucount), max_n=max(1, min(keys.numel(), dd.ucap)))
            return Round(dd, self.uvals, slots=self.slots)
        scounts, rcounts = self.t.exchange_counts(dd.ucount)
        D = self.displs
        self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
        self._server_pull(rcounts)
        self.t.alltoallv(self.rvals, rcounts, D, self.uvals, scounts, D, self.dim)
        return Round(dd, self.uvals, scounts=scounts, rcounts=rcounts,
                     stats={"sent": int(scounts.sum()), "recv": int(rcounts.sum())})

    # ------------------------------------------------------------------ push
    def push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        g = rnd.ugrad if grads is None else grads
        tab = self.table
        if self.fast1:
            tab.push_slots(rnd.slots, g, segs=tab.dev_segs(rnd.dd.ucount),
                           max_n=max(1, min(rnd.dd.n, rnd.dd.ucap)))
            tab.next_round()
        else:
            D = self.displs
            self.t.alltoallv(g, rnd.scounts, D, self.rgrads, rnd.rcounts, D, self.dim)
            self._server_apply(rnd.rcounts, resolved=True)
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
        return self.gather(rnd, keys.numel())

    def push_keys(self, keys: torch.Tensor, grads: torch.Tensor) -> None:
        """Stand-alone push of per-occurrence gradients (no pull this round).

        Duplicate keys are merged (summed) on the worker first.  Keys unknown
        to the server are created with the initialiser before the update (the
        reference CHECK-fails, sparsetable.h:184)."""
        keys = keys.reshape(-1)
        if keys.device != self.device:
            keys = keys.to(self.device)
        grads = grads.to(self.device)
        dd = self.dedup(keys)
        rnd = Round(dd, self.uvals)
        self.accumulate(rnd, grads)
        tab = self.table
        if self.fast1:
            sl = tab.dev_segs(dd.ucount)
            n = max(1, min(keys.numel(), dd.ucap))
            _hip().probe(tab.dt, dd.ukeys.data_ptr(), sl, n, self.slots.data_ptr(),
                         tab._init_native, 1, tab.size_ctr.data_ptr(), tab.err.data_ptr(), tab.G,
                         _stream())
            tab.push_slots(self.slots, dd.ugrad, segs=sl, max_n=n)
            tab.next_round()
        else:
            scounts, rcounts = self.t.exchange_counts(dd.ucount)
            D = self.displs
            self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
            self.t.alltoallv(dd.ugrad, scounts, D, self.rgrads, rcounts, D, self.dim)
            self._server_apply(rcounts, resolved=False)
        self.rounds += 1

    def barrier(self):
        self.t.barrier()
