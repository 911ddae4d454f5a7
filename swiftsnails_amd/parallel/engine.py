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
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops.dedup import DedupResult, Deduper
from .router import HashFrag
from .transport import LoopbackTransport, Transport


@dataclass
class Round:
    dd: DedupResult
    uvals: torch.Tensor                   # [N*ucap, dim] pulled rows, unique-key order
    slots: Optional[torch.Tensor] = None  # world-1 path: table slots of ukeys
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


class PSEngine:
    """Worker+server round engine for one rank.

    table         : this rank's shard (``HbmTable``) or None when not a server
    transport     : data-plane transport (RCCL on MI355X)
    max_keys      : max key occurrences per pull on this rank
    server_ranks  : ranks that host a shard (default: all — colocated mode)
    frag_num      : number of hash fragments (reference config ``frag_num``)
    """

    def __init__(self, table, transport: Optional[Transport], max_keys: int, dim: int,
                 frag_num: int = 0, server_ranks: Optional[Sequence[int]] = None, device=None):
        self.t = transport or LoopbackTransport()
        self.rank, self.world = self.t.rank, self.t.world
        self.table = table
        self.dim = int(dim)
        self.device = torch.device(device) if device is not None else (
            table.device if table is not None else torch.device("cuda"))
        self.server_ranks = list(server_ranks) if server_ranks is not None else list(
            range(self.world))
        if (table is not None) != (self.rank in self.server_ranks):
            raise ValueError("a rank owns a table iff it is listed in server_ranks")
        frag_num = frag_num or max(1024, 8 * len(self.server_ranks))
        self.router = HashFrag(len(self.server_ranks), frag_num)
        self.frag_map = self.router.rank_map(self.server_ranks)
        self.max_keys = int(max_keys)
        self.dedup = Deduper(self.max_keys, nranks=self.world,
                             frag_map=torch.from_numpy(self.frag_map.astype(np.int32)),
                             gdim=self.dim, device=self.device)
        N, cap, d = self.world, self.max_keys, self.dim
        dev = self.device
        self.uvals = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
        if self.world == 1:
            self.slots = torch.empty(cap, dtype=torch.int64, device=dev)
        else:
            # server-side receive buffers: one fixed segment per source rank
            self.rkeys = torch.empty(N * cap, dtype=torch.int64, device=dev)
            self.rslots = torch.empty(N * cap, dtype=torch.int64, device=dev)
            self.rvals = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
            self.rgrads = torch.empty((N * cap, d), dtype=torch.float32, device=dev)
        self.displs = [r * cap for r in range(N)]
        self.rounds = 0

    # ------------------------------------------------------------------ pull
    def pull(self, keys: torch.Tensor) -> Round:
        keys = keys.reshape(-1)
        dd = self.dedup(keys)
        tab = self.table
        if self.world == 1:
            tab.pull(dd.ukeys, insert=True, unique=True, out=self.uvals, slots=self.slots,
                     segs=tab.dev_segs(dd.ucount), max_n=min(keys.numel(), dd.ucap))
            return Round(dd, self.uvals, slots=self.slots)
        scounts, rcounts = self.t.exchange_counts(dd.ucount)
        D = self.displs
        self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
        nrecv = int(rcounts.sum())
        if tab is not None and nrecv:
            tab.pull(self.rkeys, insert=True, unique=False, out=self.rvals, slots=self.rslots,
                     segs=tab.segs(D, rcounts), max_n=nrecv)
        self.t.alltoallv(self.rvals, rcounts, D, self.uvals, scounts, D, self.dim)
        return Round(dd, self.uvals, scounts=scounts, rcounts=rcounts,
                     stats={"sent": int(scounts.sum()), "recv": nrecv})

    # ------------------------------------------------------------------ push
    def push(self, rnd: Round, grads: Optional[torch.Tensor] = None) -> None:
        g = rnd.ugrad if grads is None else grads
        tab = self.table
        if self.world == 1:
            tab.push_slots(rnd.slots, g, segs=tab.dev_segs(rnd.dd.ucount),
                           max_n=min(rnd.dd.n, rnd.dd.ucap))
        else:
            D = self.displs
            self.t.alltoallv(g, rnd.scounts, D, self.rgrads, rnd.rcounts, D, self.dim)
            if tab is not None:
                # one launch per source rank, in rank order: duplicate keys sent
                # by different workers are applied sequentially (no lost updates)
                for s in range(self.world):
                    c = int(rnd.rcounts[s])
                    if c:
                        tab.push_slots(self.rslots, self.rgrads, segs=tab.segs([D[s]], [c]),
                                       max_n=c)
        if tab is not None:
            tab.next_round()
        rnd.pushed = True
        self.rounds += 1

    # ------------------------------------------------------------ utilities
    def pull_dense(self, keys: torch.Tensor) -> torch.Tensor:
        """Pull rows for `keys` in occurrence order ([n, dim])."""
        rnd = self.pull(keys)
        from .._native import hip

        out = torch.empty((keys.numel(), self.dim), dtype=torch.float32, device=self.device)
        hip().gather_rows(rnd.uvals.data_ptr(), rnd.inv.data_ptr(), keys.numel(), self.dim,
                          out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out

    def push_keys(self, keys: torch.Tensor, grads: torch.Tensor) -> None:
        """Stand-alone push of per-occurrence gradients (no pull this round).

        Duplicate keys are merged (summed) on the worker first — the
        reference's ``merge_push_value`` (sparse_access_method.h:39-40).  Keys
        unknown to the server are created with the initialiser before the
        update (the reference CHECK-fails, sparsetable.h:184)."""
        from .._native import hip

        keys = keys.reshape(-1)
        grads = grads.reshape(keys.numel(), self.dim).contiguous()
        dd = self.dedup(keys)
        st = torch.cuda.current_stream().cuda_stream
        hip().scatter_add_rows(grads.data_ptr(), dd.inv.data_ptr(), keys.numel(), self.dim,
                               dd.ugrad.data_ptr(), st)
        tab = self.table
        if self.world == 1:
            sl = tab.dev_segs(dd.ucount)
            n = min(keys.numel(), dd.ucap)
            hip().probe(tab.dt, dd.ukeys.data_ptr(), sl, n, self.slots.data_ptr(),
                        tab._init_native, 1, tab.size_ctr.data_ptr(), tab.err.data_ptr(), tab.G,
                        st)
            tab.push_slots(self.slots, dd.ugrad, segs=sl, max_n=n)
            tab.next_round()
            self.rounds += 1
            return
        scounts, rcounts = self.t.exchange_counts(dd.ucount)
        D = self.displs
        self.t.alltoallv(dd.ukeys, scounts, D, self.rkeys, rcounts, D, 1)
        self.t.alltoallv(dd.ugrad, scounts, D, self.rgrads, rcounts, D, self.dim)
        if tab is not None:
            for s in range(self.world):
                c = int(rcounts[s])
                if c:
                    sl = tab.segs([D[s]], [c])
                    hip().probe(tab.dt, self.rkeys.data_ptr(), sl, c, self.rslots.data_ptr(),
                                tab._init_native, 1, tab.size_ctr.data_ptr(),
                                tab.err.data_ptr(), tab.G, st)
                    tab.push_slots(self.rslots, self.rgrads, segs=sl, max_n=c)
            tab.next_round()
        self.rounds += 1
