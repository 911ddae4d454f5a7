"""N>1 device set-up of the round engine (parallel/engine.py): the receive
buffers, the server-merge slots and the xGMI mailbox layout handed to the C++
RoundEngine.  Split out of PSEngine as a mixin; see engine.py for the round
itself."""
from __future__ import annotations

import os

import torch


def _hip():
    from .._native import hip

    return hip()


class _ServerSlot:
    """Device buffers of one ring slot's server-side merge (N>1, GPU)."""

    def __init__(self, rows: int, P: int, dev, snapshot: bool):
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

    def ptrs(self):
        t = (self.cnt, self.bstart, self.ubase, self.unum, self.pj, self.luid, self.bkeys,
             self.slots)
        return [x.data_ptr() for x in t] + [self.snap.data_ptr() if self.snap is not None else 0,
                                            self.ucount.data_ptr()]


class DeviceSetup:
    """PSEngine mixin: the N>1 GPU buffers (``_init_dist_gpu``) and the
    collective agreement on a small int64 tensor (``_agree``)."""

    # ------------------------------------------------------------ N>1 (GPU)
    def _init_dist_gpu(self) -> None:
        """Receive buffers and server-merge slots of the N>1 device path.
        Every rank lays its buckets out as a call of ``max_keys`` keys (the
        common layout the servers merge) and sends each destination its
        per-bucket runs with the keys."""
        N, cap, d, dev, h = self.world, self.max_keys, self.dim, self.device, _hip()
        for dd in self.dedupers:
            dd.lay_n = cap
        self.Pd = h.bd_buckets(cap, N, self.dedupers[0].ndest) // N
        # record exchange: a server bucket is N runs of records sized for one
        # LDS table together (bdedup.hip bd_target), no sub-buckets — or, with
        # grouped records (rec_group), the unique layout's buckets and its
        # sub-bucket split (the sender groups each run's records by it)
        bits = h.bd_record_layout_bit() | h.bd_record_group_bit()
        self.sub = 1 if (self.records and not self.rec_group) else h.srv_sub_buckets(
            N, cap, self.dedupers[0].ndest & ~bits)
        self.Ps = self.Pd * self.sub
        # sub > 1: every source groups its runs by the servers' sub-bucket
        # and sends the offsets with them (the server reads exact ranges)
        for dd in self.dedupers:
            dd.split_for_servers(self.sub)
            if self.records:
                dd.enable_records()
        Psub = self.Pd * self.sub if self.sub > 1 else 0
        # every rank's max_keys must agree (it fixes Pd)
        mk = torch.tensor([cap, -cap], dtype=torch.int64, device=dev)
        self._agree(mk)
        if int(mk[0]) != cap or int(-mk[1]) != cap:
            raise ValueError("PSEngine: max_keys differs across ranks (the N>1 bucket layout "
                             "is a function of it)")
        rows = N * cap
        self.rvals = torch.zeros((rows, d), dtype=torch.float32, device=dev)
        # xGMI: one slot past the ring (index `depth`) for the read-only
        # lookup's rounds (PSEngine.lookup), with its own deduper
        NS = self.depth + (1 if self.xg else 0)
        self.lookup_slot = self.depth if self.xg else None
        if self.xg:
            from ..ops.dedup import Deduper

            lk = Deduper(self.max_keys, nranks=N, frag_map=self.dedupers[0].frag_map.cpu(),
                         gdim=d, device=dev, record_layout=self.records,
                         record_group=self.rec_group)
            lk.lay_n = cap
            lk.split_for_servers(self.sub)
            lk.need_ukeys = True
            self._lk_dd = lk
            # the receive buffers are the arena's mailboxes: keys + the bucket
            # runs (bases, sizes) per source, rows back, gradients
            Pd, xg = self.Pd, self.xg
            xg.setup({"keys": (NS, [cap * 8, Pd * 4, Pd * 4] + ([Psub * 4] if Psub else [])),
                      "vals": (NS, [cap * 4 * d]), "grads": (NS, [cap * 4 * d])})
            self.rkeys = [xg.region("keys", 0, q, torch.int64) for q in range(NS)]
            self.rmeta = [(xg.region("keys", 1, q, torch.int32),
                           xg.region("keys", 2, q, torch.int32)) for q in range(NS)]
            self.rsub = [xg.region("keys", 3, q, torch.int32) if Psub else None
                         for q in range(NS)]
            self.uvals = [xg.region("vals", 0, q, torch.float32, d) for q in range(NS)]
            self.rgrads = [xg.region("grads", 0, q, torch.float32, d) for q in range(NS)]
        else:
            self.rkeys = [torch.empty(rows, dtype=torch.int64, device=dev)] * self.depth
            meta = [torch.zeros(2 * N * self.Pd, dtype=torch.int32, device=dev)
                    for _ in range(self.depth)]
            self.rmeta = [(m[:N * self.Pd], m[N * self.Pd:]) for m in meta]
            self.rsub = [torch.zeros(N * Psub, dtype=torch.int32, device=dev) if Psub else None
                         for _ in range(self.depth)]
            self.rgrads = [torch.empty((rows, d), dtype=torch.float32, device=dev)] * self.depth
        # region buckets (claimed server pulls, table.hip k_pull_claim_bk):
        # every shard has the same region count (same capacity), agreed with
        # the worker-only ranks, whose buckets must follow the same regions
        own = getattr(self.table, "rbits", 0) if self.table is not None else None
        rb = torch.tensor([99 if own is None else own, 1 if own is None else -own],
                          dtype=torch.int64, device=dev)
        self._agree(rb)
        lo, hi = int(rb[0]), -int(rb[1])
        self.srv_rbits = lo if (lo == hi and 0 < lo < 99 and
                                os.environ.get("SS_CLAIM", "1") != "0") else 0
        self.claim = bool(self.srv_rbits and self.xg)
        if self.claim:
            for dd in self.dedupers:
                dd.rbits = self.srv_rbits
        # the server half of every round (keys in, merge, lookup, rows out;
        # gradients in, merge + update) on its own highest-priority stream: a
        # slow compute on this rank's main stream does not hold up the rows
        # every peer waits for (SS_SERVER_STREAM=0: on the main stream)
        self.server_stream = None
        # auto (default): only when every rank has its own device — ranks
        # sharing one GPU (one-GPU rehearsals) oversubscribe its hardware
        # queues with a third stream per process (8 ranks: 21.3 vs 8.35 ms
        # per 8-rank step; 4 ranks 4.62 vs 4.41)
        ss_env = os.environ.get("SS_SERVER_STREAM", "auto")
        if self.table is not None and self.xg is not None and \
                (ss_env == "1" or (ss_env == "auto" and not self.shared_device)):
            other = getattr(self, "_streams_of", None)
            lo_prio, hi_prio = torch.cuda.Stream.priority_range()
            self.server_stream = (
                (getattr(other, "server_stream", None) or getattr(other, "_server_stream_off", None))
                if other is not None else None) or \
                torch.cuda.Stream(device=dev, priority=min(lo_prio, hi_prio))
        self.srv = None
        self.srv_ahead = os.environ.get("SS_SRV_AHEAD", "1") != "0"
        self._route_srv = None  # how the last route ran the keys-in (srv_ahead)
        if self.table is not None:
            self.svals = torch.empty((rows, d), dtype=torch.float32, device=dev)
            self.sgrad = torch.empty((rows, d), dtype=torch.float32, device=dev)
            # SS_SRV_STAGE=1: a cached copy of the received gradient rows (the
            # mailboxes are uncached; the server merge gathers per received
            # position), streamed out of the mailbox before the merge.
            # Measured neutral with 4 and 8 ranks on one GPU (4.14-4.33 vs
            # 4.17-4.24 ms, 8.23-8.26 vs 8.23-8.37): off by default
            self.gstage = (torch.empty((rows, d), dtype=torch.float32, device=dev)
                           if self.xg is not None and N > 1 and
                           os.environ.get("SS_SRV_STAGE", "0") == "1" else None)
            self.srv_err = torch.zeros(1, dtype=torch.int32, device=dev)
            snap_ok = bool(getattr(self.table, "snapshot_ok", False))
            self.srv = [_ServerSlot(rows, self.Ps, dev, snap_ok and q < self.depth)
                        for q in range(NS)]
        # record exchange: the rows of this rank's own records are written by
        # its own server into a cached buffer per ring slot (not the uncached
        # vals arena, which only peers need), and their gradients are read by
        # the server merge straight from the worker's per-sample gradient
        # through spj — never written out per occurrence (SS_REC_OCC=arena:
        # both through the arena, as the peers' records)
        self.own_vals = None
        if (self.records and self.table is not None and
                self.server_ranks == list(range(N)) and
                os.environ.get("SS_REC_OCC", "own") == "own" and
                os.environ.get("SS_XGMI_SELF", "1") != "0"):
            self.own_vals = [torch.empty((cap, d), dtype=torch.float32, device=dev)
                             for _ in range(self.depth)]
        if self.xg:
            D = NS
            self.native.set_xgmi([[self.xg.arena_of(c, q) for c in ("keys", "vals", "grads")]
                                  for q in range(D)],
                                 [sum((list(self.xg.layout("keys", p, q))
                                       for p in range(4 if Psub else 3)), []) for q in range(D)],
                                 [list(self.xg.layout("vals", 0, q)) for q in range(D)],
                                 [list(self.xg.layout("grads", 0, q)) for q in range(D)],
                                 N, self.rank, self.Pd, self.sub, cap, d, self.xg.bpp,
                                 self.xg.timeout_s)
            # a closed transport frees its arenas: the engine forgets them first
            self.xg._close_hooks.append(self.native.clear_xgmi)
            for q in range(D):
                if self.srv is not None:
                    self.native.set_server_slot(q, self.srv[q].ptrs())
            self._nodt = h.DevTable(0, 1, 16, 8, 1, 2)  # a rank without a shard
            self._noop = h.OptParams()
            self._noip = h.InitParams()

    def _agree(self, t: torch.Tensor) -> None:
        """min-all-reduce of a small int64 tensor over the data transport."""
        if self.world == 1:
            return
        self.t.allreduce_(t, "min")
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()
