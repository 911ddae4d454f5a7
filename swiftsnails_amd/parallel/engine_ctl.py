"""Read-only access and control calls of the round engine
(parallel/engine.py): the collective read-only lookup used to evaluate a
sharded model, the host-level agreements (max over ranks, termination) and the
health checks.  A PSEngine mixin."""
from __future__ import annotations

import numpy as np
import torch


class EngineControl:
    def max_over_ranks(self, value: float) -> float:
        """max of a host float over the ranks (control plane; syncs)."""
        if self.world == 1:
            return float(value)
        dev = self.device if (self.gpu and not hasattr(self.t, "aux")) else "cpu"
        t = torch.tensor([value], dtype=torch.float32 if dev != "cpu" else torch.float64,
                         device=dev)
        self.t.allreduce_(t, "max")
        return float(t.item())

    def layout_info(self) -> dict:
        """The round layout this rank runs (bench.py / the launcher put it in
        their JSON, so a number says which layout produced it): ring depth,
        the server stream, the N>1 bucket layout (occurrences per source
        bucket, server sub-buckets), claimed server inserts and the region
        bits they rely on."""
        info = {"depth": int(self.depth), "fast1": bool(getattr(self, "fast1", False))}
        if not (self.gpu and self.dist):
            return info
        from .engine import _hip

        h = _hip()
        info.update({
            "server_stream": getattr(self, "server_stream", None) is not None,
            # SS_BD_TARGET_DIST (the N>1 source-bucket target), and the target
            # this layout actually uses (a one-rank layout takes SS_BD_TARGET)
            "bd_target_dist": int(h.bd_target_dist()),
            "bucket_target": int(h.bd_target_for(self.world, bool(getattr(self, "records", False))
                                                 and not getattr(self, "rec_group", False))),
            "record_group": bool(getattr(self, "rec_group", False)),
            "buckets_per_dest": int(getattr(self, "Pd", 0)),
            "srv_sub_buckets": int(getattr(self, "sub", 1)),
            "claim": bool(getattr(self, "claim", False)),
            "srv_rbits": int(getattr(self, "srv_rbits", 0)),
            "srv_ahead": bool(getattr(self, "srv_ahead", False)),
            "shared_device": bool(self.shared_device),
        })
        return info

    def set_server_stream(self, on: bool) -> bool:
        """Run the server half of later rounds on the server stream (``on``)
        or on the caller's streams.  Synchronises the device first, so no
        round issued before the switch can reorder against one issued after
        it (calibration only: PipelinedWorker.calibrate_server_stream).
        Returns whether the server stream is in use."""
        if not self.gpu:
            return False
        cur = getattr(self, "server_stream", None)
        if on == (cur is not None):
            return on
        torch.cuda.synchronize(self.device)
        if not on:
            self._server_stream_off = cur
            self.server_stream = None
        else:
            self.server_stream = getattr(self, "_server_stream_off", None)
        return self.server_stream is not None

    # ------------------------------------------------------------ read-only
    def lookup(self, keys: torch.Tensor) -> torch.Tensor:
        """Collective READ-ONLY pull: rows [n, dim] of ``keys`` (in order)
        from whichever shard owns each key; a key no shard holds reads as
        zeros and is NOT inserted, and nothing is pushed — the reference's
        pull_with_barrier of any key from every server by any worker
        (/root/reference/src/core/parameter/global_pull_access.h:40-55), for
        evaluating a sharded model.  Every rank calls it together (a rank
        without keys passes an empty tensor).  It runs on the gloo control
        plane (host-staged): an evaluation path, not a training one."""
        keys = keys.reshape(-1)
        if self.world == 1:
            return self._read_rows(keys.to(self.device)).to(keys.device)
        if self.gpu and getattr(self, "lookup_slot", None) is not None and \
                not getattr(self, "graphed", False) and \
                not (self.table is not None and self.table.custom_pull):
            return self._lookup_xgmi(keys)
        import torch.distributed as dist

        from .router import route_keys_np

        N = self.world
        u, inv = torch.unique(keys.cpu(), return_inverse=True)
        dest = route_keys_np(u.numpy().view(np.uint64), self.frag_map) if len(u) else \
            np.zeros(0, np.int64)
        order = torch.from_numpy(np.argsort(dest, kind="stable"))
        scount = torch.from_numpy(np.bincount(dest, minlength=N).astype(np.int64))
        rcount = torch.empty(N, dtype=torch.int64)
        dist.all_to_all_single(rcount, scount)
        sk = u[order].contiguous()
        rk = torch.empty(int(rcount.sum()), dtype=torch.int64)
        dist.all_to_all_single(rk, sk, rcount.tolist(), scount.tolist())
        rows = (self._read_rows(rk.to(self.device)).cpu().contiguous() if self.table is not None
                else torch.zeros((len(rk), self.dim), dtype=torch.float32))
        back = torch.empty((len(sk), self.dim), dtype=torch.float32)
        dist.all_to_all_single(back.view(-1), rows.view(-1), [c * self.dim for c in scount.tolist()],
                               [c * self.dim for c in rcount.tolist()])
        out_u = torch.empty_like(back)
        out_u[order] = back
        return out_u[inv].to(keys.device)

    def _lookup_xgmi(self, keys: torch.Tensor) -> torch.Tensor:
        """The collective read-only lookup on the device (N>1 over the xGMI
        mailboxes): the same round as a training pull — dedup + route into
        per-server bucket runs, keys into the servers' mailboxes, every
        server's merge of the sources' keys — but the servers LOOK UP their
        distinct keys without inserting (table.hip k_lookup_bk, zeros for
        absent keys) and nothing is pushed; rows come back through the vals
        mailboxes and are gathered into occurrence order.  It runs on the
        reserved slot past the route ring, so a pipeline holding ring slots
        (routed / pulled-ahead rounds) is not disturbed.  Batches of up to
        ``max_keys`` keys per rank per round; longer key lists take several
        rounds (every rank the same number: agreed first)."""
        from .engine import FREE, _hip

        h = _hip()
        n = int(keys.numel())
        cap = self.max_keys
        nr = torch.tensor([-(-n // cap)], dtype=torch.int64)
        self.t.allreduce_(nr, "max")  # control plane (gloo): every rank the same rounds
        rounds = int(nr.item())
        q, tab, dd = self.lookup_slot, self.table, self._lk_dd
        dd.materialize_inv, dd.need_bkt, dd.need_pos = True, True, True
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        kd = keys.to(self.device, torch.int64)
        st = self.raw_stream()
        if getattr(self, "_claimed", None):
            self._commit_claimed(st)
        # every enqueued round first — server updates on the server stream and
        # pulled-ahead server halves on the pull / route streams use the same
        # svals / rvals buffers as this lookup's round (an evaluation path:
        # a device sync is cheap next to it)
        torch.cuda.synchronize(self.device)
        ss = getattr(self, "server_stream", None)
        main = torch.cuda.current_stream(self.device)
        S = self.srv[q] if self.srv is not None else None
        for i in range(rounds):
            part = kd[i * cap:(i + 1) * cap]
            m = int(part.numel())
            self.native.wait(FREE, q, st, 0)  # the previous lookup round is done
            r = dd(part, stream=st)
            ub, un = dd.run_tables(self.Pd)
            us = dd.sub_table(self.Pd).data_ptr() if dd.msub > 1 else 0
            self.native.route_end(q, 0, st, r.ukeys.data_ptr(), r.ucount.data_ptr(),
                                  ub.data_ptr(), un.data_ptr(), us, False, tab is not None,
                                  self.rkeys[q].data_ptr(), self.rmeta[q][0].data_ptr(),
                                  self.rmeta[q][1].data_ptr(),
                                  self.srv_err.data_ptr() if tab is not None else 0)
            self.native.pull_xgmi(q, 0, st, False, -1, False, S is not None,
                                  tab.dt if S else self._nodt,
                                  tab._init_native if S else self._noip,
                                  tab.size_ctr.data_ptr() if S else 0,
                                  tab.err.data_ptr() if S else 0, tab.G if S else 1,
                                  self.rkeys[q].data_ptr(), self.rmeta[q][0].data_ptr(),
                                  self.rmeta[q][1].data_ptr(),
                                  self.srv_err.data_ptr() if S else 0,
                                  self.svals.data_ptr() if S else 0, self.rvals.data_ptr(),
                                  False, r.ucount.data_ptr(), [], False, False, False, 0, 0)
            if m:
                h.gather_rows(self.uvals[q].data_ptr(), r.inv.data_ptr(), m, self.dim,
                              out[i * cap:i * cap + m].data_ptr(), st)
            self.native.record(FREE, q, st, 0)
        if ss is not None:  # later server updates after the lookup read the rows
            ss.wait_stream(main)
        self.metrics.add(lookup_keys=n)
        return out.to(keys.device)

    def _read_rows(self, keys: torch.Tensor) -> torch.Tensor:
        tab = self.table
        if len(keys) == 0:
            return torch.zeros((0, self.dim), dtype=torch.float32, device=keys.device)
        if self.gpu:
            if getattr(self, "_claimed", None):  # a claimed pull not pushed yet
                self._commit_claimed(self.raw_stream())
            torch.cuda.synchronize(self.device)  # every enqueued update applied
            return tab.pull(keys, insert=False)[0]
        rows, found = tab._t.get_rows(keys.numpy().view(np.uint64))
        r = torch.from_numpy(np.ascontiguousarray(rows[:, :self.dim]))
        r[torch.from_numpy(found == 0)] = 0.0
        return r

    # ------------------------------------------------------------ control
    def barrier(self):
        self.t.barrier()

    def all_done(self, local_done: bool) -> bool:
        """Collective termination: True once every rank reports done (every
        rank calls it at the same rounds; syncs).  A rank that finished early
        keeps serving rounds with an empty key set until then — the
        reference's master waiting for every worker's WORKER_FINISH_WORK
        before stopping the servers (master/terminate.h:44-62)."""
        self.poll()
        if self.world == 1:
            return bool(local_done)
        dev = self.device if (self.gpu and not hasattr(self.t, "aux")) else "cpu"
        flag = torch.tensor([1 if local_done else 0], dtype=torch.int64, device=dev)
        self.t.allreduce_(flag, "min")
        return int(flag.item()) == 1

    def poll(self) -> None:
        """Cheap per-round health check, no device sync: raises if a mailbox
        wait has timed out or seen a stale round tag (host-mapped error
        words of the xGMI transport)."""
        if self.xg is not None:
            self.xg.poll_error()

    def check(self) -> None:
        """Raise on a sticky device-side error (syncs): an overflowed dedup
        or server-merge bucket, a full / misused table, a mailbox peer that
        never arrived.  Called at the end of bench.py, every periodic backup
        and PSContext.finish."""
        for d in self.dedupers:
            chk = getattr(d, "check", None)
            if chk is not None:
                chk()
        if getattr(self, "srv", None) is not None and int(self.srv_err.item()) != 0:
            from ..ops.dedup import DedupOverflowError

            e = int(self.srv_err.item())
            # the fullest server bucket of each ring slot (received keys,
            # distinct keys) — what the sub-bucket split was sized against
            sizes = []
            for S in self.srv[:self.depth]:
                bs = S.bstart.to(torch.int64)
                if bs.numel() > 1:
                    sizes.append((int((bs[1:] - bs[:-1]).max()), int(S.unum.max())))
            raise DedupOverflowError(
                "server merge: a bucket of received keys "
                + ("overflowed its LDS table" if e & 1 else "")
                + (" / " if e & 3 == 3 else "")
                + ("disagreed with the sources' run tables" if e & 2 else "")
                + f" (err {e}; {self.sub} sub-buckets per bucket; fullest bucket per slot "
                f"(received, distinct): {sizes})")
        chk = getattr(self.table, "check", None) if self.table is not None else None
        if chk is not None:
            chk()
        if self.xg is not None:
            self.xg.check()
