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

            raise DedupOverflowError("server merge: a bucket of received keys overflowed its "
                                     "LDS table")
        chk = getattr(self.table, "check", None) if self.table is not None else None
        if chk is not None:
            chk()
        if self.xg is not None:
            self.xg.check()
