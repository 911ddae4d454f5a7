"""Host-count rounds of the PS engine: the exchanges whose transport needs
every alltoallv's counts on the host — RCCL (grouped send/recv), gloo /
torch.distributed, and the CPU engine (``HostTable`` shards) that tests the
multi-rank logic without GPUs.

The device-count paths — one GPU, and N>1 over the xGMI mailboxes — are
driven by the C++ round engine (``csrc/hip/round_engine.cpp``) from
``parallel/engine.py``; this mixin supplies the rest of ``PSEngine``: the
count exchange of the route stage, the keys / rows / gradients alltoallv of
the pull and push stages, and the server merge issued from Python (GPU:
the same server.hip kernels; CPU: ``torch.unique``).  Reference call stacks:
/root/reference/src/core/parameter/global_pull_access.h:40-120 and
global_push_access.h:36-149 (grouping per server, one request per server,
server-side ``get_pull_value`` / ``merge_push_value`` + ``apply_push_value``).
"""
from __future__ import annotations

import numpy as np
import torch

from .transport import Transport


def _hip():
    from .._native import hip

    return hip()


class HostRounds:
    """Mixin of ``PSEngine`` (uses its buffers and metrics)."""

    # ------------------------------------------------------------ stage 1
    def _route_counts(self, dd, slot: int, rs):
        """Route-stream exchange of this round's counts (async, host-visible
        later) and of the per-bucket runs every destination merges by."""
        ub, un = dd.owner.run_tables(self.Pd)
        Pd, N = self.Pd, self.world
        dsp = [r * Pd for r in range(N)]
        counts = self.ct.exchange_counts_async(dd.ucount, pinned=self._pins[slot], stream=rs)
        mb, mn = self.rmeta[slot]
        fixed = [Pd] * N
        self.ct.alltoallv(ub, fixed, dsp, mb, fixed, dsp, 1)
        self.ct.alltoallv(un, fixed, dsp, mn, fixed, dsp, 1)
        if self.rsub[slot] is not None:  # sub-bucket offsets of the runs
            m = self.Pd * self.sub
            fm, dm = [m] * N, [r * m for r in range(N)]
            self.ct.alltoallv(dd.owner.sub_table(Pd), fm, dm, self.rsub[slot], fm, dm, 1)
        return counts

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
                    self.srv_err.data_ptr(), st,
                    self.rsub[slot].data_ptr() if self.rsub[slot] is not None else 0)
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

    def _pull_counts(self, r, uv: torch.Tensor, tr: Transport, stream):
        """Keys out, server merge + lookup, rows back (host counts)."""
        from .engine import Round

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

    # ------------------------------------------------------------ stage 3
    def _server_push_gpu(self, slot: int) -> None:
        """Merge the gradients all sources pushed for each distinct key and
        update every such row once (fused unless a tensor-code rule runs)."""
        tab = self.table
        if tab is None:
            return
        from ..utils.streams import current_raw

        h, S, st = _hip(), self.srv[slot], current_raw(self._dix)
        args = (self.Ps, S.bstart.data_ptr(), S.ubase.data_ptr(), S.unum.data_ptr(),
                S.pj.data_ptr(), S.luid.data_ptr(), self.rgrads[slot].data_ptr())
        kind = self._server_update_kind()
        if kind is not None:
            h.srv_merge(*args, 0, self.dim, tab.dt, S.slots.data_ptr(),
                        S.snap.data_ptr() if S.snap_valid and kind == "scalar" else 0,
                        tab.opt.native(), st)
        else:
            h.srv_merge(*args, self.sgrad.data_ptr(), self.dim, st=st)
            self._apply_merged(slot)
        tab.version += 1

    def _apply_merged(self, slot: int) -> None:
        """Update from merged rows (``sgrad``): a tensor-code rule, or the
        apply kernel for optimizers / row formats the merge does not fuse."""
        tab, S = self.table, self.srv[slot]
        if tab.push_fn is not None:
            u = int(S.ucount.item())  # a tensor rule runs on host-sized tensors
            tab.apply_custom(S.slots[:u], self.sgrad[:u])
        else:
            tab.push_slots(S.slots, self.sgrad, segs=tab.dev_segs(S.ucount),
                           max_n=self.world * self.max_keys)

    def _server_push_cpu(self, rnd) -> None:
        tab = self.table
        if tab is None or rnd.server is None:
            return
        idx, uk, inv = rnd.server
        g = torch.zeros((uk.numel(), self.dim), dtype=torch.float32)
        g.index_add_(0, inv, self.rgrads[torch.from_numpy(idx)])
        tab.push_keys(uk, g)

    def _push_counts(self, rnd, g: torch.Tensor) -> None:
        """Gradient rows out (host counts), then the server merge + update."""
        D = self.displs
        self.t.alltoallv(g, rnd.scounts, D, self.rgrads[rnd.slot] if self.gpu else self.rgrads,
                         rnd.rcounts, D, self.dim)
        if self.gpu:
            self._server_push_gpu(rnd.slot)
        else:
            self._server_push_cpu(rnd)

    # ------------------------------------------------------- occurrence API
    def gather(self, rnd, n=None) -> torch.Tensor:
        """Rows in occurrence order ([n, dim]) from a pulled round."""
        n = rnd.dd.n if n is None else n
        if self.gpu:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
            _hip().gather_rows(rnd.uvals.data_ptr(), rnd.inv.data_ptr(), n, self.dim,
                               out.data_ptr(), self.raw_stream())
            return out
        return rnd.uvals[rnd.inv[:n].long()]

    def accumulate(self, rnd, grads: torch.Tensor) -> None:
        """Add per-occurrence gradients into the round's unique-key rows
        (the reference's merge_push_value, sparse_access_method.h:39-40)."""
        grads = grads.reshape(rnd.dd.n, self.dim).contiguous()
        if self.gpu:
            _hip().scatter_add_rows(grads.data_ptr(), rnd.inv.data_ptr(), rnd.dd.n, self.dim,
                                    rnd.ugrad.data_ptr(), self.raw_stream())
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
        from .engine import Round

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
            self._wait_ev(0, r, self.raw_stream())
        dd = r.dd
        if self.fast1:
            rnd = Round(dd, self.uvals[r.slot], r.slot)
            self.accumulate(rnd, grads.to(self.device))
            tab = self.table
            sl = tab.dev_segs(dd.ucount)
            n = max(1, min(dd.n, dd.ucap))
            s = self.slots[r.slot]
            _hip().probe(tab.dt, dd.ukeys.data_ptr(), sl, n, s.data_ptr(), tab._init_native, 1,
                         tab.size_ctr.data_ptr(), tab.err.data_ptr(), tab.G, self.raw_stream())
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
        rnd = self._pull_stage(r, self.uvals[r.slot], self.raw_stream() if self.gpu else None,
                               ahead=False)
        self.accumulate(rnd, grads.to(self.device))
        self._push(rnd)
