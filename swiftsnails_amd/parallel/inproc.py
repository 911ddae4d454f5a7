"""In-process multi-rank transport: a world of N ranks as N threads of one process.

The data plane of a multi-GPU job is RCCL (``RcclTransport``), which refuses
two ranks on one device, and the multi-process rehearsal on one GPU
(``TorchDistTransport`` over gloo) stages every exchange through the host.
This transport runs the N>1 engine path of N ranks — each with its own
table shard, ring buffers, route / main / pull streams and three
communicators — on ONE device, exchanging rows device-to-device with
collective semantics:

* every rank enqueues its side of an exchange on its current stream; the
  call is collective (all ranks of the group make the same calls in the same
  order, like the RCCL communicator it stands in for);
* a receiver's stream waits for the senders' events, copies its incoming
  segments, and the exchange completes on each rank's stream only once all
  peers have finished reading that rank's send buffer — what an
  ``ncclGroupStart`` … ``ncclGroupEnd`` of send/recv pairs guarantees.

Used by ``tools/rehearse_world.py`` (the bench configuration at N = 8 on one
MI355X: shard sizing, dedup bucket sizing, pull-ahead ordering, split roles)
and by the tests.  On CPU tensors the same code runs without streams.

Reference parity: the reference's only distributed test is a self-loopback
``Transfer`` in one process (/root/reference/src/unitest/core/transfer/
transfer_test.h:13-80); SURVEY §4 asks for "a single-process multi-rank fake
... N HIP streams on 1 GPU" — this is that fake, at the engine level.
"""
from __future__ import annotations

import threading
from typing import Optional, Sequence

import torch

from .transport import CountsHandle, Transport


class InprocGroup:
    """Rendezvous of ``world`` rank threads (one per communicator)."""

    def __init__(self, world: int, timeout: float = 600.0):
        self.world = int(world)
        self._bar = threading.Barrier(self.world, timeout=timeout)
        self._slots: list = [None] * self.world

    def allgather(self, rank: int, obj) -> list:
        """Every rank's ``obj``, in rank order (a host-side collective)."""
        self._slots[rank] = obj
        self._bar.wait()
        out = list(self._slots)
        self._bar.wait()  # nobody overwrites a slot before all have read it
        return out

    def abort(self) -> None:
        self._bar.abort()

    def transports(self, device=None) -> list["InprocTransport"]:
        return [InprocTransport(self, r, device) for r in range(self.world)]


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


class InprocTransport(Transport):
    """One rank's endpoint of an ``InprocGroup``."""

    def __init__(self, group: InprocGroup, rank: int, device=None):
        self.group, self.rank, self.world = group, int(rank), group.world
        self.device = torch.device(device) if device is not None else None

    # ------------------------------------------------------------ helpers
    def _ready_event(self, gpu: bool):
        if not gpu:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        return ev

    def _finish(self, gpu: bool) -> None:
        """Complete a collective: this rank's stream continues only after
        every peer's stream has consumed this rank's send buffer."""
        done = self._ready_event(gpu)
        evs = self.group.allgather(self.rank, done)
        if gpu:
            st = torch.cuda.current_stream()
            for p, e in enumerate(evs):
                if p != self.rank:
                    st.wait_event(e)

    # ------------------------------------------------------------ Transport
    def exchange_counts(self, send_counts: torch.Tensor):
        return self.exchange_counts_async(send_counts).wait()

    def exchange_counts_async(self, send_counts: torch.Tensor, pinned: Optional[torch.Tensor] = None,
                              stream=None) -> CountsHandle:
        gpu = _is_gpu(send_counts)
        if not gpu:
            s = send_counts.to(torch.int64).reshape(-1).clone()
            peers = self.group.allgather(self.rank, s)
            r = torch.stack([peers[p][self.rank] for p in range(self.world)])
            self.group.allgather(self.rank, None)
            return CountsHandle(s.numpy().copy(), r.numpy().copy())
        st = stream or torch.cuda.current_stream()
        with torch.cuda.stream(st):
            s = send_counts.to(torch.int64).reshape(-1).contiguous()
            recv = torch.empty(self.world, dtype=torch.int64, device=s.device)
            self.alltoallv(s, [1] * self.world, list(range(self.world)), recv,
                           [1] * self.world, list(range(self.world)), 1)
            pin = pinned if pinned is not None else torch.empty(
                2 * self.world, dtype=torch.int64, pin_memory=True)
            pin[:self.world].copy_(s, non_blocking=True)
            pin[self.world:2 * self.world].copy_(recv, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        return CountsHandle(event=ev, pinned=pin, world=self.world)

    def alltoallv(self, send: torch.Tensor, scounts: Sequence[int], sdispls: Sequence[int],
                  recv: torch.Tensor, rcounts: Sequence[int], rdispls: Sequence[int],
                  row_elems: int = 1) -> None:
        gpu = _is_gpu(send)
        me, re = self.rank, int(row_elems)
        sc = [int(x) for x in scounts]
        sd = [int(x) for x in sdispls]
        peers = self.group.allgather(
            me, (send.view(-1), sc, sd, self._ready_event(gpu)))
        rflat = recv.view(-1)
        if gpu:
            st = torch.cuda.current_stream()
            for p, (_, _, _, e) in enumerate(peers):
                if p != me:
                    st.wait_event(e)
        for p, (pflat, psc, psd, _) in enumerate(peers):
            c = psc[me]
            if c != int(rcounts[p]):
                raise RuntimeError(f"inproc alltoallv: rank {p} sends {c} rows to rank {me}, "
                                   f"which expects {int(rcounts[p])}")
            if c:
                s0, r0 = psd[me] * re, int(rdispls[p]) * re
                rflat[r0:r0 + c * re].copy_(pflat[s0:s0 + c * re], non_blocking=True)
        self._finish(gpu)

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        gpu = _is_gpu(t)
        peers = self.group.allgather(self.rank, (t, self._ready_event(gpu)))
        if gpu:
            st = torch.cuda.current_stream()
            for p, (_, e) in enumerate(peers):
                if p != self.rank:
                    st.wait_event(e)
        vals = torch.stack([x for x, _ in peers])
        red = {"sum": vals.sum(0), "max": vals.max(0).values, "min": vals.min(0).values}[op]
        # everyone has read every input before anyone overwrites its own
        self._finish(gpu)
        t.copy_(red)
        return t

    def barrier(self) -> None:
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
        self.group.allgather(self.rank, None)

    def abort(self) -> None:
        self.group.abort()


def run_ranks(world: int, fn, *args, timeout: float = 1800.0) -> list:
    """Run ``fn(rank, *args)`` on ``world`` threads; returns the results in
    rank order and re-raises the first failure (after unblocking the rest:
    ``fn`` should abort its groups on error, see ``InprocGroup.abort``)."""
    out: list = [None] * world
    err: list = [None] * world

    def body(r):
        try:
            out[r] = fn(r, *args)
        except BaseException as e:  # noqa: BLE001 - reported below
            err[r] = e

    ths = [threading.Thread(target=body, args=(r,), name=f"rank{r}", daemon=True)
           for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
    if any(t.is_alive() for t in ths):
        raise TimeoutError(f"inproc ranks still running after {timeout}s")
    first = next((e for e in err if e is not None and
                  not isinstance(e, threading.BrokenBarrierError)), None)
    first = first or next((e for e in err if e is not None), None)
    if first is not None:
        raise first
    return out
