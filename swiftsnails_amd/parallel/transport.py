"""Data-plane transports for the collective round engine.

The reference's transport is ZeroMQ PUSH/PULL over TCP with a per-message RPC
(/root/reference/src/core/transfer/transfer.h:75-225).  Here one pull or push
*round* is a small set of alltoallv exchanges between all ranks:

* ``RcclTransport``   — native RCCL communicator (``csrc/hip/comm.cpp``) over
  xGMI: grouped ncclSend/ncclRecv with per-peer displacements on a HIP stream.
  Bootstrapped with an ``ncclUniqueId`` broadcast through the torch.distributed
  store.  This is the MI355X data plane.
* ``TorchDistTransport`` — ``torch.distributed.all_to_all_single`` (gloo on
  CPU for the multi-process tests; also works over the nccl=RCCL backend).
* ``LoopbackTransport`` — world size 1 (device copies only).

All transports speak in *rows*: a buffer is a flat tensor of rows of
``row_elems`` elements; counts and displacements are in rows.
"""
from __future__ import annotations

import contextlib
import os
import sys
import threading
from abc import ABC, abstractmethod
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


class CountsHandle:
    """Result of an (possibly asynchronous) count exchange."""

    def __init__(self, s: Optional[np.ndarray] = None, r: Optional[np.ndarray] = None,
                 event=None, pinned: Optional[torch.Tensor] = None, world: int = 1):
        self._s, self._r, self.event, self.pinned, self.world = s, r, event, pinned, world

    def wait(self) -> tuple[np.ndarray, np.ndarray]:
        if self._s is None:
            self.event.synchronize()
            p = self.pinned.numpy()
            self._s, self._r = p[:self.world].copy(), p[self.world:2 * self.world].copy()
        return self._s, self._r


class Transport(ABC):
    rank: int = 0
    world: int = 1
    label: str = "?"   # what actually carries the data (bench.py reports it)

    @abstractmethod
    def exchange_counts(self, send_counts: torch.Tensor) -> tuple[np.ndarray, np.ndarray]:
        """All-to-all of one int64 per peer. Returns host (send_counts, recv_counts)."""

    def exchange_counts_async(self, send_counts: torch.Tensor, pinned: Optional[torch.Tensor] = None,
                              stream=None) -> CountsHandle:
        """Enqueue the count exchange; ``.wait()`` returns host counts.  The
        default implementation is synchronous."""
        s, r = self.exchange_counts(send_counts)
        return CountsHandle(s, r)

    @abstractmethod
    def alltoallv(self, send: torch.Tensor, scounts: Sequence[int], sdispls: Sequence[int],
                  recv: torch.Tensor, rcounts: Sequence[int], rdispls: Sequence[int],
                  row_elems: int = 1) -> None:
        ...

    @abstractmethod
    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        ...

    @abstractmethod
    def barrier(self) -> None:
        ...

    def close(self) -> None:
        pass


class LoopbackTransport(Transport):
    label = "loopback (world 1: device copies, no collective)"

    def __init__(self):
        self.rank, self.world = 0, 1

    def exchange_counts(self, send_counts):
        c = send_counts.detach().cpu().numpy().astype(np.int64)
        return c, c.copy()

    def exchange_counts_async(self, send_counts, pinned=None, stream=None):
        if send_counts.device.type != "cuda" or pinned is None:
            return super().exchange_counts_async(send_counts, pinned, stream)
        # GPU: D2H into pinned memory on `stream`, the host waits in wait()
        st = stream or torch.cuda.current_stream()
        with torch.cuda.stream(st):
            pinned[:1].copy_(send_counts.to(torch.int64)[:1], non_blocking=True)
            pinned[1:2].copy_(send_counts.to(torch.int64)[:1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        return CountsHandle(event=ev, pinned=pinned, world=1)

    def alltoallv(self, send, scounts, sdispls, recv, rcounts, rdispls, row_elems=1):
        n = int(scounts[0]) * row_elems
        if n and (send.data_ptr() != recv.data_ptr() or sdispls[0] != rdispls[0]):
            s0, r0 = int(sdispls[0]) * row_elems, int(rdispls[0]) * row_elems
            recv.view(-1)[r0:r0 + n].copy_(send.view(-1)[s0:s0 + n])

    def allreduce_(self, t, op="sum"):
        return t

    def barrier(self):
        pass


class TorchDistTransport(Transport):
    """torch.distributed-based transport (gloo on CPU, or nccl on GPU)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.label = (f"torch.distributed {self.backend} all_to_all_single"
                      + (" (host-staged)" if self.backend == "gloo" else ""))

    def _dev(self, t: torch.Tensor):
        return t if self.backend != "gloo" else t.cpu()

    def exchange_counts(self, send_counts):
        s = self._dev(send_counts.to(torch.int64).contiguous())
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return s.cpu().numpy(), r.cpu().numpy()

    def alltoallv(self, send, scounts, sdispls, recv, rcounts, rdispls, row_elems=1):
        sflat, rflat = send.view(-1), recv.view(-1)
        parts = [sflat[int(d) * row_elems:(int(d) + int(c)) * row_elems]
                 for c, d in zip(scounts, sdispls)]
        sbuf = self._dev(torch.cat(parts) if parts else sflat[:0])
        rtotal = int(sum(rcounts)) * row_elems
        rbuf = torch.empty(rtotal, dtype=sbuf.dtype, device=sbuf.device)
        dist.all_to_all_single(rbuf, sbuf, [int(c) * row_elems for c in rcounts],
                               [int(c) * row_elems for c in scounts], group=self.group)
        rbuf = rbuf.to(recv.device)
        o = 0
        for c, d in zip(rcounts, rdispls):
            n = int(c) * row_elems
            if n:
                rflat[int(d) * row_elems:int(d) * row_elems + n].copy_(rbuf[o:o + n])
            o += n

    def allreduce_(self, t, op="sum"):
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if self.backend == "gloo" and t.device.type != "cpu":
            c = t.cpu()
            dist.all_reduce(c, o, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, o, group=self.group)
        return t

    def barrier(self):
        dist.barrier(group=self.group)


def default_gloo_ifname() -> None:
    """Bind the gloo control plane to loopback when the job is single-host
    (every rank local — torchrun's LOCAL_WORLD_SIZE == WORLD_SIZE — or a
    loopback MASTER_ADDR), unless the user chose an interface; a multi-host
    job keeps gloo's own interface choice."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    world = os.environ.get("WORLD_SIZE", "1")
    local = os.environ.get("LOCAL_WORLD_SIZE", world)
    if local == world or addr in ("localhost", "::1") or addr.startswith("127."):
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")


_fd_lock = threading.Lock()
_fd_depth = 0
_fd_saved = -1


@contextlib.contextmanager
def _stdout_to_stderr():
    """Point fd 1 at fd 2 for the duration (native code writing to stdout).
    C stdio buffers are flushed before fd 1 is restored, so buffered native
    output lands on stderr too.  Reference-counted under a lock: nested or
    concurrent users (in-process ranks building communicators on threads)
    share one redirect, and only the outermost restores fd 1."""
    import ctypes

    global _fd_depth, _fd_saved
    libc = ctypes.CDLL(None)
    with _fd_lock:
        if _fd_depth == 0:
            sys.stdout.flush()
            _fd_saved = os.dup(1)
            os.dup2(2, 1)
        _fd_depth += 1
    try:
        yield
    finally:
        with _fd_lock:
            _fd_depth -= 1
            if _fd_depth == 0:
                libc.fflush(None)
                sys.stdout.flush()
                os.dup2(_fd_saved, 1)
                os.close(_fd_saved)
                _fd_saved = -1


class RcclTransport(Transport):
    """Native RCCL communicator over xGMI.

    ``serial`` (SS_RCCL_COMMS=1, the default): every collective of this
    communicator is enqueued on ONE dedicated comm stream, in host program
    order — the caller's stream is joined to it before and after — so the
    engine's route, pull and main streams can never have two operations of
    the communicator in flight at once, and every rank issues the same
    sequence on the same stream (no cross-rank ordering hazards).  With
    SS_RCCL_COMMS=3 the engine uses three communicators, each on the stream
    that calls it (more overlap; RCCL then relies on every rank enqueuing
    them in the same order)."""

    _DT = {torch.float32: 0, torch.float64: 1, torch.int32: 2, torch.int64: 3}

    def __init__(self, rank: int, world: int, device: torch.device, store=None,
                 uid: Optional[bytes] = None, prefix: str = "ss_rccl", serial: bool = True):
        from .._native import hip

        h = hip()
        self.rank, self.world, self.device = rank, world, torch.device(device)
        if uid is None:
            if store is None:
                raise ValueError("RcclTransport needs a store (or an explicit unique id)")
            key = f"{prefix}_uid"
            if rank == 0:
                uid = self.new_unique_id()
                store.set(key, uid)
            else:
                store.wait([key])
                uid = store.get(key)
        # RCCL prints a version banner on fd 1 when it initialises: route it
        # to stderr so a job's stdout stays the caller's (bench.py's one JSON
        # line)
        with _stdout_to_stderr():
            self.comm = h.RcclComm(rank, world, uid, self.device.index or 0)
        self.serial = bool(serial)
        self.stream = torch.cuda.Stream(device=self.device) if self.serial else None
        self.label = f"RCCL grouped send/recv ({'1 comm stream' if self.serial else 'caller streams'})"
        self._pin = torch.empty(2 * world, dtype=torch.int64, pin_memory=True)

    def nranks(self) -> int:
        """Ranks of the communicator as RCCL reports them (ncclCommCount)."""
        return int(self.comm.comm_count())

    @staticmethod
    def new_unique_id() -> bytes:
        """A fresh ncclUniqueId (RCCL's init banner goes to stderr)."""
        from .._native import hip

        with _stdout_to_stderr():
            return hip().RcclComm.unique_id()

    @contextlib.contextmanager
    def _on(self, caller=None):
        """The stream a collective goes on: the comm stream (serial), joined
        to the caller's stream on both sides, or the caller's stream."""
        cs = caller or torch.cuda.current_stream(self.device)
        if not self.serial:
            yield cs
            return
        self.stream.wait_stream(cs)
        with torch.cuda.stream(self.stream):
            yield self.stream
        cs.wait_stream(self.stream)

    def abort(self) -> None:
        """ncclCommAbort: stuck collectives return; the communicator is dead
        afterwards (failure path of parallel/watchdog.py)."""
        self.comm.abort()

    def exchange_counts(self, send_counts):
        return self.exchange_counts_async(send_counts).wait()

    def exchange_counts_async(self, send_counts, pinned=None, stream=None):
        """Counts all-to-all + D2H into pinned memory; the host only blocks
        in ``wait()`` (on an event), so the exchange overlaps with whatever
        the other streams are running."""
        pin = pinned if pinned is not None else self._pin
        with self._on(stream) as st:
            s = send_counts.to(torch.int64).contiguous()
            recv = torch.empty(self.world, dtype=torch.int64, device=self.device)
            self.comm.alltoall(s.data_ptr(), recv.data_ptr(), 1, 8, st.cuda_stream)
            pin[:self.world].copy_(s, non_blocking=True)
            pin[self.world:2 * self.world].copy_(recv, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        return CountsHandle(event=ev, pinned=pin, world=self.world)

    def alltoallv(self, send, scounts, sdispls, recv, rcounts, rdispls, row_elems=1):
        eb = send.element_size() * row_elems
        with self._on() as st:
            self.comm.alltoallv(send.data_ptr(), [int(x) for x in scounts],
                                [int(x) for x in sdispls], recv.data_ptr(),
                                [int(x) for x in rcounts], [int(x) for x in rdispls], eb,
                                st.cuda_stream, send.numel() // row_elems,
                                recv.numel() // row_elems)

    def allreduce_(self, t, op="sum"):
        with self._on() as st:
            self.comm.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), self._DT[t.dtype],
                                {"sum": 0, "max": 1, "min": 2}[op], st.cuda_stream)
        return t

    def barrier(self):
        x = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.allreduce_(x)
        torch.cuda.current_stream(self.device).synchronize()

    def close(self):
        self.comm = None


def rccl_comms_mode() -> int:
    """SS_RCCL_COMMS: 1 (default) = one communicator on one comm stream; 3 =
    data / count / pull communicators on the engine's three streams."""
    v = os.environ.get("SS_RCCL_COMMS", "1")
    if v not in ("1", "3"):
        raise ValueError(f"SS_RCCL_COMMS={v!r}: 1 or 3")
    return int(v)


def make_transport(kind: str = "auto", device=None, store=None) -> Transport:
    """auto: loopback for world 1; rccl on GPU; torch.distributed otherwise."""
    if not dist.is_available() or not dist.is_initialized():
        return LoopbackTransport()
    world = dist.get_world_size()
    if world == 1 and kind == "auto":
        return LoopbackTransport()
    dev = torch.device(device) if device is not None else None
    if kind == "rccl" or (kind == "auto" and dev is not None and dev.type == "cuda"):
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        return RcclTransport(dist.get_rank(), world, dev, store=store)
    return TorchDistTransport()
