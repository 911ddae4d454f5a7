"""xGMI peer-mailbox transport: the N>1 data plane with device-side counts.

``RcclTransport`` moves a round's segments with grouped ncclSend/ncclRecv,
which need the byte counts on the host — one D2H + host wait per round, and
no hipGraph capture of an N>1 step.  This transport (``csrc/hip/xgmi.hip``)
gives every rank uncached HBM arenas — one per (channel, ring slot), each
below 2 GiB, the largest IPC import that returns — exported through IPC
handles and mapped by every peer: a ``put`` kernel stores this rank's segment
for each peer straight into that peer's arena over xGMI, with the row count read from
device memory and written into the receiver's header, then bumps a
per-(channel, source) arrival counter there; a ``wait`` kernel on the
consumer's stream spins until all sources have arrived.  The receiver's
buffers ARE the arena: the server kernels read received keys and gradients
in place, the worker reads pulled rows in place.

The same code runs with every rank on ONE GPU (the IPC mappings are then the
same device's memory), which is how the peer data path is exercised on a
1-GPU box (tests/test_gpu_multiproc.py).  ``setup`` ends with a self-test —
every rank puts a rank-stamped pattern to every peer and checks what
arrived — so a fabric that cannot map or order peer stores fails at start-up
(bench.py then falls back to RCCL), never mid-training.

Control-plane collectives (barrier, the start-up agreement) go through
``aux`` (a gloo ``TorchDistTransport``).  Reference parity:
/root/reference/src/core/transfer/transfer.h:75-150 (send / receive loop).
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from .transport import Transport

_ALIGN = 256
# one IPC allocation must stay below 2 GiB (hipIpcOpenMemHandle of a larger
# uncached allocation never returned on the MI355X boxes; see setup)
_MAX_ARENA = 2 << 30
_DT = {torch.int64: (0, 64), torch.int32: (0, 32), torch.float32: (2, 32)}


def _al(x: int) -> int:
    return (int(x) + _ALIGN - 1) // _ALIGN * _ALIGN


class XgmiTransport(Transport):
    label = "xGMI peer stores into IPC-mapped HBM mailboxes (device-side counts)"

    def __init__(self, rank: int, world: int, device, store, aux: Optional[Transport] = None,
                 prefix: str = "ss_xgmi", timeout_s: Optional[float] = None):
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        self.store, self.prefix = store, prefix
        self.aux = aux
        self.timeout_s = float(timeout_s if timeout_s is not None else
                               os.environ.get("SS_XGMI_TIMEOUT", "120"))
        # one arena (one allocation, one IPC handle) per (channel, slot)
        self.arenas: dict = {}
        self._errs: list = []
        self._layout: dict = {}
        # workgroups per peer of a put (~1024 in all): a put is latency-bound
        # per workgroup (16 B per lane per iteration); 32 per peer measured
        # 211 us for the 42 MB keys put of a 1-rank arena
        self.bpp = int(os.environ.get("SS_XGMI_BPP", "0")) or max(128, 1024 // self.world)

    # ------------------------------------------------------------ set-up
    def setup(self, channels: dict) -> None:
        """Lay out and map the arenas.  ``channels``: name -> (slots, parts),
        parts a list of per-source segment sizes in bytes.  Collective: every
        rank calls it with the same channels, in the same order.

        Each (channel, slot) is its own arena — its own allocation, IPC
        handle and arrival flags (channel id 0 inside it).  One arena for
        everything measured as a hang: hipIpcOpenMemHandle never returned
        for an uncached allocation of 2 GB or more (0.5-1.5 GB: instant), and
        the bench's arena is 2.6 GB at N = 4 and 5.2 GB at N = 8.  Per
        (channel, slot) the largest is the keys of one round from 16 sources
        of a 10M-key batch, 1.3 GB."""
        from .._native import hip

        h = hip()
        chans = dict(channels)
        chans["_probe"] = (1, [4096])
        sizes = {}
        for name, (slots, parts) in chans.items():
            for slot in range(int(slots)):
                off = h.xgmi_flag_bytes()
                for p, seg in enumerate(parts):
                    # segments keep their exact size (source s at s * seg: the
                    # consumers index [source][row]); regions start aligned
                    hdr = _al(off)
                    data = _al(hdr + 8 * self.world)
                    self._layout[(name, p, slot)] = (hdr, data, int(seg))
                    off = data + self.world * int(seg)
                if _al(off) >= _MAX_ARENA:
                    raise ValueError(f"xgmi: the {name} mailbox of one round needs "
                                     f"{_al(off) / 2**30:.2f} GiB (< 2 GiB per IPC allocation)")
                sizes[(name, slot)] = _al(off)
        self.bytes = sum(sizes.values())
        dev = self.device.index or 0
        # a rank that cannot map its peers still takes part in the agreement
        # of the self-test, so every rank raises together (and a caller can
        # fall back to RCCL on all ranks)
        err, handles = None, {}
        try:
            for key, nb in sizes.items():
                self.arenas[key] = h.XgmiArena(self.rank, self.world, dev, nb)
            for i, (key, a) in enumerate(self.arenas.items()):
                handles[key] = self._allgather_bytes(bytes(a.ipc_handle()), i)
        except Exception as e:  # pragma: no cover - hardware dependent
            err = e
            for i in range(len(handles), len(sizes)):
                self._allgather_bytes(b"", i)  # the peers are waiting for a handle
        err = self._open_in_turns(handles if err is None else None) or err
        if err is None:
            self._errs = [torch.utils.dlpack.from_dlpack(h.dlpack_view(a.err_ptr, [2], 0, 32, dev))
                          for a in self.arenas.values()]
        self._selftest(err)

    def _allgather_bytes(self, mine: bytes, tag: int = 0) -> list:
        if self.world == 1:
            return [mine]
        self.store.set(f"{self.prefix}_h{tag}_{self.rank}", mine)
        out = []
        for r in range(self.world):
            k = f"{self.prefix}_h{tag}_{r}"
            self.store.wait([k])
            out.append(bytes(self.store.get(k)))
        return out

    def _open_in_turns(self, handles) -> Optional[Exception]:
        """Map the peers' arenas one rank at a time (the others wait on the
        store), so an exporter is never itself inside an import.  Every rank
        takes every turn, also one that cannot map (handles None)."""
        import sys
        import time

        err = None
        for turn in range(self.world):
            key = f"{self.prefix}_open{turn}"
            if turn != self.rank:
                if self.world > 1:
                    self.store.wait([key])
                continue
            t0 = time.perf_counter()
            try:
                if handles is None:
                    raise RuntimeError("no arena or peer handles")
                for k, a in self.arenas.items():
                    a.open_peers(handles[k])
            except Exception as e:  # pragma: no cover - hardware dependent
                err = e
            dt = time.perf_counter() - t0
            if dt > 5.0:
                print(f"xgmi: rank {self.rank} mapped its {self.world - 1} peers' arenas in "
                      f"{dt:.1f} s", file=sys.stderr, flush=True)
            if self.world > 1:
                self.store.set(key, b"1")
        return err

    def _selftest(self, err: Optional[Exception] = None) -> None:
        """Every rank puts (rank, peer)-stamped words to every peer; each
        checks what arrived, and all ranks agree before the transport is
        used (a failure raises on every rank)."""
        N, me = self.world, self.rank
        if err is not None:
            flag = torch.zeros(1, dtype=torch.int64)
            if self.aux is not None and N > 1:
                self.aux.allreduce_(flag, "min")
            raise RuntimeError(f"xgmi set-up failed on this rank: {err}")
        src = torch.empty((N, 1024), dtype=torch.int32, device=self.device)
        for d in range(N):
            src[d] = me * 1000003 + d * 7919 + torch.arange(1024, dtype=torch.int32,
                                                            device=self.device)
        st = torch.cuda.current_stream(self.device)
        self.put("_probe", 0, [(src, [d * 1024 for d in range(N)], None, 1024)], stream=st)
        self.wait("_probe", 0, stream=st)
        got = self.region("_probe", 0, 0, torch.int32).view(N, -1)[:, :1024].clone()
        cnt = self.counts("_probe", 0, 0).clone()
        st.synchronize()
        exp = torch.stack([s * 1000003 + me * 7919 + torch.arange(1024, dtype=torch.int32)
                           for s in range(N)])
        ok = bool(torch.equal(got.cpu(), exp)) and bool((cnt.cpu() == 1024).all()) and \
            all(int(e[0].item()) == 0 for e in self._errs)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
        if self.aux is not None and N > 1:
            self.aux.allreduce_(flag, "min")
        if int(flag.item()) != 1:
            raise RuntimeError(f"xgmi self-test failed on {'this rank' if not ok else 'a peer'}")

    # ------------------------------------------------------------ data plane
    def arena_of(self, ch: str, slot: int):
        """The XgmiArena of (channel, slot) (the C++ round engine drives it;
        its channel id is 0)."""
        return self.arenas[(ch, slot)]

    def region(self, ch: str, part: int, slot: int, dtype=torch.float32,
               cols: int = 1) -> torch.Tensor:
        """The receive area of (channel, part, slot) as a tensor: source s's
        segment at rows [s * seg_rows, ...)."""
        from .._native import hip

        hdr, data, seg = self._layout[(ch, part, slot)]
        code, bits = _DT[dtype]
        rows = self.world * seg // (bits // 8 * cols)
        shape = [rows, cols] if cols > 1 else [rows]
        return torch.utils.dlpack.from_dlpack(
            hip().dlpack_view(self.arenas[(ch, slot)].base + data, shape, code, bits,
                              self.device.index or 0))

    def counts(self, ch: str, part: int, slot: int) -> torch.Tensor:
        """int64 [world]: rows each source put into (channel, part, slot)."""
        from .._native import hip

        hdr, _, _ = self._layout[(ch, part, slot)]
        return torch.utils.dlpack.from_dlpack(
            hip().dlpack_view(self.arenas[(ch, slot)].base + hdr, [self.world], 0, 64,
                              self.device.index or 0))

    def layout(self, ch: str, part: int, slot: int) -> tuple:
        """(header offset, data offset, per-source segment bytes) in the
        (channel, slot) arena."""
        return self._layout[(ch, part, slot)]

    def seg_rows(self, ch: str, part: int, row_bytes: int) -> int:
        return self._layout[(ch, part, 0)][2] // row_bytes

    def put(self, ch: str, slot: int, parts: Sequence, stream=None) -> None:
        """parts: (src tensor, per-destination row displacements, device
        int64 [world] row counts or None, fixed row count, [row elems])."""
        spec = []
        for p, part in enumerate(parts):
            src, displs, cnt, fixed = part[:4]
            row_elems = part[4] if len(part) > 4 else 1
            hdr, data, seg = self._layout[(ch, p, slot)]
            rb = src.element_size() * row_elems
            spec.append([src.data_ptr(), cnt.data_ptr() if cnt is not None else 0,
                         int(fixed or 0), rb, hdr, data, seg] + [int(d) * rb for d in displs])
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.arenas[(ch, slot)].put(0, spec, self.bpp, st.cuda_stream)

    def wait(self, ch: str, slot: int, stream=None, fixed_parts: Sequence = (),
             metrics: Sequence = (), bytes_per_key: float = 0.0) -> None:
        """Block ``stream`` until every source's put of this (channel, slot)'s
        next round has arrived.  ``fixed_parts``: (part, bytes) of fixed-size
        parts read as zeros if a source never arrives.  ``metrics``: (sent
        [world] i64, recv [world] i64, acc [3] f64, xval [1] i64, xacc [1]
        f64) tensors or None, added on the device after the wait:
        acc += (sum sent, sum recv, bytes_per_key * both), xacc += xval."""
        fx = []
        for p, nb in fixed_parts:
            _, data, seg = self._layout[(ch, p, slot)]
            fx.append([data, seg, int(nb)])
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        mp = [t.data_ptr() if t is not None else 0 for t in metrics]
        self.arenas[(ch, slot)].wait(0, fx, self.timeout_s, st.cuda_stream, mp,
                                     float(bytes_per_key))

    def check(self) -> None:
        for e in self._errs:
            v = int(e[0].item())
            if v & 1:
                raise RuntimeError(f"xgmi: a peer did not arrive within {self.timeout_s} s")
            if v & 2:
                raise RuntimeError("xgmi: a put exceeded its segment (counts corrupt)")

    # ------------------------------------------------------------ control plane
    def exchange_counts(self, send_counts):
        raise NotImplementedError("xgmi keeps counts on the device (use put / wait)")

    def alltoallv(self, send, scounts, sdispls, recv, rcounts, rdispls, row_elems=1):
        raise NotImplementedError("xgmi moves segments with put / wait")

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world == 1:
            return t
        if self.aux is None:
            raise RuntimeError("xgmi: control-plane collectives need an aux transport")
        return self.aux.allreduce_(t, op)

    def barrier(self) -> None:
        if self.aux is not None and self.world > 1:
            self.aux.barrier()

    def close(self) -> None:
        if self.arenas:
            torch.cuda.synchronize(self.device)
        self.arenas = {}
