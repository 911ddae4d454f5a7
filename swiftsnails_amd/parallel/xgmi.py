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
1-GPU box (tests/test_gpu_multiproc.py).

Fail-safe start-up (``setup``): the arenas are mapped, then a message-passing
LITMUS runs on the real arenas — every (channel, slot) arena, full-size
segments of every part, the production put geometry, ``2 x depth`` rounds
reusing the slots, each round's words stamped with (round, source,
destination, channel, part) and checked word by word by the receiver — once
per publish tier, in order:

  ``drain``  — fence-free (drained uncached stores, relaxed flag add);
  ``fenced`` — one system-scope release per put block towards arenas on
               another device, one system-scope acquire after each wait.

The first tier that passes on EVERY rank is used (``tier``); if none does,
``setup`` raises and the caller falls back to RCCL (``select.build_engine``).
``SS_XGMI_FORCE_TIER=fenced|rccl`` makes the earlier tiers fail on purpose
(proves each fallback step end to end); ``SS_XGMI_VERIFY=1`` keeps checking
at run time: every put block writes a round tag after its payload, every
wait checks them, and a stale tag (a flag that overtook its data) sets a
sticky error that ``poll_error`` sees without a device sync.

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
        self.verify = os.environ.get("SS_XGMI_VERIFY", "0") not in ("0", "")
        self.force_tier = os.environ.get("SS_XGMI_FORCE_TIER", "").strip().lower()
        if self.force_tier not in ("", "drain", "fenced", "rccl"):
            raise ValueError("SS_XGMI_FORCE_TIER: drain, fenced or rccl")
        self.tier: Optional[str] = None
        self.litmus_log: list = []   # (tier, passed, seconds, reason)
        self.remote_mask = 0
        self.devices = 1             # distinct devices among the ranks
        self._channels: dict = {}
        self._close_hooks: list = []  # engines holding arena pointers (clear_xgmi)

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
        self._channels = chans
        sizes = {}
        for name, (slots, parts) in chans.items():
            for slot in range(int(slots)):
                off = h.xgmi_head_bytes()
                for p, seg in enumerate(parts):
                    # segments keep their exact size (source s at s * seg: the
                    # consumers index [source][row]); regions start aligned
                    hdr = _al(off)
                    data = _al(hdr + 8 * self.world)
                    self._layout[(name, p, slot)] = (hdr, data, int(seg))
                    off = data + self.world * int(seg)
                if _al(off) >= _MAX_ARENA:
                    # a RuntimeError like every other set-up failure: callers
                    # fall back to RCCL on it
                    raise RuntimeError(f"xgmi: the {name} mailbox of one round needs "
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
        self._peer_devices(h, dev)
        self._select_tier(err)

    # ------------------------------------------------------------ tiers
    TIERS = ("drain", "fenced")

    def _peer_devices(self, h, dev: int) -> None:
        """Which ranks' arenas live on another device (the fenced tier
        releases only towards those), and how many distinct devices the job
        spans.  SS_XGMI_FENCE_ALL=1 treats every peer as remote (tests of
        the fenced tier with all ranks on one GPU)."""
        try:
            mine = h.device_pci_id(dev).encode()
        except Exception:  # pragma: no cover - hardware dependent
            mine = f"dev{dev}".encode()
        ids = self._allgather_bytes(mine, "pci")
        self.devices = len(set(ids))
        fence_all = os.environ.get("SS_XGMI_FENCE_ALL", "0") not in ("0", "")
        self.remote_mask = sum(1 << r for r, x in enumerate(ids)
                               if r != self.rank and (fence_all or x != mine))

    def _set_tier(self, tier: str) -> None:
        t = self.TIERS.index(tier)
        for a in self.arenas.values():
            a.set_tier(t, self.remote_mask, self.verify)

    def _select_tier(self, err: Optional[Exception]) -> None:
        """Run the litmus per tier; keep the first that passes on every rank
        (all ranks see the same agreed results, so all pick the same tier or
        all raise)."""
        import time

        # every rank agrees on the set-up first: a rank that could not map
        # its peers must not leave the others in a litmus it never joins
        ok, _ = self._agree_ok(err is None)
        if not ok:
            raise RuntimeError(f"xgmi set-up failed on {'this rank' if err else 'a peer'}"
                               + (f": {err}" if err else ""))
        reasons = []
        for tier in self.TIERS:
            # a failed earlier tier's sticky error bits (a stale round tag, a
            # corrupt count) must not fail this tier's litmus or the first
            # training round: clear the device and host-mapped error words
            # once that tier's work has drained (reset_err synchronises)
            self.reset_errors()
            self._set_tier(tier)
            forced = self.force_tier == "rccl" or (self.force_tier == "fenced" and tier == "drain")
            t0 = time.perf_counter()
            ok, why = self._litmus(fail=forced)
            # agreed collectively: passed on every rank; timed out on any
            ok, timed_out = self._agree_ok(ok, why == "timeout")
            dt = time.perf_counter() - t0
            self.litmus_log.append((tier, ok, round(dt, 3), "" if ok else (why or "a peer failed")))
            if ok:
                self.tier = tier
                return
            reasons.append(f"{tier}: {why or 'a peer failed'}")
            if timed_out:
                break  # the arrival counters are no longer in step: no retry
        raise RuntimeError("xgmi litmus failed on every tier (" + "; ".join(reasons) + ")")

    def reset_errors(self) -> None:
        """Clear every arena's sticky device and host-mapped error words
        (waits for the device)."""
        for a in self.arenas.values():
            a.reset_err()

    def _agree_ok(self, ok: bool, timed_out: bool = False):
        """(every rank ok, any rank timed out), the same on every rank."""
        flag = torch.tensor([1 if ok else 0, 0 if timed_out else 1], dtype=torch.int64)
        if self.aux is not None and self.world > 1:
            self.aux.allreduce_(flag, "min")
        return int(flag[0].item()) == 1, int(flag[1].item()) == 0

    @staticmethod
    def _seed(rnd: int, src: int, dst: int, ch: int, part: int) -> int:
        x = (rnd * 0x9E3779B1 + src * 0x85EBCA77 + dst * 0xC2B2AE3D + ch * 0x27D4EB2F +
             part * 0x165667B1 + 0x5BD1E995)
        return x & 0xFFFFFFFF

    def _litmus(self, fail: bool = False):
        """Message-passing litmus on the real arenas (see the module doc).
        Returns (passed on this rank, reason).  A rank whose GPU work fails
        keeps taking every round's barrier (its peers' waits on it time out)
        so the ranks never diverge in their collectives."""
        from .._native import hip

        h = hip()
        N, dev = self.world, self.device
        st = torch.cuda.current_stream(dev)
        names = sorted(self._channels)
        rounds = max(2, 2 * max(int(sl) for sl, _ in self._channels.values()))
        failed, srcs = None, {}
        try:
            bad = torch.zeros(1, dtype=torch.int32, device=dev)
            cnt_bad = torch.zeros(1, dtype=torch.int64, device=dev)
            for name in names:
                for p, seg in enumerate(self._channels[name][1]):
                    if int(seg) % 4:
                        raise ValueError(f"segment of {name}/{p} not whole words")
                    srcs[(name, p)] = torch.empty(N * int(seg) // 4, dtype=torch.int32,
                                                  device=dev)
        except Exception as e:  # pragma: no cover - hardware dependent
            failed = f"exception: {e}"
        for rnd in range(rounds):
            if failed is None:
                try:
                    self._litmus_round(h, rnd, names, srcs, bad, cnt_bad, st)
                    st.synchronize()
                except Exception as e:  # pragma: no cover - hardware dependent
                    failed = f"exception: {e}"
            # no rank rewrites a slot before every receiver checked it
            if self.aux is not None and N > 1:
                self.aux.barrier()
        errs = [int(e[0].item()) for e in self._errs]
        if any(e & 1 for e in errs):
            return False, "timeout"
        if failed is not None:
            return False, failed
        if any(e for e in errs):
            return False, f"error word {max(errs)}"
        nb, nc = int(bad.item()), int(cnt_bad.item())
        if nb or nc:
            return False, f"{nb} words and {nc} counts wrong"
        if fail:
            return False, "forced (SS_XGMI_FORCE_TIER)"
        return True, ""

    def _litmus_round(self, h, rnd: int, names, srcs, bad, cnt_bad, st) -> None:
        """One litmus round: every channel's slot rnd % slots, full-size
        segments stamped (round, source, destination, channel, part), put,
        waited for, every received word checked."""
        N, me, dev = self.world, self.rank, self.device
        tmo = min(self.timeout_s, float(os.environ.get("SS_XGMI_LITMUS_TIMEOUT", "30")))
        for ci, name in enumerate(names):
            slots, parts = self._channels[name]
            slot = rnd % int(slots)
            spec = []
            for p, seg in enumerate(parts):
                w = int(seg) // 4
                src = srcs[(name, p)]
                for d in range(N):
                    h.xgmi_pattern(src.data_ptr() + 4 * d * w, w,
                                   self._seed(rnd, me, d, ci, p), st.cuda_stream)
                full = torch.full((N,), w, dtype=torch.int64, device=dev)
                spec.append((src, [d * w for d in range(N)], full, None))
                srcs[(name, p, "cnt")] = full  # alive until the put ran
            self.put(name, slot, spec, stream=st)
            # at start-up every rank is ready: a peer that has not arrived
            # within the litmus timeout is not coming
            self.wait(name, slot, stream=st, timeout_s=tmo)
            for p, seg in enumerate(parts):
                w = int(seg) // 4
                got = self.region(name, p, slot, torch.int32)
                for s_ in range(N):
                    h.xgmi_check(got.data_ptr() + 4 * s_ * w, w, self._seed(rnd, s_, me, ci, p),
                                 bad.data_ptr(), st.cuda_stream)
                cnt_bad += (self.counts(name, p, slot) != w).sum()

    def _allgather_bytes(self, mine: bytes, tag=0) -> list:
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
             metrics: Sequence = (), bytes_per_key: float = 0.0,
             timeout_s: Optional[float] = None) -> None:
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
        self.arenas[(ch, slot)].wait(0, fx, self.timeout_s if timeout_s is None else timeout_s,
                                     st.cuda_stream, mp, float(bytes_per_key))

    def check(self) -> None:
        for e in self._errs:
            v = int(e[0].item())
            if v & 1:
                raise RuntimeError(f"xgmi: a peer did not arrive within {self.timeout_s} s")
            if v & 2:
                raise RuntimeError("xgmi: a put exceeded its segment (counts corrupt)")
            if v & 4:
                raise RuntimeError("xgmi: a round tag was stale when its flag arrived "
                                   f"(publish ordering failed on tier {self.tier})")

    def poll_error(self) -> None:
        """Raise if a wait kernel has flagged an error (timeout, stale round
        tag): reads the host-mapped error words, no device sync — cheap
        enough for every round (engine.all_done, the bench loop)."""
        v = 0
        for a in self.arenas.values():
            v |= int(a.host_err())
        if v & 1:
            raise RuntimeError(f"xgmi: a peer did not arrive within {self.timeout_s} s "
                               "(SS_XGMI_TIMEOUT)")
        if v & 4:
            raise RuntimeError("xgmi: a round tag was stale when its flag arrived "
                               f"(publish ordering failed on tier {self.tier})")

    def describe(self) -> dict:
        """What the start-up chose: tier, litmus results, distinct devices."""
        return {"xgmi_tier": self.tier, "devices": self.devices,
                "xgmi_verify": bool(self.verify),
                "litmus": [{"tier": t, "passed": ok, "s": dt, **({"why": w} if w else {})}
                           for t, ok, dt, w in self.litmus_log]}

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
        for f in getattr(self, "_close_hooks", []):
            f()
        self._close_hooks = []
        self._errs = []
        self.arenas = {}
