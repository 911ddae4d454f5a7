"""Data-plane selection with a fail-safe fallback chain (bench.py and the
config launcher, framework/gpu.py, share it).

``transport: auto`` (the default) tries, in order:

  1. the xGMI mailboxes with the fence-free ``drain`` publish,
  2. the xGMI mailboxes with the ``fenced`` publish,
  3. RCCL (one native communicator),

where each xGMI tier must pass the start-up litmus on every rank
(parallel/xgmi.py) before a single training byte moves through it.  A
failure of both tiers — or any other mailbox set-up failure (an IPC mapping
that fails, a layout over the 2 GiB import limit) — closes the mailbox
transport, frees its arenas, and builds the engine on RCCL instead; the
result says which plane runs, which tier, whether it fell back and why, and
how many distinct devices the ranks span (``PlaneInfo``), so a silent
degradation shows up in the bench JSON.  Reference parity: the reference has
one transport (ZeroMQ, /root/reference/src/core/transfer/transfer.h:75-150);
a plane the sender can rely on is the property kept.
"""
from __future__ import annotations

import gc
import os
from dataclasses import asdict, dataclass, field
from typing import Callable, Optional

import torch


@dataclass
class PlaneInfo:
    transport: str                      # label of what carries the data
    plane: str                          # xgmi | rccl | gloo | torch | loopback
    xgmi_tier: Optional[str] = None     # drain | fenced (xgmi only)
    fell_back: bool = False
    fallback_reason: str = ""
    devices: int = 1                    # distinct devices among the ranks
    comms: int = 0                      # native RCCL communicators
    litmus: list = field(default_factory=list)

    def asdict(self) -> dict:
        return asdict(self)


def distinct_devices(store, rank: int, world: int, device, prefix: str = "ss_devid") -> int:
    """How many distinct GPUs the ranks run on (PCI bus ids over the store;
    N ranks pinned to one GPU report 1)."""
    if world <= 1 or store is None:
        return 1
    from .._native import hip

    dev = torch.device(device).index or 0
    try:
        mine = hip().device_pci_id(dev)
    except Exception:  # pragma: no cover - hardware dependent
        mine = f"dev{dev}"
    store.set(f"{prefix}_{rank}", mine)
    ids = set()
    for r in range(world):
        k = f"{prefix}_{r}"
        store.wait([k])
        ids.add(bytes(store.get(k)).decode())
    return len(ids)


def _plane_of(t) -> str:
    from .transport import LoopbackTransport, RcclTransport, TorchDistTransport
    from .xgmi import XgmiTransport

    if isinstance(t, XgmiTransport):
        return "xgmi"
    if isinstance(t, RcclTransport):
        return "rccl"
    if isinstance(t, TorchDistTransport):
        return "gloo" if getattr(t, "backend", "") == "gloo" else "torch"
    if isinstance(t, LoopbackTransport):
        return "loopback"
    return type(t).__name__


def make_transports(kind: str, rank: int, world: int, device, store, prefix: str = "ss_xgmi"):
    """(data transport, count transport, pull transport, native comms) for
    ``kind`` in auto | xgmi | rccl | gloo.  World 1: loopback, or with
    SS_ENGINE_GENERAL=xgmi|rccl a size-1 mailbox arena / communicator (the
    N>1 engine path on one GPU).  ``prefix``: the mailboxes' store keys (a
    second engine of the same job needs its own)."""
    from .transport import (LoopbackTransport, RcclTransport, TorchDistTransport,
                            rccl_comms_mode)
    from .xgmi import XgmiTransport

    dev = torch.device(device)
    if world <= 1:
        general = os.environ.get("SS_ENGINE_GENERAL", "0")
        if general == "xgmi" or (general == "1" and kind in ("auto", "xgmi")):
            return XgmiTransport(0, 1, dev, None), None, None, 0
        if general in ("rccl", "1"):
            return RcclTransport(0, 1, dev, uid=RcclTransport.new_unique_id()), None, None, 1
        return LoopbackTransport(), None, None, 0
    if kind == "gloo":
        return TorchDistTransport(), None, None, 0
    if kind in ("auto", "xgmi"):
        # the mailboxes are laid out, mapped and litmus-tested when the
        # engine is built (PSEngine -> XgmiTransport.setup)
        return (XgmiTransport(rank, world, dev, store, aux=TorchDistTransport(), prefix=prefix),
                None, None, 0)
    if kind != "rccl":
        raise ValueError(f"transport {kind!r}: auto, xgmi, rccl or gloo")
    if rccl_comms_mode() == 1:
        # one native communicator, every collective on its comm stream in
        # program order (the conservative default)
        return RcclTransport(rank, world, dev, store=store, prefix="ss_rccl_data"), None, None, 1
    # three communicators, one per engine stream: data plane (main:
    # gradients), route (counts, bucket runs), pull (keys, rows)
    mk = lambda p: RcclTransport(rank, world, dev, store=store, prefix=p, serial=False)  # noqa: E731
    return mk("ss_rccl_data"), mk("ss_rccl_counts"), mk("ss_rccl_pull"), 3


def _rccl_fallback(rank: int, world: int, device, store):
    from .transport import RcclTransport

    if world <= 1:
        return RcclTransport(0, 1, torch.device(device), uid=RcclTransport.new_unique_id())
    return RcclTransport(rank, world, torch.device(device), store=store, prefix="ss_rccl_fb")


def build_engine(kind: str, rank: int, world: int, device, store,
                 make_engine: Callable, log: Optional[Callable[[str], None]] = None,
                 prefix: str = "ss_xgmi"):
    """Build the round engine on the selected data plane, falling back from
    the xGMI mailboxes to RCCL when ``kind`` is auto.  ``make_engine(tr, ct,
    pt)`` builds a PSEngine (its construction lays out and litmus-tests the
    mailboxes).  Returns (engine, transports, PlaneInfo); every rank takes
    the same branch (the litmus verdict is agreed collectively)."""
    from .xgmi import XgmiTransport

    tr, ct, pt, comms = make_transports(kind, rank, world, device, store, prefix)
    fell, reason = False, ""
    litmus = []
    try:
        engine = make_engine(tr, ct, pt)
    except (RuntimeError, ValueError) as e:
        if not (isinstance(tr, XgmiTransport) and kind == "auto"):
            raise
        fell, reason = True, str(e)
        litmus = [dict(tier=t, passed=ok, s=dt, **({"why": w} if w else {}))
                  for t, ok, dt, w in tr.litmus_log]
        if log is not None:
            log(f"xgmi mailboxes unusable ({e}); falling back to RCCL")
        # free the arenas before the RCCL engine sizes its ring on free memory
        tr.close()
        del tr
        gc.collect()
        torch.cuda.empty_cache()
        tr, ct, pt, comms = _rccl_fallback(rank, world, device, store), None, None, 1
        engine = make_engine(tr, None, None)
    info = PlaneInfo(transport=getattr(tr, "label", type(tr).__name__), plane=_plane_of(tr),
                     fell_back=fell, fallback_reason=reason, comms=comms, litmus=litmus)
    if isinstance(tr, XgmiTransport):
        d = tr.describe()
        info.xgmi_tier, info.devices, info.litmus = d["xgmi_tier"], d["devices"], d["litmus"]
    else:
        info.devices = distinct_devices(store, rank, world, device)
    return engine, (tr, ct, pt), info
