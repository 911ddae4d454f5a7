"""Tracing / profiling hooks (the reference has none beyond an unused Timer,
/root/reference/src/utils/Timer.h:14-44 — SURVEY §5).

* ``Tracer.range(name)``: a roctx range (visible in ``rocprofv3
  --marker-trace`` timelines) plus host wall-time accounting per name;
* ``Tracer.gpu_range(name)``: HIP-event bracketed device time per name
  (no host synchronisation until ``summary()``);
* ``Metrics``: throughput counters (samples/s, keys/s, bytes/s) per rank.

roctx comes from the ROCm runtime torch already loaded (libroctx64); if it
cannot be found, ranges degrade to host timing only.
"""
from __future__ import annotations

import contextlib
import ctypes
import time
from collections import defaultdict
from typing import Optional

import torch


_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx or None
    # the rocprofiler-sdk roctx first: rocprofv3 --marker-trace records its
    # ranges; the legacy libroctx64 ranges do not reach rocprofv3
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                 "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return None


class Tracer:
    def __init__(self, enabled: bool = True, roctx: bool = True):
        self.enabled = enabled
        self._rx = _load_roctx() if (enabled and roctx) else None
        self.host_time = defaultdict(float)
        self.calls = defaultdict(int)
        self._gpu: list[tuple[str, torch.cuda.Event, torch.cuda.Event]] = []

    @contextlib.contextmanager
    def range(self, name: str):
        if not self.enabled:
            yield
            return
        if self._rx:
            self._rx.roctxRangePushA(name.encode())
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.host_time[name] += time.perf_counter() - t0
            self.calls[name] += 1
            if self._rx:
                self._rx.roctxRangePop()

    @contextlib.contextmanager
    def gpu_range(self, name: str, stream: Optional[torch.cuda.Stream] = None):
        if not self.enabled or not torch.cuda.is_available():
            yield
            return
        s = stream or torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        with self.range(name):
            yield
        b.record(s)
        self._gpu.append((name, a, b))

    def summary(self) -> dict:
        gpu = defaultdict(float)
        for name, a, b in self._gpu:
            b.synchronize()
            gpu[name] += a.elapsed_time(b) * 1e-3
        self._gpu.clear()
        return {"host_s": dict(self.host_time), "gpu_s": dict(gpu), "calls": dict(self.calls)}


class Metrics:
    """Per-rank counters.  ``add`` takes host numbers; ``add_device`` takes
    a device scalar tensor (a count a kernel wrote) and accumulates it on the
    device, so the hot path never syncs — ``counters`` folds those in when
    read (one sync)."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self._host = defaultdict(float)
        self._dev: dict = {}

    def add(self, **kw):
        for k, v in kw.items():
            self._host[k] += v

    def device_block(self, names, device) -> torch.Tensor:
        """A persistent float64 device vector whose entries accumulate the
        counters ``names`` (a kernel adds into it; folded into ``counters``
        when read)."""
        key = tuple(names)
        blk = self._dev.get(key)
        if blk is None:
            blk = self._dev[key] = torch.zeros(len(names), dtype=torch.float64, device=device)
        return blk

    def add_device(self, **kw):
        for k, v in kw.items():
            acc = self._dev.get(k)
            if acc is None:
                acc = self._dev[k] = torch.zeros(1, dtype=torch.float64, device=v.device)
            acc.add_(v.reshape(-1)[:1].to(torch.float64))

    @property
    def counters(self) -> dict:
        out = defaultdict(float, self._host)
        for k, acc in self._dev.items():
            if isinstance(k, tuple):
                for name, v in zip(k, acc.tolist()):
                    out[name] += v
            else:
                out[k] += float(acc.item())
        return out

    def rates(self) -> dict:
        el = max(1e-9, time.perf_counter() - self.t0)
        return {f"{k}_per_s": v / el for k, v in self.counters.items()}
