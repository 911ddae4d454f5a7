"""Cheap current-stream handling for the per-step launch path.

A training step enqueues a dozen kernels on three streams.  Going through
``torch.cuda.current_stream()`` / ``torch.cuda.stream(s)`` for each costs a
resolution chain per call (default device -> availability check -> env
lookups -> ``Stream`` object): measured ~45 us of host time per word2vec step
(0.13 ms, host-bound), i.e. a third of it.  These helpers take the device
index explicitly and talk to the same runtime state torch uses
(``torch._C._cuda_getCurrentRawStream`` / ``_cuda_setStream``), so a stream
switched here is the stream torch ops see, and vice versa.
"""
from __future__ import annotations

import torch

_C = torch._C
_raw = getattr(_C, "_cuda_getCurrentRawStream", None)
_get = getattr(_C, "_cuda_getCurrentStream", None)
_set = getattr(_C, "_cuda_setStream", None)
_dev = getattr(_C, "_cuda_getDevice", None)


def current_device() -> int:
    return _dev() if _dev is not None else torch.cuda.current_device()


def current_raw(device_index: int | None = None) -> int:
    """hipStream_t (as int) of the current stream of ``device_index``."""
    idx = current_device() if device_index is None else device_index
    if _raw is not None:
        return _raw(idx)
    return torch.cuda.current_stream(idx).cuda_stream


def current(device_index: int) -> torch.cuda.Stream:
    """The current stream of ``device_index`` as a torch ``Stream``."""
    return torch.cuda.current_stream(device_index)


class use_stream:
    """``with use_stream(s):`` — ``torch.cuda.stream(s)`` without the default
    device resolution (``s`` must be a torch ``Stream``)."""

    __slots__ = ("s", "prev")

    def __init__(self, s: torch.cuda.Stream):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        if _get is None or _set is None:
            self.prev = torch.cuda.current_stream(s.device_index)
            torch.cuda.set_stream(s)
            return s
        self.prev = _get(s.device_index)
        _set(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        p = self.prev
        if isinstance(p, torch.cuda.Stream):
            torch.cuda.set_stream(p)
        else:
            _set(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False
