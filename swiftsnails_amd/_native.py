"""Loader for the in-tree native extensions (``swiftsnails_amd/_lib``).

``torch`` is imported first on purpose: the HIP module links
``libamdhip64.so.7`` / ``librccl.so.1`` by soname, and when torch's bundled
ROCm runtime is already mapped the dynamic loader re-uses it, so kernels,
the caching allocator and RCCL all share ONE HIP runtime.

GPU code never silently falls back: ``hip()`` raises if the extension is
missing, and ``require_gpu_native()`` raises on a GPU box where the module
cannot be loaded.
"""
from __future__ import annotations

import importlib
import os
import sys

import torch  # noqa: F401  (must precede the HIP extension, see module doc)

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_mods: dict[str, object] = {}


class NativeExtensionMissing(ImportError):
    pass


def _load(name: str, autobuild: bool = True):
    if name in _mods:
        return _mods[name]
    if _LIB not in sys.path:
        sys.path.insert(0, _LIB)
    try:
        mod = importlib.import_module(name)
    except ImportError as e:
        if autobuild and os.environ.get("SS_NO_AUTOBUILD", "0") != "1":
            from . import _build

            try:
                if name == "_ss_hip":
                    _build.build_hip()
                else:
                    _build.build_host()
            except Exception as be:  # pragma: no cover - surfaced below
                raise NativeExtensionMissing(f"{name}: build failed: {be}") from e
            importlib.invalidate_caches()
            mod = importlib.import_module(name)
        else:
            raise NativeExtensionMissing(
                f"native extension {name} not built (python -m swiftsnails_amd._build)") from e
    _mods[name] = mod
    return mod


def hip():
    """The gfx950 kernel + RCCL module (loud failure if unavailable)."""
    return _load("_ss_hip")


def host():
    """The host C++ runtime module."""
    return _load("_ss_host")


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require_gpu_native() -> None:
    if gpu_available():
        hip()


def loaded_paths() -> list[str]:
    return [getattr(m, "__file__", "?") for m in _mods.values()]
