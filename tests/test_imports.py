"""Every module of the package imports on a machine without a GPU (a syntax
or indentation error in a GPU-only model module otherwise surfaces only on
the GPU box)."""
import importlib
import pkgutil

import swiftsnails_amd


def test_every_module_imports():
    failed = {}
    for m in pkgutil.walk_packages(swiftsnails_amd.__path__, "swiftsnails_amd."):
        if m.name.endswith("__main__"):
            continue
        try:
            importlib.import_module(m.name)
        except Exception as e:  # noqa: BLE001 — report every module that fails
            failed[m.name] = repr(e)
    assert not failed, failed
