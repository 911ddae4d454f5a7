import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_memlog(request):
    """SS_TEST_MEMLOG=<file>: one line per GPU test with the device's free
    memory and the caching allocator's reservation before it (diagnostics of
    state that builds up over a long single-process GPU run)."""
    path = os.environ.get("SS_TEST_MEMLOG")
    if path and "gpu" in request.keywords:
        import torch

        free, total = torch.cuda.mem_get_info()
        with open(path, "a") as f:
            f.write(f"{request.node.nodeid} free={free / 2**30:.1f}G "
                    f"reserved={torch.cuda.memory_reserved() / 2**30:.1f}G\n")
    yield
    if "gpu" in request.keywords and os.environ.get("SS_TEST_GC", "1") != "0":
        # tear a GPU test's engines down now, not whenever a later test's
        # allocations trigger the cyclic GC: an earlier test's xGMI arenas
        # (IPC exports, host-mapped words) freed in the middle of a later
        # test's hipGraph replays segfaulted inside hipGraphLaunch
        import gc

        import torch

        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
