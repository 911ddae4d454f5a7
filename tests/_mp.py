"""Multi-process test plumbing: a file rendezvous (no TCP port to race for:
a port picked free and bound later can be taken in between on a shared box)
and result collection that fails fast when a rank process dies."""
import os
import queue
import tempfile
import time
import uuid


def file_init() -> str:
    """A fresh ``file://`` init method for ``init_process_group``."""
    return "file://" + os.path.join(tempfile.gettempdir(),
                                    f"ss_rdzv_{os.getpid()}_{uuid.uuid4().hex}")


def init_gloo(init: str, rank: int, world: int) -> None:
    import torch.distributed as dist

    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)


def collect(q, procs, n: int, timeout: float) -> list:
    """``n`` results from ``q``; raises as soon as a rank exits non-zero
    without having produced its result, or at the timeout (killing the rest)."""
    out, t_end = [], time.monotonic() + timeout
    while len(out) < n:
        try:
            out.append(q.get(timeout=1.0))
            continue
        except queue.Empty:
            pass
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if dead or time.monotonic() > t_end:
            for p in procs:
                if p.is_alive():
                    p.kill()
            raise RuntimeError(f"rank process exit codes {[p.exitcode for p in procs]}"
                               if dead else f"no result within {timeout} s")
    return out
