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


def _child_main(fn, args, q):
    try:
        fn(*args)
        q.put(("ok", ""))
    except BaseException:  # noqa: BLE001 - the parent re-raises it
        import traceback

        q.put(("fail", traceback.format_exc()))


def in_child(fn, *args, timeout: float = 240.0) -> None:
    """Run ``fn(*args)`` (a module-level test body) — in this process, or
    with SS_TEST_IN_CHILD=1 in a spawned one, re-raising its failure here.
    The hipGraph tests used to need the child: a replay in a process that had
    already run many other GPU tests segfaulted inside hipGraphLaunch.  The
    cause was teardown order — a collected worker's graph execs outlived the
    round engine's HIP events their nodes reference — and the graphs are now
    owned so they are destroyed first (models/base.py _GraphSet), so the
    graph tests run in the one pytest process again."""
    if os.environ.get("SS_TEST_IN_CHILD", "0") != "1":
        saved = dict(os.environ)  # the bodies set SS_* knobs for themselves
        try:
            fn(*args)
        finally:
            os.environ.clear()
            os.environ.update(saved)
        return
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child_main, args=(fn, args, q))
    p.start()
    res = collect(q, [p], 1, timeout)[0]
    p.join(60)
    if res[0] != "ok":
        raise AssertionError("in the child process:\n" + res[1])
