"""Failure detection (parallel/watchdog.py): round watchdog, heartbeats and
fault injection, over real multi-process gloo jobs on the CPU."""
import os
import subprocess
import sys
import textwrap
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_fires_without_beats_and_not_with():
    from swiftsnails_amd.parallel.watchdog import Watchdog

    fired = []
    w = Watchdog(0.5, lambda r, c: fired.append((r, c)), poll=0.05)
    for i in range(12):  # beating keeps it quiet
        time.sleep(0.1)
        w.beat(i)
    assert not fired
    w.pause()
    time.sleep(0.8)  # paused: quiet
    assert not fired
    w.resume()
    time.sleep(1.0)
    assert fired and fired[0][1] == 3 and "last completed: 11" in fired[0][0]
    w.stop()


class _DictStore:
    def __init__(self):
        self.d, self.lock = {}, threading.Lock()

    def set(self, k, v):
        with self.lock:
            self.d[k] = v.encode() if isinstance(v, str) else v

    def get(self, k):
        with self.lock:
            return self.d[k]

    def check(self, ks):
        with self.lock:
            return all(k in self.d for k in ks)


def test_heartbeat_detects_silent_peer():
    from swiftsnails_amd.parallel.watchdog import Heartbeat

    st = _DictStore()
    got = []
    a = Heartbeat(st, 0, 2, lambda r, c: got.append((r, c)), interval=0.05, peer_timeout=0.5)
    b = Heartbeat(st, 1, 2, lambda r, c: None, interval=0.05, peer_timeout=0.5)
    time.sleep(1.0)
    assert not got  # both alive
    b.stop()  # rank 1 goes silent
    time.sleep(1.5)
    assert got and got[0][1] == 4 and "rank 1" in got[0][0]
    assert a.dead == 1
    a.stop()


def test_fault_injector_spec():
    from swiftsnails_amd.parallel.watchdog import FaultInjector

    f = FaultInjector("slow:rank=1:step=2:secs=0.2", rank=1)
    t0 = time.time()
    f.maybe(1)
    f.maybe(2)
    assert time.time() - t0 >= 0.2
    FaultInjector("slow:rank=0:step=2:secs=5", rank=1).maybe(2)  # other rank: no-op
    with pytest.raises(ValueError):
        FaultInjector("explode")


def test_fault_injector_delay_every_step():
    """delay: a straggler rank sleeps in every step from `step` on."""
    from swiftsnails_amd.parallel.watchdog import FaultInjector

    for spec in ("delay:1:30", "delay:rank=1:ms=30"):
        f = FaultInjector(spec, rank=1)
        assert f.kind == "delay" and f.rank == 1 and abs(f.secs - 0.03) < 1e-9
        t0 = time.time()
        for i in range(4):
            f.maybe(i)
        assert time.time() - t0 >= 0.12
    t0 = time.time()
    FaultInjector("delay:0:500", rank=1).maybe(3)  # other rank: no-op
    g = FaultInjector("delay:rank=1:ms=500:step=5", rank=1)
    g.maybe(4)  # before its first step
    assert time.time() - t0 < 0.25


_WORKER = textwrap.dedent("""
    import os, sys, datetime
    sys.path.insert(0, %(root)r)
    import torch, torch.distributed as dist
    from swiftsnails_amd.parallel.watchdog import (FailureHandler, FaultInjector, Heartbeat,
                                                   Watchdog)
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank,
                            world_size=world, timeout=datetime.timedelta(seconds=120))
    store = dist.distributed_c10d._get_default_store()
    fail = FailureHandler(grace=0.2)
    wd = Watchdog(%(round_timeout)s, fail, poll=0.05)
    hb = Heartbeat(store, rank, world, fail, interval=0.1, peer_timeout=%(peer_timeout)s)
    fault = FaultInjector(rank=rank)
    x = torch.ones(4)
    for step in range(1, 40):
        dist.all_reduce(x)  # one collective "round"
        wd.beat(step)
        fault.maybe(step)
    hb.stop(); wd.stop()
    dist.destroy_process_group()
    print("clean exit", rank)
""")


def _run_job(tmp_path, fault, round_timeout=2.0, peer_timeout=3.0, world=2, timeout=60):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / "job.py"
    script.write_text(_WORKER % dict(root=ROOT, port=port, round_timeout=round_timeout,
                                     peer_timeout=peer_timeout))
    env = dict(os.environ, SS_FAULT=fault, GLOO_SOCKET_IFNAME="lo")
    procs = [subprocess.Popen([sys.executable, str(script), str(r), str(world)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    t0 = time.time()
    out = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=max(1, timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("job hung: watchdog did not fire")
        out.append((p.returncode, o, e))
    return out, time.time() - t0


def test_no_fault_job_exits_cleanly(tmp_path):
    out, _ = _run_job(tmp_path, "")
    assert all(rc == 0 for rc, _, _ in out), out


def test_hung_rank_is_detected_and_job_ends(tmp_path):
    """Rank 1 hangs after step 3: rank 0 blocks in the next collective; the
    round watchdogs end BOTH processes (exit 3) instead of hanging."""
    out, dt = _run_job(tmp_path, "hang:rank=1:step=3")
    codes = sorted(rc for rc, _, _ in out)
    assert codes == [3, 3], out
    assert all("watchdog" in e for _, _, e in out)
    assert dt < 45


def test_crashed_rank_is_detected(tmp_path):
    """Rank 1 dies: rank 0 does not hang (gloo error, missing heartbeats or the
    round watchdog — whichever comes first), the job ends non-zero."""
    out, dt = _run_job(tmp_path, "crash:rank=1:step=3", round_timeout=5.0, peer_timeout=1.5)
    rc0 = out[0][0]
    assert out[1][0] == 17  # the injected crash
    assert rc0 != 0, out[0]
    assert dt < 45
