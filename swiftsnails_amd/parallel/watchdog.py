"""Failure detection: round watchdog, cross-rank heartbeats, fault injection.

The reference's only failure handling is timeouts that abort the process:
``StateBarrier::time_limit`` watchdogs on node registration, hashfrag fetch
and master registration (/root/reference/src/utils/Barrier.h:90-101,
core/system/node_init.h:79-82,136-143, core/system/master/init.h:68-70),
``CHECK(1 == 2)`` on expiry.  The collective design needs the same at ROUND
granularity: a collective that one rank never joins hangs every other rank
inside RCCL, so

* ``Watchdog`` — a host thread that expects a ``beat()`` per training round
  within ``round_timeout`` seconds; on expiry it runs the abort hooks
  (``ncclCommAbort`` on the RCCL communicators, which makes the stuck
  kernels return) and terminates the process with a distinct exit code, so
  ``torchrun`` tears the job down instead of hanging until its own timeout;
* ``Heartbeat`` — every rank bumps a counter in the rendezvous TCPStore every
  ``interval`` seconds and watches everyone else's; a peer whose counter has
  not moved for ``peer_timeout`` seconds is reported dead (a crashed or
  wedged process, not just a slow round) and the same abort path runs;
* ``FaultInjector`` — ``SS_FAULT=hang|crash|slow[:rank=R][:step=S][:secs=T]``
  makes the failure paths testable (tests/test_watchdog.py).

Recovery is restart-from-checkpoint (``resume_from``, utils/checkpoint.py),
the same capability level as the reference plus resume.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, List, Optional

from ..utils.logging import get_logger

log = get_logger("swiftsnails.watchdog")

EXIT_ROUND_TIMEOUT = 3
EXIT_PEER_DEAD = 4
EXIT_INJECTED = 17


class FailureHandler:
    """Runs abort hooks once, then exits the process (unless ``exit=False``)."""

    def __init__(self, exit_process: bool = True, grace: float = 2.0):
        self.hooks: List[Callable[[], None]] = []
        self.exit_process = exit_process
        self.grace = grace
        self.reason: Optional[str] = None
        self._lock = threading.Lock()

    def add_hook(self, fn: Callable[[], None]) -> None:
        self.hooks.append(fn)

    def __call__(self, reason: str, code: int) -> None:
        with self._lock:
            if self.reason is not None:
                return
            self.reason = reason
        log.error("failure detected: %s — aborting communicators", reason)
        print(f"[swiftsnails] FAILURE: {reason}", file=sys.stderr, flush=True)
        for h in self.hooks:
            try:
                h()
            except Exception as e:  # abort is best effort
                log.error("abort hook failed: %s", e)
        if self.exit_process:
            time.sleep(self.grace)  # let the main thread surface the aborted op first
            sys.stderr.flush()
            os._exit(code)


class Watchdog:
    """Expects ``beat()`` at least every ``timeout`` seconds while armed."""

    def __init__(self, timeout: float, on_fail: Callable[[str, int], None], name: str = "round",
                 poll: float = 0.25):
        self.timeout = float(timeout)
        self.on_fail = on_fail
        self.name = name
        self.poll = poll
        self._last = time.monotonic()
        self._tag = None
        self._armed = True
        self._stop = threading.Event()
        self.fired = False
        self._t = threading.Thread(target=self._run, name=f"ss-watchdog-{name}", daemon=True)
        self._t.start()

    def beat(self, tag=None) -> None:
        self._last = time.monotonic()
        self._tag = tag

    def pause(self) -> None:
        self._armed = False

    def resume(self) -> None:
        self._last = time.monotonic()
        self._armed = True

    def stop(self) -> None:
        self._stop.set()
        self._t.join(timeout=5)

    def _run(self):
        while not self._stop.wait(self.poll):
            if self._armed and time.monotonic() - self._last > self.timeout:
                self.fired = True
                self.on_fail(f"{self.name} watchdog: no progress for {self.timeout:.1f}s "
                             f"(last completed: {self._tag})", EXIT_ROUND_TIMEOUT)
                return


class Heartbeat:
    """Counter-based liveness over a key-value store (TCPStore-compatible:
    ``set``, ``get``, ``check``).  Counters, not timestamps, so host clocks
    need not agree."""

    def __init__(self, store, rank: int, world: int, on_fail: Callable[[str, int], None],
                 interval: float = 2.0, peer_timeout: float = 30.0, prefix: str = "ss_hb"):
        self.store, self.rank, self.world = store, rank, world
        self.on_fail = on_fail
        self.interval, self.peer_timeout, self.prefix = interval, peer_timeout, prefix
        self._stop = threading.Event()
        self._seen = {}  # peer -> (counter, monotonic time it last changed)
        self._n = 0
        self.dead: Optional[int] = None
        self._beat()
        self._t = threading.Thread(target=self._run, name="ss-heartbeat", daemon=True)
        self._t.start()

    def _key(self, r: int) -> str:
        return f"{self.prefix}/{r}"

    def _beat(self):
        self._n += 1
        self.store.set(self._key(self.rank), str(self._n))

    def stop(self) -> None:
        self._stop.set()
        self._t.join(timeout=5)

    def _run(self):
        t0 = time.monotonic()
        while not self._stop.wait(self.interval):
            try:
                self._beat()
                now = time.monotonic()
                for r in range(self.world):
                    if r == self.rank:
                        continue
                    k = self._key(r)
                    v = int(self.store.get(k)) if self.store.check([k]) else 0
                    last = self._seen.get(r)
                    if last is None or last[0] != v:
                        self._seen[r] = (v, now)
                    elif now - last[1] > self.peer_timeout and now - t0 > self.peer_timeout:
                        self.dead = r
                        self.on_fail(f"rank {r} stopped heart-beating for "
                                     f"{now - last[1]:.1f}s", EXIT_PEER_DEAD)
                        return
            except Exception as e:  # the store itself died (rank 0 gone)
                if self._stop.is_set():
                    return
                self.dead = 0
                self.on_fail(f"heartbeat store unreachable: {e}", EXIT_PEER_DEAD)
                return


class FaultInjector:
    """``SS_FAULT=kind[:rank=R][:step=S][:secs=T][:ms=M][:p=P]``; kind in
    hang, crash, slow (once, at step S), delay (a straggler: rank R's host
    loop sleeps M ms in every step from S on, or in a fraction P of them;
    ``delay:<rank>:<ms>`` also parses) and gpudelay (the same as device work:
    a kernel that keeps one wave busy for M ms on the rank's current stream —
    a slow or contended GPU rather than a slow host)."""

    def __init__(self, spec: Optional[str] = None, rank: int = 0):
        spec = spec if spec is not None else os.environ.get("SS_FAULT", "")
        self.kind = None
        self.rank, self.step, self.secs = None, 0, 1.0
        self.me = rank
        if not spec:
            return
        parts = spec.split(":")
        self.kind = parts[0]
        self.p = 1.0
        if self.kind not in ("hang", "crash", "slow", "delay", "gpudelay"):
            raise ValueError(f"SS_FAULT kind {self.kind!r}")
        if self.kind in ("delay", "gpudelay"):
            self.secs = 0.001
            pos = [p for p in parts[1:] if "=" not in p]
            if pos:  # delay:<rank>:<ms>
                self.rank = int(pos[0])
                if len(pos) > 1:
                    self.secs = float(pos[1]) / 1e3
        for p in parts[1:]:
            k, _, v = p.partition("=")
            if k == "rank":
                self.rank = int(v)
            elif k == "step":
                self.step = int(v)
            elif k == "secs":
                self.secs = float(v)
            elif k == "ms":
                self.secs = float(v) / 1e3
            elif k == "p":
                self.p = float(v)

    def maybe(self, step: int) -> None:
        if self.kind is None or (self.rank is not None and self.rank != self.me):
            return
        if self.kind in ("delay", "gpudelay"):
            # a fraction p of the steps, chosen by a hash of the step (the
            # same steps on every run)
            if step < self.step or (self.p < 1.0 and
                                    ((step * 2654435761) % 1000003) / 1000003.0 >= self.p):
                return
            if self.kind == "delay":
                time.sleep(self.secs)
            else:
                import torch

                from .._native import hip

                hip().spin_us(self.secs * 1e6, torch.cuda.current_stream().cuda_stream)
            return
        if step != self.step:
            return
        log.error("SS_FAULT: injecting %s on rank %d at step %d", self.kind, self.me, step)
        if self.kind == "crash":
            sys.stderr.flush()
            os._exit(EXIT_INJECTED)
        elif self.kind == "hang":
            while True:
                time.sleep(3600)
        else:
            time.sleep(self.secs)
