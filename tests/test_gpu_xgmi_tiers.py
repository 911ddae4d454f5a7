"""The fail-safe xGMI start-up: publish tiers, the full-size litmus, the
forced fallback chain and the run-time round-tag check (parallel/xgmi.py,
parallel/select.py, csrc/hip/xgmi.hip).

All ranks share cuda:0 (the only device of the test box); SS_XGMI_FENCE_ALL
makes the fenced tier release towards same-device peers too, so its fences
and acquires really execute here.  The 8-GPU node runs the same code with
peers on distinct devices (`remote` mask from the PCI bus ids)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from test_gpu_multiproc import _free_port, _run

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("tier", ["drain", "fenced"])
def test_tier_litmus_and_engine_oracle(world, tier):
    """Each xGMI tier passes the litmus with `world` processes on one GPU and
    then carries the engine's rounds (round tags verified on every wait)
    reproducing the single-table oracle."""
    env = {"SS_XGMI_VERIFY": "1"}
    if tier == "fenced":
        env.update(SS_XGMI_FORCE_TIER="fenced", SS_XGMI_FENCE_ALL="1")
    planes = _run(world, list(range(world)), list(range(world)), "adagrad", "xgmi", env)
    for p in planes:
        assert p["xgmi_tier"] == tier and p["devices"] == 1 and p["xgmi_verify"]
        lit = p["litmus"]
        assert lit[-1] == {"tier": tier, "passed": True, "s": lit[-1]["s"]}
        if tier == "fenced":
            assert lit[0]["tier"] == "drain" and not lit[0]["passed"]
            assert "forced" in lit[0]["why"]


def test_server_gradient_staging_oracle():
    """SS_SRV_STAGE=1 (off by default: measured neutral): the servers stream
    the peers' gradient rows out of the mailbox into a cached buffer
    (k_xstage) before the merge; the rounds still reproduce the oracle."""
    planes = _run(4, list(range(4)), list(range(4)), "adagrad", "xgmi", {"SS_SRV_STAGE": "1"})
    assert all(p["xgmi_tier"] in ("drain", "fenced") for p in planes)


def test_stale_round_tag_is_detected():
    """A tag overwritten between a put and its wait (what a flag overtaking
    its data looks like) sets the sticky error, and poll_error raises
    without a device sync."""
    os.environ["SS_XGMI_VERIFY"] = "1"
    try:
        from swiftsnails_amd._native import hip
        from swiftsnails_amd.parallel.xgmi import XgmiTransport

        dev = torch.device("cuda", 0)
        tr = XgmiTransport(0, 1, dev, None, timeout_s=10)
        tr.setup({"c": (1, [4096])})
        assert tr.tier == "drain"
        tr.poll_error()
        src = torch.arange(1024, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev)
        tr.put("c", 0, [(src, [0], None, 1024)], stream=st)
        base = tr.arena_of("c", 0).base
        tags = torch.utils.dlpack.from_dlpack(
            hip().dlpack_view(base + 128 * 16 * 16, [16], 0, 32, 0))
        tags.fill_(7)  # stale: not this round's number
        tr.wait("c", 0, stream=st)
        st.synchronize()
        with pytest.raises(RuntimeError, match="round tag"):
            tr.poll_error()
        with pytest.raises(RuntimeError, match="round tag"):
            tr.check()
        tr.close()
    finally:
        del os.environ["SS_XGMI_VERIFY"]


def test_failed_tier_error_bits_do_not_fail_next_tier(monkeypatch):
    """A drain-tier litmus that fails with sticky error bits set (what a stale
    round tag under SS_XGMI_VERIFY=1 leaves behind) must not fail the fenced
    tier's litmus, nor the first rounds after it: the error words are cleared
    before each tier."""
    monkeypatch.setenv("SS_XGMI_VERIFY", "1")
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    orig = XgmiTransport._litmus

    def litmus(self, fail=False):
        ok, why = orig(self, fail)
        if self.tier is None and not getattr(self, "_poisoned", False):
            self._poisoned = True  # the drain tier: a stale tag seen by the waits
            torch.cuda.synchronize()
            for e in self._errs:
                e.fill_(4)
            torch.cuda.synchronize()
            return False, "stale round tag (injected)"
        return ok, why

    monkeypatch.setattr(XgmiTransport, "_litmus", litmus)
    dev = torch.device("cuda", 0)
    tr = XgmiTransport(0, 1, dev, None, timeout_s=10)
    tr.setup({"c": (2, [4096])})
    assert tr.tier == "fenced"
    assert [x[1] for x in tr.litmus_log] == [False, True]
    tr.poll_error()
    tr.check()
    src = torch.arange(1024, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    for r in range(4):
        tr.put("c", r % 2, [(src, [0], None, 1024)], stream=st)
        tr.wait("c", r % 2, stream=st)
    st.synchronize()
    tr.poll_error()
    tr.check()
    got = tr.region("c", 0, 1, torch.int32)[:1024]
    assert torch.equal(got, src)
    tr.close()


def _bench(env, extra=(), nproc=1, shape=("--steps", "4", "--warmup", "2", "--batch", "4096",
                                          "--features", "2000000")):
    e = dict(os.environ, GLOO_SOCKET_IFNAME="lo", **env)
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc)]
        e["SS_BENCH_DEVICE"] = "0"
    cmd += [*shape, *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


@pytest.mark.parametrize("force,plane,tier,fell", [
    ("", "xgmi", "drain", False),
    ("fenced", "xgmi", "fenced", False),
    ("rccl", "rccl", None, True),
])
def test_bench_fallback_chain(force, plane, tier, fell):
    """bench.py through the N>1 engine path on one GPU (a size-1 plane):
    each step of the chain drain -> fenced -> RCCL runs end to end when the
    earlier tiers are made to fail, and the JSON names what ran."""
    env = {"SS_ENGINE_GENERAL": "xgmi"}
    if force:
        env["SS_XGMI_FORCE_TIER"] = force
    j, err = _bench(env)
    c = j["config"]
    assert c["plane"] == plane and c["xgmi_tier"] == tier and c["fell_back"] is fell, c
    assert c["devices"] == 1 and j["value"] > 0 and np.isfinite(c["loss_last"])
    # the number says which round layout produced it
    lay = c["layout"]
    for k in ("depth", "server_stream", "bd_target_dist", "srv_sub_buckets", "claim",
              "srv_rbits", "buckets_per_dest"):
        assert k in lay, lay
    assert lay["depth"] >= 3 and lay["srv_sub_buckets"] >= 1 and lay["bd_target_dist"] > 0
    if plane == "xgmi":
        # one rank with a device of its own: the server stream exists and the
        # calibration decided whether to keep it; the layout reports that
        ss = c["calibration"]["server_stream"]
        assert ss["server_stream"] == lay["server_stream"]
        assert len(ss["off_ms"]) == len(ss["on_ms"]) == ss["windows"]
        assert lay["claim"] and lay["srv_rbits"] > 0
        # SS_XCHG=auto (default): both exchanges timed, the JSON names the pick
        x = c["calibration"]["exchange"]
        assert x["exchange"] == c["exchange"] and x["default"] == "unique"
        assert len(x["unique_ms"]) == len(x["records_ms"]) == x["windows"]
    if fell:
        assert "litmus failed on every tier" in c["fallback_reason"]
        assert "falling back to RCCL" in err


def test_bench_world2_fenced_verified():
    """bench.py at N = 2 (both ranks on cuda:0) on the fenced tier with round
    tags verified every wait: the driver's N>1 path on the defensive tier."""
    j, _ = _bench({"SS_XGMI_FORCE_TIER": "fenced", "SS_XGMI_FENCE_ALL": "1",
                   "SS_XGMI_VERIFY": "1"}, nproc=2,
                  shape=("--steps", "6", "--warmup", "3", "--batch", "8192", "--features",
                         "4000000", "--cal-steps", "0"))
    c = j["config"]
    assert c["plane"] == "xgmi" and c["xgmi_tier"] == "fenced" and not c["fell_back"]
    assert c["devices"] == 1 and j["n_gpus"] == 2
    assert c["loss_last"] < c["loss_first"]
    assert np.isfinite(j["value"]) and j["value"] > 0


@pytest.mark.parametrize("pick", ["records", "unique"])
def test_bench_world2_exchange_calibration(pick):
    """bench.py at N = 2 (both ranks on cuda:0) with SS_XCHG=auto: the unique
    and the record exchange are built on one table, timed on the live world,
    and the loser's engine and arenas are torn down on every rank before the
    timed steps (SS_CAL_XCHG forces either outcome, so both teardowns run);
    the survivor then trains on."""
    j, _ = _bench({"SS_CAL_XCHG": pick}, nproc=2,
                  shape=("--steps", "6", "--warmup", "3", "--batch", "8192", "--features",
                         "4000000", "--cal-steps", "3", "--cal-windows", "1"))
    c = j["config"]
    assert c["plane"] == "xgmi" and c["exchange"] == pick
    x = c["calibration"]["exchange"]
    assert x["exchange"] == pick and len(x["unique_ms"]) == len(x["records_ms"]) == 1
    assert c["loss_last"] < c["loss_first"]
    assert np.isfinite(j["value"]) and j["value"] > 0
