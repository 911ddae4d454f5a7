"""End-to-end CLI: reference-style role processes over TCP loopback (CPU) and
the MI355X collective mode (GPU, world 1) with backup + resume."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cli_master_server_worker_processes(tmp_path):
    port = _port()
    out = tmp_path / "final.txt"
    sets = ["--set", f"listen_addr=tcp://127.0.0.1:{port}",
            "--set", f"master_addr=tcp://127.0.0.1:{port}",
            "--set", f"param_output={out}", "--set", "num_iters=30"]
    base = [sys.executable, "-m", "swiftsnails_amd.launch", "--config",
            os.path.join(ROOT, "configs", "dense_lr_cpu.conf")] + sets
    env = dict(os.environ, PYTHONPATH=ROOT)
    procs = [subprocess.Popen(base + ["--role", r], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE) for r in ("master", "server", "worker")]
    for p in procs:
        try:
            p.wait(120)
        except subprocess.TimeoutExpired:
            p.kill()
            raise
    for p in procs:
        assert p.returncode == 0, p.stderr.read().decode()[-2000:]
    lines = out.read_text().splitlines()
    assert len(lines) == 64  # dense_dim weights, one "key\tvalue" line each
    assert sorted(int(x.split("\t")[0]) for x in lines) == list(range(64))


@pytest.mark.gpu
def test_cli_gpu_sparse_lr_backup_and_resume(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    common = [sys.executable, "-m", "swiftsnails_amd.launch", "--config",
              os.path.join(ROOT, "configs", "sparse_lr_10m.conf"),
              "--set", "batch_size=4096", "--set", "num_features=1000000",
              "--set", f"param_backup_root={tmp_path}", "--set", "param_backup_period=5"]
    r = subprocess.run(common + ["--steps", "10", "--set", f"param_output={tmp_path}/final"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["samples_per_s"] > 0 and stats["steps"] == 10 and stats["rounds_timed"] == 10
    assert (tmp_path / "param-5.shard0-of-1.bin").exists()
    assert (tmp_path / "param-10.shard0-of-1.bin").exists()
    txt = tmp_path / "final.shard0-of-1.txt"
    assert txt.exists() and txt.read_text().count("\n") > 1000
    r2 = subprocess.run(common + ["--steps", "2", "--set", f"resume_from={tmp_path}/param-10"],
                        cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert json.loads(r2.stdout.strip().splitlines()[-1])["start_round"] == 10
    # restart-after-failure: resume_from=latest picks the newest complete
    # backup and continues the round count (backups numbered from there)
    (tmp_path / "param-10.shard0-of-1.bin").rename(tmp_path / "param-10.partial")
    r3 = subprocess.run(common + ["--steps", "5", "--set", "resume_from=latest"],
                        cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r3.returncode == 0, r3.stderr[-3000:]
    assert json.loads(r3.stdout.strip().splitlines()[-1])["start_round"] == 5
    assert (tmp_path / "param-10.shard0-of-1.bin").exists()  # written again at round 10


@pytest.mark.gpu
def test_cli_gpu_trace_phases(tmp_path):
    """`trace: 1`: per-phase device times (route / pull / compute / push, HIP
    events on the stream each phase runs on) in the job's stats line."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "swiftsnails_amd.launch", "--config",
                        os.path.join(ROOT, "configs", "sparse_lr_10m.conf"), "--steps", "6",
                        "--set", "batch_size=4096", "--set", "num_features=1000000",
                        "--set", "trace=1", "--set", "table_stats=0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    tr = json.loads(r.stdout.strip().splitlines()[-1])["trace"]
    for ph in ("route", "pull", "compute", "push"):
        assert tr["calls"][ph] >= 6 and tr["gpu_s"][ph] > 0, (ph, tr)
    assert tr["calls"]["step"] == 6


def test_cluster_script_two_servers_two_workers(tmp_path):
    """tools/cluster_test.sh: master + 2 servers + 2 workers as processes; each
    server dumps its own shard, together covering every key exactly once."""
    out = tmp_path / "final.txt"
    env = dict(os.environ, PYTHONPATH=ROOT, SERVERS="2", WORKERS="2", LOG_DIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "cluster_test.sh"),
                        os.path.join(ROOT, "configs", "dense_lr_cpu.conf"),
                        "--set", "num_iters=15", "--set", f"param_output={out}"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    shards = sorted(tmp_path.glob("final.txt.s*"))
    assert len(shards) == 2
    keys = [int(ln.split("\t")[0]) for f in shards for ln in f.read_text().splitlines()]
    assert sorted(keys) == list(range(64))


def test_latest_checkpoint_picks_newest_complete_set(tmp_path):
    from swiftsnails_amd.utils import checkpoint as ck

    for name in ("param-5.shard0-of-2.bin", "param-5.shard1-of-2.bin",
                 "param-10.shard0-of-2.txt", "param-10.shard1-of-2.txt",
                 "param-20.shard1-of-2.bin",  # incomplete: rank 0 never wrote
                 "param-7.shard0-of-1.bin.tmp", "other-30.shard0-of-1.bin"):
        (tmp_path / name).write_bytes(b"x")
    assert ck.latest_checkpoint(str(tmp_path)) == (str(tmp_path / "param-10"), 10, 2, "text")
    assert ck.latest_checkpoint(str(tmp_path / "missing")) is None


@pytest.mark.gpu
def test_cli_gpu_graph_replay_counts_rounds_run():
    """With `graph: 1` a replay runs a whole graph (4 ring periods = 16 steps
    by default), so 10 requested steps run 16 rounds and the stats divide by
    the rounds the device ran."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "swiftsnails_amd.launch", "--config",
                        os.path.join(ROOT, "configs", "sparse_lr_10m.conf"),
                        "--set", "batch_size=4096", "--set", "num_features=1000000",
                        "--set", "graph=1", "--steps", "10", "--warmup", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["hipgraph"] is True and stats["steps"] == 10
    assert stats["rounds_timed"] % 4 == 0 and stats["rounds_timed"] >= 10
    assert stats["ms_per_step"] == pytest.approx(1000 * stats["seconds"] / stats["rounds_timed"])
