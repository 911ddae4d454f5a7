"""Checkpoint formats (reference text format + binary) and resharded resume."""
import numpy as np
import pytest

from swiftsnails_amd.ops.host_table import HostTable
from swiftsnails_amd.ops.optim import InitConfig, Optimizer
from swiftsnails_amd.parallel.router import HashFrag
from swiftsnails_amd.utils import checkpoint as ck


def _table(dim=4, opt="adagrad", seed=0):
    t = HostTable(dim, 3, Optimizer(opt, lr=0.1), InitConfig("normal", 0.5, 0.01, seed=seed))
    keys = np.random.default_rng(seed).integers(0, 1 << 50, 2000).astype(np.int64)
    t.pull_keys(keys)
    t.push_keys(np.unique(keys), np.ones((len(np.unique(keys)), dim), np.float32))
    return t


def test_text_format_matches_reference_layout(tmp_path):
    t = _table(dim=1)
    p = str(tmp_path / "param-10.txt")
    n = ck.save_text(t, p, precision=6)
    lines = open(p).read().splitlines()
    assert n == len(lines) == t.size()
    k, v = lines[0].split("\t")  # "key\tvalue" (sparsetable.h:49-56)
    assert k.isdigit() and len(v.split()) == 1


@pytest.mark.parametrize("fmt", ["text", "bin"])
def test_roundtrip_exact_with_state(tmp_path, fmt):
    t = _table()
    p = str(tmp_path / ("c.txt" if fmt == "text" else "c.bin"))
    if fmt == "text":
        ck.save_text(t, p, precision=9, with_state=True)
    else:
        ck.save_binary(t, p)
    t2 = HostTable(4, 5, Optimizer("adagrad", lr=0.1), InitConfig("zero", 0, 0.01))
    (ck.load_text if fmt == "text" else ck.load_binary)(t2, p)
    a, b = t.to_dict(True), t2.to_dict(True)
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


def test_reference_vec_prefix_and_params_only(tmp_path):
    p = tmp_path / "ref.txt"
    p.write_text("17\tVec:\t0.5 -1.25 2 \n99\t3 4 5\n")
    t = HostTable(3, 2, Optimizer("adagrad"), InitConfig("zero", 0, 0.1))
    assert ck.load_text(t, str(p)) == 2
    d = t.to_dict(True)
    np.testing.assert_allclose(d[17], [0.5, -1.25, 2, 0.1, 0.1, 0.1])
    np.testing.assert_allclose(d[99], [3, 4, 5, 0.1, 0.1, 0.1])


def test_sharded_resume_on_different_world_size(tmp_path):
    src = _table(dim=2, seed=3)
    keys = np.array(list(src.to_dict().keys()), dtype=np.uint64)
    # split into 3 "server" shards by the world-3 router, save them
    hf3 = HashFrag(3, 64)
    m3 = hf3.rank_map()
    all_rows = src.to_dict(True)
    prefix = str(tmp_path / "ckpt" / "model")
    for r in range(3):
        t = HostTable(2, 2, Optimizer("adagrad", lr=0.1))
        mine = keys[ck.owner_filter(m3, r)(keys)]
        t.assign(mine.view(np.int64), np.stack([all_rows[int(k)] for k in mine]))
        ck.save_sharded(t, prefix, r, 3, fmt="bin" if r != 1 else "text")
    # resume on world 2
    hf2 = HashFrag(2, 64)
    m2 = hf2.rank_map()
    merged = {}
    for r in range(2):
        t = HostTable(2, 2, Optimizer("adagrad", lr=0.1))
        ck.load_sharded(t, prefix, owner_fn=ck.owner_filter(m2, r))
        d = t.to_dict(True)
        assert not (set(d) & set(merged))
        merged.update(d)
    assert set(merged) == set(all_rows)
    for k in all_rows:
        np.testing.assert_array_equal(merged[k], all_rows[k])


class _Chunked:
    """Wraps a table so export() yields many small chunks (as HbmTable does)."""

    def __init__(self, t, c):
        self.t, self.c = t, c

    def __getattr__(self, a):
        return getattr(self.t, a)

    def export(self, *a, **k):
        for kk, rr in self.t.export():
            for i in range(0, len(kk), self.c):
                yield kk[i:i + self.c], rr[i:i + self.c]


def test_streaming_binary_and_text_chunks(tmp_path):
    t = _table(dim=3, seed=5)
    p = str(tmp_path / "s.bin")
    assert ck.save_binary(_Chunked(t, 97), p) == t.size()
    hdr, keys, rows = ck.read_binary(p)
    chunks = list(ck.iter_binary(p, chunk=101))
    assert len(chunks) == -(-t.size() // 101)
    np.testing.assert_array_equal(np.concatenate([c[0] for c in chunks]), keys)
    np.testing.assert_array_equal(np.concatenate([c[1] for c in chunks]), rows)
    t2 = HostTable(3, 5, Optimizer("adagrad", lr=0.1), InitConfig("zero", 0, 0.01))
    assert ck.load_binary(t2, p, chunk=64) == t.size()
    a, b = t.to_dict(True), t2.to_dict(True)
    assert a.keys() == b.keys() and all(np.array_equal(a[k], b[k]) for k in a)
    # text: blocks much smaller than the file, cut at line ends
    pt = str(tmp_path / "s.txt")
    ck.save_text(t, pt, with_state=True)
    got = list(ck.iter_text(pt, 3, 5, block_bytes=1000))
    assert len(got) > 10
    assert sum(len(k) for k, _ in got) == t.size()


def test_binary_save_detects_size_mismatch(tmp_path):
    t = _table(dim=2)

    class Lying(_Chunked):
        def size(self):
            return self.t.size() - 1

    with pytest.raises(RuntimeError):
        ck.save_binary(Lying(t, 50), str(tmp_path / "x.bin"))
    assert not (tmp_path / "x.bin").exists() and not (tmp_path / "x.bin.tmp").exists()


class _CrashingTable:
    """Export yields one chunk, then the 'process dies' mid-dump."""

    def __init__(self, t):
        self.t, self.dim, self.width = t, t.dim, t.width

    def export(self):
        for i, kr in enumerate(self.t.export()):
            yield kr
            raise KeyboardInterrupt("crash while dumping")


def test_text_save_is_atomic_and_crash_leaves_no_shard(tmp_path):
    """a crash during a text backup must not leave a truncated
    shard under its final name for resume_from=latest to pick up."""
    t = _table(dim=2)
    root = tmp_path
    for r in range(2):  # round 5: a complete text set
        ck.save_sharded(t, str(root / "param-5"), r, 2, fmt="text")
    ck.save_sharded(t, str(root / "param-9"), 0, 2, fmt="text")
    with pytest.raises(KeyboardInterrupt):
        ck.save_text(_CrashingTable(t), ck.shard_path(str(root / "param-9"), 1, 2, "text"))
    assert not (root / "param-9.shard1-of-2.txt").exists()
    assert not list(root.glob("*.tmp"))
    assert ck.latest_checkpoint(str(root)) == (str(root / "param-5"), 5, 2, "text")


def test_load_sharded_uses_one_set_only(tmp_path):
    """stale shards of another world size (or format) next to the
    chosen set are never loaded into the table."""
    new, old = _table(dim=2, seed=1), _table(dim=2, seed=2)
    prefix = str(tmp_path / "param-7")
    ck.save_sharded(new, prefix, 0, 1, fmt="bin")          # the newer 1-server set
    for r in range(2):                                      # a stale 2-server set
        ck.save_sharded(old, prefix, r, 2, fmt="text")
    with pytest.raises(ValueError, match="world sizes"):
        ck.select_shards(prefix)
    t = HostTable(2, 2, Optimizer("adagrad", lr=0.1))
    ck.load_sharded(t, prefix, world=1)
    a, b = new.to_dict(True), t.to_dict(True)
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    with pytest.raises(FileNotFoundError):
        ck.load_sharded(t, prefix, world=3)
    # both formats of one shard: ambiguous unless fmt is given
    ck.save_sharded(new, prefix, 0, 1, fmt="text")
    with pytest.raises(ValueError, match="fmt"):
        ck.select_shards(prefix, world=1)
    assert ck.select_shards(prefix, world=1, fmt="bin") == [ck.shard_path(prefix, 0, 1, "bin")]


def test_latest_checkpoint_with_two_formats_in_one_round(tmp_path):
    """A round holding complete .bin and .txt sets of the same world (the
    checkpoint format changed between runs): the newest set is chosen with its
    format, and loading it reads that set only (no 'pass fmt=' error)."""
    import os
    import time

    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.utils import checkpoint as ck

    t = HostTable(2, 2, Optimizer("sgd", lr=1.0), InitConfig("zero"))
    keys = np.arange(1, 41, dtype=np.int64)
    t.push_keys(keys, np.ones((40, 2), np.float32))
    root = tmp_path
    for r in range(2):
        ck.save_sharded(t, str(root / "param-4"), r, 2, fmt="bin")
    old = time.time() - 100
    for f in root.glob("param-4.*.bin"):
        os.utime(f, (old, old))
    for r in range(2):
        ck.save_sharded(t, str(root / "param-4"), r, 2, fmt="text")
    found = ck.latest_checkpoint(str(root))
    assert found == (str(root / "param-4"), 4, 2, "text")
    t2 = HostTable(2, 2, Optimizer("sgd", lr=1.0), InitConfig("zero"))
    n = ck.load_sharded(t2, found[0], world=found[2], fmt=found[3])
    assert n == 2 * 40  # both shards hold the whole (unsharded) table
    np.testing.assert_allclose(t2.pull_keys(keys).numpy(), -np.ones((40, 2)))


def test_backups_fire_when_rounds_cross_a_period():
    """PSContext.maybe_backup with rounds that advance in jumps (hipGraph
    replays of 16 steps): a backup whenever a period boundary was crossed,
    labelled with the round reached, and none right after a resume."""
    from swiftsnails_amd.framework.gpu import PSContext

    class Stub:
        backup_period = 10
        _last_backup = -1
        watchdog = None
        backup_root = "/nonexistent"

        def __init__(self):
            self.saved = []

            class E:
                def check(self_):
                    pass
            self.engine = E()

        def save(self, prefix, fmt=None):
            self.saved.append(int(prefix.rsplit("-", 1)[1]))

    s = Stub()
    for r in (16, 32, 48, 64, 80, 96):
        PSContext.maybe_backup(s, r)
    assert s.saved == [16, 32, 48, 64, 80, 96]  # 10,20,30,... crossed each time
    s2 = Stub()
    s2._last_backup = 30  # resumed from param-30
    for r in (31, 35, 39, 41, 45):
        PSContext.maybe_backup(s2, r)
    assert s2.saved == [41]
