"""Host C++ runtime: hashing, router, config, codec, channels, CPU table.

Behavioral spec from the reference's gtest suite:
unitest/utils/{ConfigParser,Buffer,string,queue}_test.h,
unitest/core/{BasicChannel,AsynExec}_test.h,
unitest/core/parameter/{hashfrag,sparsetable}_test.h.
"""
import os
import struct

import numpy as np
import pytest

from swiftsnails_amd._native import host
from swiftsnails_amd.parallel.router import HashFrag
from swiftsnails_amd.utils.hashing import fmix64, fmix64_int

DATA = os.path.join(os.path.dirname(__file__), "data")


def test_fmix64_parity_scalar_numpy_cpp():
    # reference get_hash_code (utils/HashFunction.h:16-24), python-int oracle
    xs = [0, 1, 2, 12345, 2**32 + 7, 2**63 - 1, 2**64 - 2]
    h = host()
    for x in xs:
        ref = fmix64_int(x)
        assert h.fmix64(x) == ref
        assert int(fmix64(np.array([x], dtype=np.uint64))[0]) == ref
    arr = np.random.default_rng(0).integers(0, 2**63, 1000, dtype=np.int64).view(np.uint64)
    np.testing.assert_array_equal(h.fmix64_array(arr), fmix64(arr))


def test_fmix64_known_value():
    # fmix64(1) from MurmurHash3's published finalizer constants
    assert fmix64_int(0) == 0
    assert fmix64_int(1) == 0xB456BCFC34C2CB2C


def test_hashfrag_layout_matches_reference_rule():
    # hashfrag.h:30-46: frag i -> i // (frag_num // num_nodes) + 1, clamped
    hf = HashFrag(7, 100)
    each = 100 // 7
    exp = np.clip(np.arange(100) // each + 1, 1, 7)
    np.testing.assert_array_equal(hf.map_table, exp)
    c = host().HashFrag(7, 100)
    np.testing.assert_array_equal(np.array(c.map_table()), exp)
    keys = np.arange(5000, dtype=np.uint64) * np.uint64(2654435761)
    np.testing.assert_array_equal(hf.to_node_id(keys), c.to_node_ids(keys))
    # wire format {i32 num_nodes, i32 num_frags, u32 map[]} identical in both
    assert hf.serialize() == c.serialize()
    assert struct.unpack_from("<ii", hf.serialize()) == (7, 100)
    hf2 = HashFrag.deserialize(c.serialize())
    np.testing.assert_array_equal(hf2.map_table, hf.map_table)


def test_hashfrag_rejects_fewer_frags_than_nodes():
    with pytest.raises(ValueError):
        HashFrag(8, 4)
    with pytest.raises(RuntimeError):
        host().HashFrag(8, 4)


def test_hashfrag_rank_map_split_roles():
    hf = HashFrag(4, 64)
    rm = hf.rank_map([1, 3, 5, 7])  # servers on odd ranks
    assert set(np.unique(rm)) == {1, 3, 5, 7}
    assert (rm == np.array([1, 3, 5, 7])[hf.map_table.astype(int) - 1]).all()


def test_config_parser_reference_fixture():
    c = host().ConfigParser()
    c.load_conf(os.path.join(DATA, "1.conf"))
    c.parse()
    assert c.get_config("ip") == "tcp://127.0.0.1:8080"  # split on FIRST ':'
    assert c.get_int32("thread_num") == 12
    with pytest.raises(RuntimeError):
        c.get_config("missing")


def test_config_import_first_definition_wins():
    c = host().ConfigParser()
    c.parse_file(os.path.join(DATA, "child.conf"))
    assert c.get_int32("thread_num") == 4
    assert abs(c.get_float("learning_rate") - 0.05) < 1e-9
    assert c.get_bool("local_train") is True
    c.set("local_train", "yes")
    with pytest.raises(RuntimeError):
        c.get_bool("local_train")
    assert c.register_config("new_key", "1") and not c.register_config("thread_num", "7")
    assert c.get_int32("thread_num") == 4


def test_config_python_facade():
    from swiftsnails_amd.utils.config import Config

    cfg = Config.from_string("a: 1\n# c\nb: x:y\n")
    assert cfg["a"] == "1" and cfg.get_int("a") == 1 and cfg["b"] == "x:y"
    assert cfg.get("zzz", "d") == "d"
    cfg2 = Config.from_file(os.path.join(DATA, "child.conf"), overrides={"thread_num": "8"})
    assert cfg2.get_int("thread_num") == 8


def test_binary_buffer_roundtrip_and_growth():
    b = host().BinaryBuffer()
    for i in range(400):  # > 1024 bytes forces growth (Buffer_test.h:88-114)
        b.put_i32(i)
        b.put_f64(i * 0.5)
    b.put_str("hello")
    assert b.size() == 400 * 12 + 4 + 5
    for i in range(400):
        assert b.get_i32() == i
        assert b.get_f64() == i * 0.5
    assert b.get_str() == "hello"
    assert b.read_finished()
    with pytest.raises(RuntimeError):
        b.get_i32()


def test_string_utils():
    h = host()
    assert h.trim("  a b \t\n") == "a b"
    assert h.split("hello world@bb", " @") == ["hello", "world", "bb"]
    assert h.key_value_split("k: v: w", ":") == ("k", " v: w")


def test_channel_and_pool():
    h = host()
    P, N = 4, 2000
    assert h.channel_selftest(P, N) == sum(range(P * N))  # close drains, nothing lost
    pool = h.ThreadPool(4)
    hits = []
    pool.parallel_for(40, lambda i: hits.append(i))  # AsynExec_test: count == 40
    assert sorted(hits) == list(range(40))
    pool.stop()


@pytest.mark.parametrize("kind", ["sgd", "adagrad", "ftrl", "adam"])
def test_host_table_matches_reference(kind):
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer, apply_reference, init_reference

    opt = Optimizer(kind, lr=0.1, l1=0.01, l2=0.001, grad_scale=0.5)
    opt.step = 1
    init = InitConfig("uniform", 0.5, 0.05, seed=3)
    t = HostTable(6, shard_num=5, optimizer=opt, init=init)
    keys = np.unique(np.random.default_rng(1).integers(0, 1 << 40, 3000)).astype(np.int64)
    v = t.pull_keys(keys).numpy()
    ref0 = init_reference(init, keys, 6, t.width)
    np.testing.assert_array_equal(v, ref0[:, :6])
    assert t.size() == len(keys)
    g = np.random.default_rng(2).standard_normal((len(keys), 6)).astype(np.float32)
    t.push_keys(keys, g)
    d = t.to_dict(with_state=True)
    rows = np.stack([d[int(k)] for k in keys.view(np.uint64)])
    np.testing.assert_allclose(rows, apply_reference(opt, ref0, g, 6), rtol=1e-5, atol=1e-6)


def test_host_table_text_checkpoint_roundtrip(tmp_path):
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer

    t = HostTable(3, shard_num=4, optimizer=Optimizer("adagrad"), init=InitConfig("normal", 0.3))
    keys = np.arange(100, 400, dtype=np.int64)
    t.pull_keys(keys)
    t.push_keys(keys, np.ones((len(keys), 3), np.float32))
    p = str(tmp_path / "param.txt")
    t.write_text(p, with_state=True)
    lines = open(p).read().splitlines()
    assert len(lines) == 300
    k, rest = lines[0].split("\t")
    assert int(k) in set(range(100, 400)) and "|" in rest
    t2 = HostTable(3, shard_num=2, optimizer=Optimizer("adagrad"))
    assert t2.load_text(p) == 300
    a, b = t.to_dict(True), t2.to_dict(True)
    for kk in a:
        np.testing.assert_array_equal(a[kk], b[kk])
    # params-only (reference format) loads too, state from state_init
    p2 = str(tmp_path / "p2.txt")
    t.write_text(p2, precision=6)
    t3 = HostTable(3, optimizer=Optimizer("adagrad"))
    assert t3.load_text(p2) == 300
