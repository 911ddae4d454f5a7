"""Property-based checks (hypothesis) of the host-side invariants the GPU path
builds on: the fmix64 router (bit-identical C++ / numpy / Python-int, the
reference's fragment rule, hashfrag.h:30-53), the BinaryBuffer codec
(Buffer.h:174-234), the config parser's first-definition-wins semantics
(ConfigParser.h:87-119), the text checkpoint row format (sparsetable.h:49-56)
and the round engine's pull / merge / push against a dict oracle.
All CPU; example counts are kept small so the suite stays fast.
"""
import numpy as np
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from swiftsnails_amd._native import host
from swiftsnails_amd.parallel.router import HashFrag
from swiftsnails_amd.utils.hashing import fmix64, fmix64_int

U64 = st.integers(min_value=0, max_value=2**64 - 1)
FAST = settings(max_examples=40, deadline=None,
                suppress_health_check=[HealthCheck.too_slow])


@FAST
@given(st.lists(U64, min_size=1, max_size=64))
def test_fmix64_three_implementations_agree(xs):
    h = host()
    arr = np.array(xs, dtype=np.uint64)
    ref = [fmix64_int(x) for x in xs]
    assert [int(v) for v in fmix64(arr)] == ref
    assert [int(v) for v in h.fmix64_array(arr)] == ref


@FAST
@given(st.integers(1, 16).flatmap(lambda n: st.tuples(st.just(n), st.integers(n, 4 * n + 300))),
       st.lists(U64, min_size=1, max_size=200))
def test_hashfrag_rule_routing_and_codec(nf, keys):
    n, f = nf
    hf = HashFrag(n, f)
    c = host().HashFrag(n, f)
    m = hf.map_table.astype(np.int64)
    # reference rule: contiguous, non-decreasing ranges of server ids 1..n
    each = f // n
    np.testing.assert_array_equal(m, np.clip(np.arange(f) // each + 1, 1, n))
    assert (np.diff(m) >= 0).all() and m[0] == 1 and m[-1] == n
    assert set(np.unique(m)) == set(range(1, n + 1))  # every server owns fragments
    np.testing.assert_array_equal(np.array(c.map_table()), m)
    ka = np.array(keys, dtype=np.uint64)
    ids = hf.to_node_id(ka)
    np.testing.assert_array_equal(ids, c.to_node_ids(ka))
    np.testing.assert_array_equal(ids, [m[fmix64_int(k) % f] for k in keys])
    assert HashFrag.deserialize(hf.serialize()).serialize() == c.serialize()


_ITEM = st.one_of(
    st.tuples(st.just("i32"), st.integers(-2**31, 2**31 - 1)),
    st.tuples(st.just("f64"), st.floats(allow_nan=False)),
    st.tuples(st.just("str"), st.text(max_size=40)),
)


@FAST
@given(st.lists(_ITEM, max_size=300))
def test_binary_buffer_roundtrip(items):
    b = host().BinaryBuffer()
    for kind, v in items:
        getattr(b, "put_" + kind)(v)
    for kind, v in items:
        assert getattr(b, "get_" + kind)() == v
    assert b.read_finished()


_KEY = st.from_regex(r"[a-z][a-z0-9_]{0,11}", fullmatch=True)
_VAL = st.from_regex(r"[A-Za-z0-9_./:]{1,16}", fullmatch=True)


@FAST
@given(st.lists(st.tuples(_KEY, _VAL), min_size=1, max_size=30), st.data())
def test_config_first_definition_wins(pairs, data):
    lines, expect = [], {}
    for k, v in pairs:
        if data.draw(st.booleans()):
            lines.append(f"# {k}: ignored")  # comments never define a key
        lines.append(f"{k}: {v}")
        expect.setdefault(k, v)
    text = "\n".join(lines) + "\n"
    c = host().ConfigParser()
    c.parse_string(text)
    for k, v in expect.items():
        assert c.get_config(k) == v
    from swiftsnails_amd.utils.config import Config

    cfg = Config.from_string(text)
    for k, v in expect.items():
        assert cfg[k] == v


@FAST
@given(st.integers(1, 6), st.lists(U64, min_size=1, max_size=50, unique=True), st.integers(0, 9))
def test_text_rows_roundtrip(dim, keys, seed):
    """key<TAB>values rows: format then parse is the identity at full precision."""
    h = host()
    rows = np.random.default_rng(seed).standard_normal((len(keys), dim)).astype(np.float32)
    ka = np.array(keys, dtype=np.uint64)
    text = h.format_rows(ka, rows, dim, dim, False, 9, 2)
    assert text.count(b"\n") == len(keys) and text.count(b"\t") == len(keys)
    k2, r2 = h.parse_rows(text, dim, dim, 0.0, 2)
    order = np.argsort(k2)  # the formatter may emit rows in any order
    np.testing.assert_array_equal(np.sort(ka), k2[order])
    np.testing.assert_array_equal(rows[np.argsort(ka)], np.asarray(r2).reshape(-1, dim)[order])


@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.lists(st.integers(0, 60), min_size=1, max_size=80), min_size=1, max_size=4),
       st.sampled_from(["sgd", "adagrad"]))
def test_engine_rounds_match_dict_oracle(batches, kind):
    """World-1 round engine (CPU) over arbitrary key multisets: every pull
    returns the oracle's rows, and duplicate keys' gradients are merged
    before one optimizer update per key and round."""
    from swiftsnails_amd.ops.host_table import HostTable
    from swiftsnails_amd.ops.optim import InitConfig, Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.parallel.transport import LoopbackTransport

    dim = 2
    mk = lambda: HostTable(dim, 3, Optimizer(kind, lr=0.1), InitConfig("uniform", 0.3, 0.01))  # noqa: E731
    table, oracle = mk(), mk()
    eng = PSEngine(table, LoopbackTransport(), max_keys=80, dim=dim, frag_num=16, device="cpu")
    for i, b in enumerate(batches):
        k = np.array(b, dtype=np.int64)
        g = np.stack([np.sin(k + i), np.cos(0.5 * k)], 1).astype(np.float32)
        r = eng.pull(torch.from_numpy(k))
        np.testing.assert_allclose(eng.gather(r).numpy(), oracle.pull_keys(k).numpy(), rtol=1e-6)
        eng.accumulate(r, torch.from_numpy(g))
        eng.push(r)
        u, inv = np.unique(k, return_inverse=True)
        m = np.zeros((len(u), dim), np.float32)
        np.add.at(m, inv, g)
        oracle.push_keys(u, m)
        oracle.next_round()
    a, b2 = table.to_dict(with_state=True), oracle.to_dict(with_state=True)
    assert a.keys() == b2.keys()
    for key in a:
        np.testing.assert_allclose(a[key], b2[key], rtol=1e-5, atol=1e-6)
