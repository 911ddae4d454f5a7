"""The RCCL communicator's alltoallv peer schedule (ss/a2a_schedule.h), run
for all N ranks of an exchange against each other on the CPU.

The reference's only distributed test is a self-loopback transfer
(/root/reference/src/unitest/core/transfer/transfer_test.h:13-80); here the
schedule every rank issues inside its ncclGroupStart/End is checked for
N = 2..8 with random counts and displacements: each message is sent exactly
once and received exactly once with the same size, in the same step on both
sides (rank r sends to r+k while r+k receives from r), and every byte range
lies inside its buffer without two receives overlapping.
"""
import numpy as np
import pytest

from swiftsnails_amd._native import host


def _exchange(rng, N, elem, cap):
    """Random alltoallv of N ranks: counts[s][d] elements from s to d, each
    rank's send/recv segments at shuffled, non-overlapping displacements."""
    counts = rng.integers(0, cap // N + 1, size=(N, N))
    counts[rng.random((N, N)) < 0.2] = 0  # some empty pairs
    plans = []
    for r in range(N):
        sc, rc = counts[r], counts[:, r]
        so, ro = rng.permutation(N), rng.permutation(N)
        sd, rd = np.zeros(N, np.int64), np.zeros(N, np.int64)
        o = 0
        for p in so:
            sd[p] = o
            o += sc[p]
        o = 0
        for p in ro:
            rd[p] = o
            o += rc[p]
        plans.append((sc.tolist(), sd.tolist(), rc.tolist(), rd.tolist()))
    return counts, plans


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("elem", [1, 8, 36])
def test_schedule_pairs_every_message(N, elem):
    h = host()
    rng = np.random.default_rng(100 * N + elem)
    for trial in range(20):
        cap = 64 * N
        counts, plans = _exchange(rng, N, elem, cap)
        sched = []
        for r, (sc, sd, rc, rd) in enumerate(plans):
            steps = h.a2a_schedule(r, N, sc, sd, rc, rd, elem, cap, cap)
            assert [s[0] for s in steps] == list(range(N))
            sched.append(steps)
        sends, recvs = {}, {}
        for r in range(N):
            recv_ranges = []
            for k, to, so, sb, frm, ro, rb in sched[r]:
                if to >= 0:
                    assert (r, to) not in sends
                    sends[(r, to)] = (k, sb)
                    assert 0 <= so and so + sb <= cap * elem
                    assert sb == counts[r][to] * elem > 0
                if frm >= 0:
                    assert (frm, r) not in recvs
                    recvs[(frm, r)] = (k, rb)
                    assert 0 <= ro and ro + rb <= cap * elem
                    assert rb == counts[frm][r] * elem > 0
                    recv_ranges.append((ro, ro + rb))
            recv_ranges.sort()
            for (a0, a1), (b0, b1) in zip(recv_ranges, recv_ranges[1:]):
                assert a1 <= b0, "two receives overlap"
        # every nonzero message is sent once and received once, same size
        nz = {(s, d) for s in range(N) for d in range(N) if counts[s][d] > 0}
        assert set(sends) == nz == set(recvs)
        for key in nz:
            ks, bs = sends[key]
            kr, br = recvs[key]
            assert bs == br
            s, d = key
            # step pairing: s sends to d in step (d - s) mod N, d receives from
            # s in the same step (self: step 0 on both sides)
            assert ks == kr == (d - s) % N


def test_schedule_rejects_malformed_exchanges():
    h = host()
    ok = ([1, 2], [0, 1], [1, 3], [0, 1])
    h.a2a_schedule(0, 2, *ok, 4, 3, 4)
    with pytest.raises(ValueError, match="nranks entries"):
        h.a2a_schedule(0, 2, [1], [0], [1], [0], 4)
    with pytest.raises(ValueError, match="negative"):
        h.a2a_schedule(0, 2, [1, -1], [0, 1], [1, 3], [0, 1], 4)
    with pytest.raises(ValueError, match="send buffer"):
        h.a2a_schedule(0, 2, *ok, 4, 2, 4)     # 1 + 2 elements past a 2-element buffer
    with pytest.raises(ValueError, match="receive buffer"):
        h.a2a_schedule(0, 2, *ok, 4, 3, 3)
    with pytest.raises(ValueError, match="self"):
        h.a2a_schedule(0, 2, [2, 2], [0, 2], [1, 3], [0, 1], 4)
    with pytest.raises(ValueError, match="rank"):
        h.a2a_schedule(2, 2, *ok, 4)


def test_xgmi_arenas_stay_below_the_ipc_limit():
    """Importing an uncached allocation of 2 GB or more through
    hipIpcOpenMemHandle never returned on the MI355X boxes, so the mailbox
    transport gives every (channel, ring slot) its own allocation and
    refuses one of 2 GiB or more before allocating anything.  The bench's
    largest mailbox, one round of keys from 8 sources of a 262144 x 39
    batch, is 0.65 GB."""
    import torch

    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    t = XgmiTransport(0, 8, torch.device("cuda", 0), None)
    with pytest.raises(RuntimeError, match="2 GiB"):
        t.setup({"keys": (4, [10_223_616 * 8 * 4])})
    assert 8 * 10_223_616 * 8 < (2 << 30)


def test_auto_plane_falls_back_when_the_mailbox_layout_is_refused(monkeypatch):
    """transport=auto: a mailbox set-up failure (here the 2 GiB IPC limit)
    closes the xGMI transport and builds the engine on the fallback plane,
    and the PlaneInfo says so (bench.py / the launcher report it)."""
    from swiftsnails_amd.parallel import select
    from swiftsnails_amd.parallel.transport import LoopbackTransport
    from swiftsnails_amd.parallel.xgmi import XgmiTransport

    monkeypatch.setenv("SS_ENGINE_GENERAL", "xgmi")
    monkeypatch.setattr(select, "_rccl_fallback", lambda *a: LoopbackTransport())
    built = []

    def make_engine(tr, ct, pt):
        built.append(tr)
        if isinstance(tr, XgmiTransport):
            tr.setup({"keys": (4, [10_223_616 * 8 * 4 * 8])})
        return "engine"

    eng, (tr, ct, pt), info = select.build_engine("auto", 0, 1, "cpu", None, make_engine)
    assert eng == "engine" and isinstance(tr, LoopbackTransport)
    assert isinstance(built[0], XgmiTransport) and built[0].arenas == {}
    assert info.fell_back and "2 GiB" in info.fallback_reason and info.plane == "loopback"
    with pytest.raises(RuntimeError, match="2 GiB"):  # transport=xgmi: no fallback
        select.build_engine("xgmi", 0, 1, "cpu", None, make_engine)
