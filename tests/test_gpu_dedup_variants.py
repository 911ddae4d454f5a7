"""The bucketed dedup under its scatter / key-width knobs.

The knobs are read once per process (static in bdedup.hip), so each variant
runs in a child process: the unsorted scatter (SS_BD_SORT=0), 8-byte keys
for calls whose keys fit 32 bits (SS_BD_REC=8), and both.  Every variant must
route each occurrence to its unique key (ukeys[inv] == keys), count the
distinct keys exactly, and give the LR gradient merge the per-key sums of a
numpy reference — the scatter writes the bucket-ordered keys and the
occurrence list pj as two arrays, and the dedup and merge read them."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_BODY = r'''
import numpy as np, torch
from swiftsnails_amd._native import hip
from swiftsnails_amd.ops.dedup import Deduper
from swiftsnails_amd.parallel.router import HashFrag
dev = torch.device("cuda", 0)
rng = np.random.default_rng(11)
for nranks in (1, 3):
    fm = torch.from_numpy(HashFrag(nranks, 64).rank_map().astype(np.int32))
    d = Deduper(300_000, nranks=nranks, frag_map=fm, gdim=1, device=dev, mode="bucket")
    cases = [np.array([42]), rng.integers(0, 50, 65), rng.integers(0, 10**9, 4097),
             np.concatenate([np.full(150_000, 123456789), rng.integers(0, 999, 3000)]),
             rng.integers(0, 1 << 40, 20000),
             (rng.zipf(1.3, 260_000) % 300_000)]
    for k in cases:
        k = k.astype(np.int64)
        r = d(torch.from_numpy(k).to(dev))
        torch.cuda.synchronize()
        inv = r.inv.cpu().numpy().view(np.uint32).astype(np.int64)
        np.testing.assert_array_equal(r.ukeys.cpu().numpy()[inv], k)
        assert int(r.ucount.sum().item()) == len(np.unique(k))
    d.check()
    # the LR merge over the last call's partition: per-key sums of gs[j // F]
    F = 13
    n = (len(k) // F) * F
    k = k[:n]
    r = d(torch.from_numpy(k).to(dev))
    gs = torch.from_numpy(rng.standard_normal(n // F).astype(np.float32)).to(dev)
    ug = torch.zeros(nranks * d.ucap, dtype=torch.float32, device=dev)
    d.reduce(n, gs, F, ug)
    torch.cuda.synchronize()
    inv = r.inv.cpu().numpy().view(np.uint32).astype(np.int64)
    ref = np.zeros(nranks * d.ucap, np.float64)
    np.add.at(ref, inv, np.repeat(gs.cpu().numpy().astype(np.float64), F))
    got = ug.cpu().numpy()
    np.testing.assert_allclose(got[inv], ref[inv], rtol=1e-4, atol=1e-4)
print("ok")
'''


@pytest.mark.parametrize("env", [{"SS_BD_SORT": "0"}, {"SS_BD_REC": "8"},
                                 {"SS_BD_SORT": "0", "SS_BD_REC": "8"}],
                         ids=["unsorted", "key8", "unsorted-key8"])
def test_bucket_dedup_scatter_variants(env):
    e = dict(os.environ, PYTHONPATH=ROOT, **env)
    p = subprocess.run([sys.executable, "-c", _BODY], env=e, cwd=ROOT, capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout[-2000:] + p.stderr[-4000:]
