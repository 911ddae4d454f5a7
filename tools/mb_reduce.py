"""Bucket-reduce microbenchmark: time k_bd_reduce (LR) and k_bd_reduce_fm on
CTR-shaped (Zipf heads) and uniform keys, with the bucket-size distribution.

python tools/mb_reduce.py [--batch 65536] [--fields 39] [--dim 9]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def time_calls(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--dim", type=int, default=9)
    a = ap.parse_args()
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.sparse_lr import CtrSynth
    from swiftsnails_amd.ops.dedup import Deduper

    h = hip()
    dev = torch.device("cuda", 0)
    B, F, D = a.batch, a.fields, a.dim
    n = B * F
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    labels = torch.empty(B, device=dev)
    CtrSynth(batch_size=B, num_fields=F).generate(0, 0, 1, keys, labels)
    uni = torch.randint(0, 1 << 40, (n,), device=dev)
    gs = torch.randn(B, device=dev)
    gss = torch.randn(B * (D - 1), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for name, k in (("ctr", keys), ("uniform", uni)):
        d = Deduper(n, device=dev, mode="bucket", zero_grad=False, gdim=D)
        d(k)
        torch.cuda.synchronize()
        U = int(d.ucount.sum())
        uvals = torch.randn(n, D, device=dev)
        ug = torch.empty(n, D, device=dev)
        ug1 = torch.empty(n, device=dev)
        t_lr = time_calls(lambda: h.bd_reduce(n, 1, d.scratch.data_ptr(), d.pj.data_ptr(),
                                              d.luid.data_ptr(), gs.data_ptr(), 0, F,
                                              ug1.data_ptr(), st))
        t_fm = time_calls(lambda: h.bd_reduce_fm(n, 1, d.scratch.data_ptr(), d.pj.data_ptr(),
                                                 d.luid.data_ptr(), gs.data_ptr(), gss.data_ptr(),
                                                 F, D, uvals.data_ptr(), ug.data_ptr(), st))
        ovf = torch.zeros(h.bd_fm_ovf_words(n), dtype=torch.int32, device=dev)
        ug2 = torch.empty(n, D, device=dev)
        t_fms = time_calls(lambda: h.bd_reduce_fm(n, 1, d.scratch.data_ptr(), d.pj.data_ptr(),
                                                  d.luid.data_ptr(), gs.data_ptr(), gss.data_ptr(),
                                                  F, D, uvals.data_ptr(), ug2.data_ptr(), st,
                                                  ovf.data_ptr()))
        torch.cuda.synchronize()
        err = (ug2[:U] - ug[:U]).abs().max().item()  # compact rows [0, U) at world 1
        P, o_bs, o_un, _ = h.bd_offsets(n, 1)
        sc = d.scratch.cpu().numpy().view(np.uint32).astype(np.int64)
        occ = np.diff(sc[o_bs:o_bs + P + 1])
        un = sc[o_un:o_un + P]
        # largest single-key count per bucket (same-address LDS atomics)
        lu = d.luid[:n].cpu().numpy().view(np.uint32).astype(np.int64)
        top = 0
        for b in np.argsort(occ)[-8:]:
            seg = lu[sc[o_bs + b]:sc[o_bs + b + 1]]
            top = max(top, int(np.bincount(seg[seg < 4096]).max()) if len(seg) else 0)
        print(f"{name:8s} n={n} U={U} P={P} occ/bucket mean={occ.mean():.0f} p99={np.percentile(occ, 99):.0f} "
              f"max={occ.max()} uniq/bucket mean={un.mean():.0f} max={un.max()} hottest key in a "
              f"big bucket={top}  reduce_lr={t_lr:.1f} us reduce_fm<{D}>={t_fm:.1f} us "
              f"sorted={t_fms:.1f} us (overflow buckets {int(ovf[0])}, max |diff| {err:.2e})",
              flush=True)


if __name__ == "__main__":
    main()
