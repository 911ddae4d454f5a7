"""Dedup microbenchmark: time Deduper (bucket vs hash) on CTR-shaped and uniform keys.

python tools/mb_dedup.py [--batch 65536] [--fields 39]
Prints per-call device time and the bucket-size distribution (bucket mode)."""
import argparse
import sys
import os

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
    a = ap.parse_args()
    from swiftsnails_amd._native import hip
    from swiftsnails_amd.models.sparse_lr import CtrSynth
    from swiftsnails_amd.ops.dedup import Deduper

    dev = torch.device("cuda", 0)
    n = a.batch * a.fields
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    labels = torch.empty(a.batch, device=dev)
    CtrSynth(batch_size=a.batch, num_fields=a.fields).generate(0, 0, 1, keys, labels)
    uni = torch.randint(0, 1 << 40, (n,), device=dev)
    h = hip()
    for name, k in (("ctr", keys), ("uniform", uni)):
        for mode in ("bucket", "hash"):
            d = Deduper(n, device=dev, mode=mode, zero_grad=False)
            us = time_calls(lambda: d(k))
            torch.cuda.synchronize()
            line = f"{name:8s} {mode:6s} n={n} unique={int(d.ucount.sum())} {us:8.1f} us/call"
            if mode == "bucket":
                P = h.bd_buckets(n, 1)
                # bstart follows hist [nch*P] and btot [P] in the scratch (see bdedup.hip)
                sizes = None
                try:
                    _, o_bs, _, _ = h.bd_offsets(n, 1)
                    bs = d.scratch[o_bs:o_bs + P + 1].cpu().numpy().astype(np.int64)
                    sizes = np.diff(bs)
                except Exception as ex:  # layout drift: skip the stats
                    line += f" (no stats: {ex})"
                if sizes is not None:
                    line += (f" P={P} occ/bucket mean={sizes.mean():.0f} max={sizes.max()}"
                             f" p99={np.percentile(sizes, 99):.0f} >4096: {(sizes > 4096).sum()}")
            print(line, flush=True)
            if mode == "bucket" and d.dbg is not None:
                d(k)
                torch.cuda.synchronize()
                ts = d.dbg.view(-1, 8)[:, :4].cpu().numpy().astype(np.float64) * 0.01  # 100 MHz
                t0 = ts[:, 0].min()
                ph = np.diff(ts, axis=1)
                print("   phases us (mean/p50/max): " + "  ".join(
                    f"{nm}={ph[:, i].mean():.1f}/{np.median(ph[:, i]):.1f}/{ph[:, i].max():.1f}"
                    for i, nm in enumerate(["insert", "compact", "write"])))
                st = ts[:, 0] - t0
                en = ts[:, 3] - t0
                print(f"   block start spread: {st.min():.1f}..{st.max():.1f} us, "
                      f"end max {en.max():.1f} us, mean lifetime {(en - st).mean():.1f} us")


if __name__ == "__main__":
    main()
