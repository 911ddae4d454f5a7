#!/usr/bin/env python3
"""File-fed sparse LR: HBM-resident shard vs host fill + per-step H2D copy.

Writes a libsvm file of synthetic CTR rows (the bench generator's keys: 39
fields, Zipf ids over a 1B-feature space), parses it with the native loader
and trains the bench's LR step from it, once with the shard resident in HBM
(`data_resident: hbm`, batch cut out by k_csr_batch) and once host-fed
(`data_resident: host`, pinned-ring prefetch + H2D copy per step).

    python tools/bench_file_data.py --rows 600000 --batch 262144 --steps 20
    python tools/bench_file_data.py --model word2vec --lines 400000 --vocab 1000000

Prints one JSON line per mode.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_libsvm(path: str, rows: int, fields: int, features: int, dev) -> float:
    from swiftsnails_amd.models.sparse_lr import CtrSynth

    t0 = time.perf_counter()
    d = CtrSynth(batch_size=65536, num_fields=fields, num_features=features)
    with open(path, "w") as f:
        done = 0
        step = 0
        while done < rows:
            keys = torch.empty(d.batch_size * fields, dtype=torch.int64, device=dev)
            labels = torch.empty(d.batch_size, dtype=torch.float32, device=dev)
            d.generate(step, 0, 1, keys, labels)
            k = keys.view(-1, fields).cpu().numpy()
            y = labels.cpu().numpy().astype(np.int64)
            m = min(d.batch_size, rows - done)
            cols = [y[:m].astype(str)] + [k[:m, j].astype(str) for j in range(fields)]
            lines = cols[0]
            for c in cols[1:]:
                lines = np.char.add(np.char.add(lines, " "), c)
            f.write("\n".join(lines.tolist()) + "\n")
            done += m
            step += 1
    return time.perf_counter() - t0


def run(path, resident, a, dev):
    from swiftsnails_amd.models.sparse_lr import SparseLRWorker, make_lr_table
    from swiftsnails_amd.ops.optim import Optimizer
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.utils.dataio import FileCtrSource

    t0 = time.perf_counter()
    src = FileCtrSource(path, "libsvm", batch_size=a.batch, num_fields=a.fields,
                        resident=resident, device=dev, nthreads=a.threads)
    load_s = time.perf_counter() - t0
    table = make_lr_table(a.features, 1, Optimizer("adagrad", lr=0.05), load=0.5, device=dev)
    eng = PSEngine(table, None, max_keys=a.batch * a.fields, dim=1, device=dev)
    w = SparseLRWorker(eng, src)
    for _ in range(a.warmup):
        w.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        w.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.check()
    out = {"mode": resident, "rows": src.rows, "batch": a.batch, "steps": a.steps,
           "load_s": round(load_s, 2), "ms_per_step": round(1000 * el / a.steps, 3),
           "samples_per_s": round(a.batch * a.steps / el, 1),
           "resident_bytes": src.device_bytes() if resident == "hbm" else 0,
           "loss": round(w.mean_loss(), 5)}
    src.close()
    return out


def run_w2v(path, resident, a, dev):
    from swiftsnails_amd.models.word2vec import Word2VecWorker, make_w2v_table_args
    from swiftsnails_amd.ops.table import HbmTable
    from swiftsnails_amd.parallel.engine import PSEngine
    from swiftsnails_amd.utils.dataio import FileCorpusSource

    t0 = time.perf_counter()
    src = FileCorpusSource(path, batch_size=a.w2v_batch, window=5, negatives=5,
                           resident=resident, device=dev, nthreads=a.threads)
    load_s = time.perf_counter() - t0
    opt, init = make_w2v_table_args(128)
    table = HbmTable(128, int(2 * src.vocab / 0.5) + 1024, optimizer=opt, init=init, device=dev)
    eng = PSEngine(table, None, max_keys=src.n_keys, dim=128, device=dev)
    w = Word2VecWorker(eng, src)
    for _ in range(a.warmup):
        w.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        w.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.check()
    pairs = a.w2v_batch * 10 * a.steps
    out = {"model": "word2vec", "mode": resident, "tokens": src.corpus.size,
           "vocab": src.vocab, "batch": a.w2v_batch, "steps": a.steps,
           "load_s": round(load_s, 2), "ms_per_step": round(1000 * el / a.steps, 3),
           "pairs_per_s": round(pairs / el, 1), "loss": round(w.mean_loss(), 5)}
    src.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=600_000)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--path", default="/tmp/ss_bench_file.svm")
    ap.add_argument("--model", default="sparse_lr", choices=["sparse_lr", "word2vec"])
    ap.add_argument("--lines", type=int, default=400_000, help="word2vec corpus sentences")
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--w2v-batch", type=int, default=16384)
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.model == "word2vec":
        import subprocess

        path = a.path + ".w2v.txt"
        t0 = time.perf_counter()
        subprocess.check_call([sys.executable, os.path.join(os.path.dirname(
            os.path.abspath(__file__)), "gen_word2vec_data.py"), path, "--lines", str(a.lines),
            "--vocab", str(a.vocab), "--zipf", "1.1", "--min-len", "8", "--max-len", "40"])
        print(json.dumps({"file": path, "bytes": os.path.getsize(path),
                          "write_s": round(time.perf_counter() - t0, 1)}), flush=True)
        for mode in ("hbm", "host"):
            print(json.dumps(run_w2v(path, mode, a, dev)), flush=True)
        os.remove(path)
        return 0
    wr = write_libsvm(a.path, a.rows, a.fields, a.features, dev)
    print(json.dumps({"file": a.path, "bytes": os.path.getsize(a.path), "write_s": round(wr, 1)}),
          flush=True)
    for mode in ("hbm", "host"):
        print(json.dumps(run(a.path, mode, a, dev)), flush=True)
    os.remove(a.path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
