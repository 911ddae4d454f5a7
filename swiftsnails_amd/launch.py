"""Command-line launcher (the reference's ``-config <file> [-data <file>]``
binaries and run_{master,server,worker}.sh scripts, /root/reference/src/tools/).

MI355X collective mode (default): one process per GPU under torchrun::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m swiftsnails_amd.launch --config configs/sparse_lr_1b.conf [--steps 100]

Host (CPU) cluster roles, one process each (reference deployment)::

    python -m swiftsnails_amd.launch --role master --config configs/dense_lr_cpu.conf
    python -m swiftsnails_amd.launch --role server --config configs/dense_lr_cpu.conf
    python -m swiftsnails_amd.launch --role worker --config configs/dense_lr_cpu.conf \\
        --app swiftsnails_amd.models.dense_lr:DenseLR [--data file]

``--set key=value`` overrides config entries (overrides win; otherwise the
reference's first-definition-wins rule applies).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys


def _load_app(spec: str):
    mod, _, cls = spec.partition(":")
    return getattr(importlib.import_module(mod), cls)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="swiftsnails_amd.launch")
    ap.add_argument("--config", "-config", required=True)
    ap.add_argument("--role", choices=["gpu", "master", "server", "worker"], default="gpu")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--app", default="swiftsnails_amd.models.dense_lr:DenseLR")
    ap.add_argument("--data", "-data", default=None)
    ap.add_argument("--dim", type=int, default=1)
    a = ap.parse_args(argv)

    from .utils.config import Config

    over = dict(kv.split("=", 1) for kv in a.set)
    cfg = Config.from_file(a.config, overrides=over)
    if a.role == "gpu":
        from .framework.gpu import run_training

        stats = run_training(cfg, steps=a.steps, warmup=a.warmup)
        import os

        if os.environ.get("RANK", "0") == "0":
            print(json.dumps(stats))
        return 0
    from .framework.cluster import SwiftMaster, SwiftServer, SwiftWorker

    if a.role == "master":
        SwiftMaster(cfg).run()
    elif a.role == "server":
        SwiftServer(cfg, dim=a.dim).run()
    else:
        cls = _load_app(a.app)
        if cls.__name__ == "DenseLR":
            from .models.dense_lr import DenseLRData

            alg = cls(DenseLRData(dim=int(cfg.get("dense_dim", 64))),
                      steps=int(cfg.get("num_iters", 50)))
        else:
            alg = cls()
        if a.data:
            alg.set_data_path(a.data)
        SwiftWorker(cfg, alg, dim=a.dim).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
