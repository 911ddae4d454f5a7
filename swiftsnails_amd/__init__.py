"""swiftsnails_amd — an MI355X-native parameter server with SwiftSnails' capabilities.

Public API (mirrors the reference umbrella header /root/reference/src/swiftsnails.h:8-17):

* roles        : ``SwiftMaster``, ``SwiftServer``, ``SwiftWorker``, ``BaseAlgorithm``
                 (host/TCP clusters) and ``PSContext``/``run_training`` (MI355X
                 collective mode, one process per GPU)
* parameters   : ``HbmTable`` (GPU shard), ``HostTable`` (CPU shard),
                 ``Optimizer`` / ``InitConfig`` (the Pull/PushAccessMethod menu)
* access       : ``GlobalParamCache``, ``global_pull_access().pull_with_barrier``,
                 ``global_push_access().push_with_barrier`` (the reference's calls,
                 over a GPU engine or a host client); ``PSEngine.pull`` / ``push`` /
                 ``pull_dense`` / ``push_keys`` (the round engine underneath);
                 ``HbmTable.set_push_method`` (user-defined update rules)
* routing      : ``HashFrag`` (key -> fragment -> server)
* config       : ``Config``, ``global_config`` (``key: value`` files)
* checkpoints  : ``swiftsnails_amd.utils.checkpoint``
* models       : sparse LR, word2vec (SGNS), FM, dense LR
"""
from __future__ import annotations

__version__ = "0.1.0"

from .utils.config import Config, global_config  # noqa: E402
from .parallel.router import HashFrag  # noqa: E402
from .ops.optim import InitConfig, Optimizer  # noqa: E402


def __getattr__(name):  # lazy: GPU modules import torch/HIP on first use
    lazy = {
        "HbmTable": ("ops.table", "HbmTable"),
        "HostTable": ("ops.host_table", "HostTable"),
        "PSEngine": ("parallel.engine", "PSEngine"),
        "RcclTransport": ("parallel.transport", "RcclTransport"),
        "TorchDistTransport": ("parallel.transport", "TorchDistTransport"),
        "LoopbackTransport": ("parallel.transport", "LoopbackTransport"),
        "SwiftMaster": ("framework.cluster", "SwiftMaster"),
        "SwiftServer": ("framework.cluster", "SwiftServer"),
        "SwiftWorker": ("framework.cluster", "SwiftWorker"),
        "BaseAlgorithm": ("framework.cluster", "BaseAlgorithm"),
        "PSContext": ("framework.gpu", "PSContext"),
        "run_training": ("framework.gpu", "run_training"),
        "SparseLRWorker": ("models.sparse_lr", "SparseLRWorker"),
        "Word2VecWorker": ("models.word2vec", "Word2VecWorker"),
        "FMWorker": ("models.fm", "FMWorker"),
        "DenseLR": ("models.dense_lr", "DenseLR"),
        "GlobalParamCache": ("access", "GlobalParamCache"),
        "global_pull_access": ("access", "global_pull_access"),
        "global_push_access": ("access", "global_push_access"),
        "set_global_target": ("access", "set_global_target"),
    }
    if name in lazy:
        import importlib

        mod, attr = lazy[name]
        return getattr(importlib.import_module(f".{mod}", __name__), attr)
    raise AttributeError(name)


__all__ = ["Config", "global_config", "HashFrag", "InitConfig", "Optimizer", "HbmTable",
           "HostTable", "PSEngine", "SwiftMaster", "SwiftServer", "SwiftWorker", "BaseAlgorithm",
           "PSContext", "run_training", "SparseLRWorker", "Word2VecWorker", "FMWorker", "DenseLR",
           "GlobalParamCache", "global_pull_access", "global_push_access", "set_global_target"]
