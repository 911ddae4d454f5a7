"""Master / server / worker roles (the reference's public framework API).

Reference: ``SwiftMaster`` (/root/reference/src/core/framework/SwiftMaster.h:8-29),
``SwiftServer<Key,Val,Grad,PullMethod,PushMethod>`` (SwiftServer.h:17-53),
``SwiftWorker<Algorithm>`` + ``BaseAlgorithm`` (SwiftWorker.h:19-153).

Two deployments share this API:

* **host cluster** (any machine, what the reference is): one process per role,
  talking over the C++ TCP RPC layer (``csrc/host/transfer.h``); servers hold
  CPU ``HostTable`` shards.  ``SwiftMaster``/``SwiftServer``/``SwiftWorker``
  below drive the C++ ``Master``/``Server``/``WorkerClient``.
* **MI355X collective mode** (``swiftsnails_amd.framework.gpu``): one process
  per GPU under torchrun, HBM table shards, RCCL alltoallv rounds.

``local_train > 0`` runs ``train()`` against an in-process table with no
networking, as in the reference (SwiftWorker.h:114-123).
"""
from __future__ import annotations

import abc
from typing import Optional

import numpy as np

from .._native import host
from ..ops.host_table import HostTable
from ..ops.optim import InitConfig, Optimizer
from ..utils.config import Config


def _cfg(config) -> Config:
    if isinstance(config, Config):
        return config
    if isinstance(config, dict):
        return Config.from_dict(config)
    return Config.from_file(str(config))


def optimizer_from_config(cfg: Config) -> Optimizer:
    return Optimizer(cfg.get("optimizer", "sgd"), lr=float(cfg.get("learning_rate", 0.01)),
                     l1=float(cfg.get("l1", 0.0)), l2=float(cfg.get("l2", 0.0)),
                     eps=float(cfg.get("adagrad_eps", 1e-8)),
                     ftrl_alpha=float(cfg.get("ftrl_alpha", 0.05)),
                     ftrl_beta=float(cfg.get("ftrl_beta", 1.0)))


def init_from_config(cfg: Config) -> InitConfig:
    return InitConfig(cfg.get("param_init", "zero"), float(cfg.get("param_init_scale", 0.0)),
                      float(cfg.get("optimizer_state_init", 0.0)),
                      int(cfg.get("param_init_seed", 2015)))


class SwiftMaster:
    """Registration, routing, hash fragments and termination (rank-0 role)."""

    def __init__(self, config):
        self.cfg = _cfg(config)
        self._m = host().Master(self.cfg.native)

    @property
    def addr(self) -> str:
        return self._m.addr

    def init(self):
        self._m.init()

    def terminate(self):
        self._m.terminate()

    def __call__(self):
        self._m.init()
        self._m.terminate()

    run = __call__


class SwiftServer:
    """A parameter-server shard: pull = lookup-or-init, push = optimizer apply."""

    def __init__(self, config, dim: int = 1, push_method=None):
        """``push_method``: a user-defined update rule ``fn(rows [n, width],
        grads [n, dim]) -> new rows`` (torch tensors) instead of the
        configured optimizer (the reference's PushAccessMethod)."""
        self.cfg = _cfg(config)
        self._s = host().Server(self.cfg.native, int(dim))
        if push_method is not None:
            from ..ops.host_table import set_table_push_method

            set_table_push_method(self._s.table(), push_method)

    def __call__(self, timeout: float = 1e9):
        self._s.connect()
        self._s.wait_terminate(timeout)

    run = __call__

    def connect(self):
        self._s.connect()

    def wait_terminate(self, timeout: float = 1e9):
        self._s.wait_terminate(timeout)

    @property
    def table(self):
        return self._s.table()

    @property
    def push_count(self) -> int:
        return self._s.push_count

    @property
    def client_id(self) -> int:
        return self._s.client_id


class BaseAlgorithm(abc.ABC):
    """User algorithm run by a worker (reference BaseAlgorithm, SwiftWorker.h:19-57).

    ``train()`` uses ``self.pull(keys)`` / ``self.push(keys, grads)``;
    ``parse_record(line)`` turns one input line into a record.
    """

    def __init__(self):
        self._client = None
        self._data_path: Optional[str] = None
        self.cfg: Optional[Config] = None

    @abc.abstractmethod
    def train(self):
        ...

    def parse_record(self, line: str):
        raise NotImplementedError

    def set_data_path(self, path: str):
        self._data_path = path

    @property
    def data_path(self) -> str:
        if not self._data_path:
            raise RuntimeError("should set_data_path first")
        return self._data_path

    def records(self):
        with open(self.data_path) as f:
            for line in f:
                line = line.rstrip("\n")
                if line:
                    yield self.parse_record(line)

    # parameter access (global_pull_access / global_push_access)
    def pull(self, keys) -> np.ndarray:
        return self._client.pull(np.ascontiguousarray(keys, dtype=np.uint64))

    def push(self, keys, grads) -> None:
        self._client.push(np.ascontiguousarray(keys, dtype=np.uint64),
                          np.ascontiguousarray(grads, dtype=np.float32))


class _LocalClient:
    """local_train: an in-process table instead of remote servers."""

    def __init__(self, cfg: Config, dim: int):
        self.table = HostTable(dim, int(cfg.get("shard_num", 8)), optimizer_from_config(cfg),
                               init_from_config(cfg))

    def pull(self, keys):
        return self.table.pull_keys(keys.view(np.int64)).numpy()

    def push(self, keys, grads):
        self.table.push_keys(keys.view(np.int64), grads.reshape(len(keys), -1))


class SwiftWorker:
    """Runs an algorithm against the servers (or locally when local_train > 0)."""

    def __init__(self, config, algorithm: BaseAlgorithm, dim: int = 1):
        self.cfg = _cfg(config)
        self.alg = algorithm
        self.alg.cfg = self.cfg
        self.dim = dim
        self.num_iters = int(self.cfg.get("num_iters", 1))
        self.learning_rate = float(self.cfg.get("learning_rate", 0.01))
        if self.num_iters <= 0 or self.learning_rate <= 0:
            raise ValueError("num_iters and learning_rate must be > 0")
        self.local_train = int(str(self.cfg.get("local_train", 0)).replace("true", "1")
                               .replace("false", "0")) > 0
        self._w = None
        if not self.local_train:
            self._w = host().WorkerClient(self.cfg.native)

    def __call__(self):
        if self.local_train:
            self.alg._client = _LocalClient(self.cfg, self.dim)
            self.alg.train()
            return
        self._w.connect()
        self.alg._client = self._w
        try:
            self.alg.train()
        finally:
            self._w.finish()

    run = __call__

    @property
    def client_id(self) -> int:
        return self._w.client_id if self._w is not None else -1
