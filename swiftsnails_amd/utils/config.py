"""Python facade over the C++ ``ConfigParser`` (``key: value`` files).

Same syntax/semantics as the reference (/root/reference/src/utils/ConfigParser.h):
first definition wins, ``import <path>``, ``#`` comments, missing keys are an
error.  ``overrides`` (e.g. from the command line) take precedence.

Keys understood by the framework (reference names kept):
``listen_addr, async_exec_num, listen_thread_num, master_addr, init_timeout,
expected_node_num, master_time_out, frag_num, shard_num, param_backup_period,
param_backup_root, num_iters, learning_rate, async_channel_thread_num,
local_train`` plus the MI355X additions ``optimizer, l1, l2, param_init,
param_init_scale, param_output, server_ranks, worker_ranks, table_capacity,
batch_size``, data input ``data_path, data_format, data_threads, min_count,
sample`` and failure detection ``round_timeout, peer_timeout,
heartbeat_interval, watchdog_exit`` (parallel/watchdog.py).
"""
from __future__ import annotations

from typing import Mapping, Optional

from .._native import host


class Config:
    def __init__(self, parser=None):
        self._p = parser if parser is not None else host().ConfigParser()

    @classmethod
    def from_file(cls, path: str, overrides: Optional[Mapping[str, object]] = None) -> "Config":
        c = cls()
        for k, v in (overrides or {}).items():
            c._p.set(str(k), str(v))  # inserted first => they win
        c._p.parse_file(path)
        return c

    @classmethod
    def from_string(cls, text: str, base_dir: str = ".",
                    overrides: Optional[Mapping[str, object]] = None) -> "Config":
        c = cls()
        for k, v in (overrides or {}).items():
            c._p.set(str(k), str(v))
        c._p.parse_string(text, base_dir)
        return c

    @classmethod
    def from_dict(cls, d: Mapping[str, object]) -> "Config":
        c = cls()
        for k, v in d.items():
            c._p.set(str(k), str(v).lower() if isinstance(v, bool) else str(v))
        return c

    @property
    def native(self):
        return self._p

    def __getitem__(self, key: str) -> str:
        return self._p.get_config(key)

    def __contains__(self, key: str) -> bool:
        return self._p.has(key)

    def get(self, key: str, default=None):
        return self._p.get(key, "") if self._p.has(key) else default

    def get_int(self, key: str, default: Optional[int] = None) -> int:
        if default is not None and not self._p.has(key):
            return default
        return self._p.get_int64(key)

    def get_float(self, key: str, default: Optional[float] = None) -> float:
        if default is not None and not self._p.has(key):
            return default
        return self._p.get_float(key)

    def get_bool(self, key: str, default: Optional[bool] = None) -> bool:
        if default is not None and not self._p.has(key):
            return default
        return self._p.get_bool(key)

    def set(self, key: str, value) -> None:
        self._p.set(key, str(value).lower() if isinstance(value, bool) else str(value))

    def register(self, key: str, value="") -> bool:
        return self._p.register_config(key, str(value))

    def items(self):
        return self._p.items()

    def as_dict(self) -> dict:
        return dict(self._p.items())

    def __repr__(self):
        return f"Config({self.as_dict()})"


_GLOBAL: Optional[Config] = None


def global_config() -> Config:
    """Process-wide config (reference ``global_config()``, ConfigParser.h:126-129)."""
    global _GLOBAL
    if _GLOBAL is None:
        _GLOBAL = Config(host().global_config())
    return _GLOBAL
