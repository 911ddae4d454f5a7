"""Structured per-rank logging (the reference uses glog LOG/CHECK everywhere,
/root/reference/src/utils/common.h:31).  Level from SS_LOG_LEVEL
(DEBUG/INFO/WARNING/ERROR or 0-3, shared with the C++ runtime)."""
from __future__ import annotations

import logging
import os
import sys

_LEVELS = {"0": logging.DEBUG, "1": logging.INFO, "2": logging.WARNING, "3": logging.ERROR}


def _level() -> int:
    v = os.environ.get("SS_LOG_LEVEL", "2").upper()
    return _LEVELS.get(v, getattr(logging, v, logging.WARNING))


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = os.environ.get("RANK", "0")
        return True


def get_logger(name: str = "swiftsnails") -> logging.Logger:
    lg = logging.getLogger(name)
    if not lg.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(levelname).1s %(asctime)s r%(rank)s %(name)s] "
                                         "%(message)s"))
        h.addFilter(_RankFilter())
        lg.addHandler(h)
        lg.setLevel(_level())
        lg.propagate = False
    return lg
