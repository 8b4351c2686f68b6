"""Small utilities (reference ``core/util.py``): logging with levels (an
ERROR no longer calls ``exit()``: it raises), byte-unit conversion, directory
helpers and dict-list search."""
from __future__ import annotations

import logging
import os
from typing import Any, Iterable, List, Optional

LOG_LEVEL_DEBUG, LOG_LEVEL_INFO, LOG_LEVEL_WARNING, LOG_LEVEL_ERROR = 0, 1, 2, 3
_log = logging.getLogger("tiresias_amd")


class SchedulerError(RuntimeError):
    pass


def print_fn(msg: str, level: int = LOG_LEVEL_INFO) -> None:
    if level == LOG_LEVEL_DEBUG:
        _log.debug(msg)
    elif level == LOG_LEVEL_INFO:
        _log.info(msg)
    elif level == LOG_LEVEL_WARNING:
        _log.warning(msg)
    else:
        _log.error(msg)
        raise SchedulerError(msg)


_UNITS = {"B": 1, "KiB": 2 ** 10, "MiB": 2 ** 20, "GiB": 2 ** 30, "TiB": 2 ** 40,
          "KB": 1e3, "MB": 1e6, "GB": 1e9, "TB": 1e12}


def convert_bytes(n: float, unit: str = "MiB") -> float:
    if unit not in _UNITS:
        raise ValueError(f"unknown unit {unit}")
    return float(n) / _UNITS[unit]


def make_dir_if_not_exist(path: str) -> str:
    os.makedirs(path, exist_ok=True)
    return path


def search_dict_list(dlist: Iterable[dict], key: str, value: Any) -> Optional[dict]:
    for d in dlist:
        if d.get(key) == value:
            return d
    return None
