"""gflags-style flag registry (CLI-compatible with the reference).

Same surface as ``/root/reference/core/flags.py:14-125``: module-level
``FLAGS`` with lazy parsing on first attribute read, ``DEFINE_string /
integer / float / boolean / list / version``, ``--noX`` negation for booleans,
unknown arguments ignored. Differences: values are typed and validated, the
registry can be re-parsed with an explicit argv (tests, sweeps), and
``FLAGS.as_dict()`` feeds the typed :class:`~tiresias_amd.config.SimConfig`.
"""
from __future__ import annotations

import argparse
import sys
from typing import Any, Dict, List, Optional

_TRUE = {"true", "t", "1", "yes", "y"}
_FALSE = {"false", "f", "0", "no", "n"}


def _parse_bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    raise argparse.ArgumentTypeError(f"invalid boolean value {v!r}")


class _FlagValues:
    def __init__(self):
        object.__setattr__(self, "_defs", {})
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_parsed", False)
        object.__setattr__(self, "_version", None)

    # -- definition -------------------------------------------------------
    def _define(self, name: str, default, help: str, kind: str):
        self._defs[name] = dict(default=default, help=help, kind=kind)
        if self._parsed:
            self._values.setdefault(name, default)

    # -- parsing ------------------------------------------------------------
    def _parser(self) -> argparse.ArgumentParser:
        p = argparse.ArgumentParser(add_help=False, allow_abbrev=False)
        for name, d in self._defs.items():
            k = d["kind"]
            if k == "bool":
                p.add_argument(f"--{name}", nargs="?", const=True, default=d["default"],
                               type=_parse_bool, help=d["help"])
                p.add_argument(f"--no{name}", dest=name, action="store_false")
            elif k == "int":
                p.add_argument(f"--{name}", type=int, default=d["default"], help=d["help"])
            elif k == "float":
                p.add_argument(f"--{name}", type=float, default=d["default"], help=d["help"])
            elif k == "list":
                p.add_argument(f"--{name}", type=lambda s: [x for x in s.split(",") if x],
                               default=d["default"], help=d["help"])
            else:
                p.add_argument(f"--{name}", type=str, default=d["default"], help=d["help"])
        if self._version is not None:
            p.add_argument("--version", action="version", version=self._version)
        return p

    def parse(self, argv: Optional[List[str]] = None) -> List[str]:
        argv = sys.argv[1:] if argv is None else list(argv)
        ns, unknown = self._parser().parse_known_args(argv)
        object.__setattr__(self, "_values", vars(ns))
        object.__setattr__(self, "_parsed", True)
        return unknown

    def reset(self):
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_parsed", False)

    # -- access -------------------------------------------------------------
    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(name)
        if not self._parsed:
            self.parse()
        if name in self._values:
            return self._values[name]
        raise AttributeError(f"flag --{name} is not defined")

    def __setattr__(self, name: str, value):
        if name not in self._defs:
            raise AttributeError(f"flag --{name} is not defined")
        if not self._parsed:
            self.parse([])
        self._values[name] = value

    def __contains__(self, name: str) -> bool:
        return name in self._defs

    def as_dict(self) -> Dict[str, Any]:
        if not self._parsed:
            self.parse()
        return dict(self._values)

    def help_text(self) -> str:
        return self._parser().format_help()


FLAGS = _FlagValues()


def DEFINE_string(name, default, help=""):
    FLAGS._define(name, default, help, "str")


def DEFINE_integer(name, default, help=""):
    FLAGS._define(name, default, help, "int")


def DEFINE_float(name, default, help=""):
    FLAGS._define(name, default, help, "float")


def DEFINE_boolean(name, default, help=""):
    FLAGS._define(name, default, help, "bool")


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help=""):
    FLAGS._define(name, default, help, "list")


def DEFINE_version(v: str):
    object.__setattr__(FLAGS, "_version", v)
