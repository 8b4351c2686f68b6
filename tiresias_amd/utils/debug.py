"""Kernel debug mode: run every HIP op synchronously and check
what it wrote.

``enable()`` (or ``TAM_DEBUG=1`` in the environment, or ``--debug_kernels``
on the CLIs) must run before the first HIP call of the process:

* sets ``HIP_LAUNCH_BLOCKING=1`` (every launch returns only after the kernel
  finished, so an invalid access faults at the op that caused it) and
  ``AMD_LOG_LEVEL`` (runtime error messages; level 2 unless already set);
* makes ``ops._lib.ops()`` return a proxy of ``torch.ops.tam`` that, after
  every op, synchronises the device (an asynchronous HIP error is raised
  with the op's name) and -- level >= 2 -- checks every floating-point
  tensor argument the op may have written for NaN / Inf, naming the op and
  the argument position.

It is a debugging aid: a step runs many times slower. Graph capture cannot be
combined with it (synchronising inside a capture is illegal), so trainers
built while it is on run eagerly.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

_LEVEL = 0


class KernelDebugError(RuntimeError):
    pass


def level() -> int:
    return _LEVEL


def enable(lvl: int = 2) -> None:
    """Turn the debug mode on (call before any GPU work)."""
    global _LEVEL
    _LEVEL = int(lvl)
    if _LEVEL > 0:
        os.environ["HIP_LAUNCH_BLOCKING"] = "1"
        os.environ.setdefault("AMD_LOG_LEVEL", "2")


def from_env() -> None:
    v = os.environ.get("TAM_DEBUG", "")
    if v and v != "0":
        enable(int(v) if v.isdigit() else 2)


class _CheckedOp:
    def __init__(self, name: str, op):
        self.name, self.op = name, op

    def __call__(self, *args, **kwargs):
        try:
            out = self.op(*args, **kwargs)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except RuntimeError as e:
            raise KernelDebugError(f"tam.{self.name}: {e}") from e
        if _LEVEL >= 2:
            for i, a in enumerate(list(args) + list(kwargs.values())):
                tensors = a if isinstance(a, (list, tuple)) else [a]
                for t in tensors:
                    if isinstance(t, torch.Tensor) and t.is_floating_point() and t.numel() and \
                            not bool(torch.isfinite(t).all()):
                        raise KernelDebugError(f"tam.{self.name}: non-finite values in argument {i} "
                                               f"(shape {tuple(t.shape)}, {t.dtype})")
        return out


class OpsProxy:
    """``torch.ops.tam`` with every op wrapped by ``_CheckedOp``."""

    def __init__(self, ns):
        self._ns = ns

    def __getattr__(self, name: str):
        return _CheckedOp(name, getattr(self._ns, name))


def wrap(ns) -> Optional[object]:
    return OpsProxy(ns) if _LEVEL > 0 else ns


from_env()
