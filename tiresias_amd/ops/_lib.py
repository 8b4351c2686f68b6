"""Loader for the in-tree HIP kernel library (``tiresias_amd/_C.so``).

On a GPU box the library is REQUIRED: every GPU op goes through it and a
missing/broken build raises instead of silently falling back to PyTorch.
On CPU-only hosts the ops use their PyTorch reference implementations (used by
the CPU test-suite and the gloo-distributed rehearsals).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# TAM_LIB_PATH: an alternative build of the same library (A/B measurements)
_LIB = Path(os.environ.get("TAM_LIB_PATH") or Path(__file__).resolve().parent.parent / "_C.so")
_lock = threading.Lock()
_loaded = False


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB


def load(required: bool | None = None) -> bool:
    """Load the kernel library once. ``required`` defaults to "a GPU is present"."""
    global _loaded
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if required is None:
            required = torch.cuda.is_available()
        if not _LIB.exists():
            if os.environ.get("TAM_AUTOBUILD", "1") == "1" and required:
                from tiresias_amd import _build

                _build.build()
            if not _LIB.exists():
                if required:
                    raise NativeLibraryMissing(
                        f"{_LIB} not found: run `python -m tiresias_amd._build` (hipcc, gfx950)")
                return False
        torch.ops.load_library(str(_LIB))
        _loaded = True
        return True


def ops():
    """``torch.ops.tam`` (or, in kernel debug mode -- ``utils/debug.py``,
    ``TAM_DEBUG=1`` -- a proxy that synchronises and checks after every op)."""
    load(required=True)
    from ..utils import debug

    return debug.wrap(torch.ops.tam)


def is_loaded() -> bool:
    return _loaded
