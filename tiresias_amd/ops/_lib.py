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
        if torch.cuda.is_available():
            load_routes()
        return True


# Per-device GEMM routing table (measured (path, tile, split-K) per GEMM
# shape, ``torch.ops.tam.gemm_routes()`` format) shipped with the framework:
# a cold process starts with the decisions instead of timing every new shape
# on its first jobs' first steps. TAM_GEMM_ROUTES=<file> overrides, "0"
# disables. Keyed by device so a table is only used on the hardware it was
# measured on.
ROUTES_DIR = Path(__file__).resolve().parent.parent.parent / "profiles"


def device_key(index: int = 0) -> str:
    p = torch.cuda.get_device_properties(index)
    arch = getattr(p, "gcnArchName", "unknown").split(":")[0]
    return f"{arch}_{p.multi_processor_count}cu"


def routes_file(index: int = 0) -> Path:
    env = os.environ.get("TAM_GEMM_ROUTES")
    if env and env != "0":
        return Path(env)
    return ROUTES_DIR / f"gemm_routes_{device_key(index)}.txt"


def load_routes(index: int = 0) -> int:
    """Pre-load the routing table for this device (if one exists); returns
    the number of shapes loaded."""
    if os.environ.get("TAM_GEMM_ROUTES") == "0":
        return 0
    try:
        f = routes_file(index)
    except Exception:
        return 0
    if not f.exists():
        return 0
    return int(torch.ops.tam.gemm_routes_load(f.read_text()))


def save_routes(path: str | None = None, index: int = 0) -> str:
    """Write this process's routing decisions (merged with the file's)."""
    f = Path(path) if path else routes_file(index)
    cur = torch.ops.tam.gemm_routes()
    lines = {}
    if f.exists():
        for ln in f.read_text().splitlines():
            if ln.strip():
                lines[" ".join(ln.split()[:7])] = ln
    for ln in cur.splitlines():
        if ln.strip():
            lines[" ".join(ln.split()[:7])] = ln
    f.parent.mkdir(parents=True, exist_ok=True)
    f.write_text("".join(v + "\n" for _, v in sorted(lines.items())))
    return str(f)


def ops():
    """``torch.ops.tam`` (or, in kernel debug mode -- ``utils/debug.py``,
    ``TAM_DEBUG=1`` -- a proxy that synchronises and checks after every op)."""
    load(required=True)
    from ..utils import debug

    return debug.wrap(torch.ops.tam)


def is_loaded() -> bool:
    return _loaded
