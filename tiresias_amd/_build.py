"""Native build for tiresias_amd: compiles the HIP kernel library, the torch
op bindings and the checkpoint engine for gfx950 with hipcc, and links them
into an in-tree shared object ``tiresias_amd/_C.so`` (travels with the repo
snapshot to the GPU box; no JIT cache, no hipify, no setup.py).

Usage: ``python -m tiresias_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
PKG = ROOT / "tiresias_amd"
LIB = PKG / "_C.so"
ARCH = os.environ.get("TAM_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build tiresias_amd)")


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    return tdir / "include", tdir / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _sources():
    kern = sorted((CSRC / "kernels").glob("*.hip"))
    host = sorted((CSRC / "bindings").glob("*.cpp")) + sorted((CSRC / "ckpt").glob("*.cpp"))
    return kern, host


def _headers():
    return sorted((CSRC / "include").rglob("*.h"))


def _deps(obj: Path):
    """Headers a TU included at its last compile (the -MMD file next to the
    object), or None when unknown."""
    d = obj.with_suffix(".d")
    if not d.exists():
        return None
    txt = d.read_text().replace("\\\n", " ")
    toks = txt.split(":", 1)[1].split() if ":" in txt else []
    return [Path(t) for t in toks if t.endswith(".h")]


def _needs(obj: Path, src: Path, hdr_mtime: float) -> bool:
    if not obj.exists():
        return True
    m = obj.stat().st_mtime
    if m < src.stat().st_mtime:
        return True
    deps = _deps(obj)
    if deps is None:
        return m < hdr_mtime
    return any((not h.exists()) or m < h.stat().st_mtime for h in deps)


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    tinc, tlib, abi = _torch_paths()
    OBJ.mkdir(parents=True, exist_ok=True)
    kern, host = _sources()
    hdr_mtime = max((h.stat().st_mtime for h in _headers()), default=0.0)
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC / 'include'}", f"--offload-arch={ARCH}",
              "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    torch_flags = [f"-I{tinc}", f"-I{tinc / 'torch' / 'csrc' / 'api' / 'include'}",
                   "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                   "-Wno-ignored-attributes", "-fms-extensions"]
    cmds = []
    objs = []
    for src in kern + host:
        obj = OBJ / (src.parent.name + "_" + src.stem + ".o")
        objs.append(obj)
        if force or _needs(obj, src, hdr_mtime):
            extra = torch_flags if src.suffix == ".cpp" else []
            lang = ["-x", "hip"] if src.suffix == ".cpp" else []
            cmds.append([hipcc, *common, *extra, *lang, "-MMD", "-MF", str(obj.with_suffix(".d")), "-c",
                         str(src), "-o", str(obj)])
    jobs = jobs or min(8, os.cpu_count() or 4)
    if cmds:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(subprocess.run, c, capture_output=True, text=True): c for c in cmds}
            failed = []
            for f in cf.as_completed(futs):
                r = f.result()
                c = futs[f]
                if verbose:
                    print("[tam-build]", " ".join(c[-3:]), file=sys.stderr)
                if r.returncode != 0:
                    failed.append((c, r.stderr))
            if failed:
                for c, err in failed:
                    print("FAILED:", " ".join(c), "\n", err[-6000:], file=sys.stderr)
                raise RuntimeError(f"tiresias_amd native build failed ({len(failed)} TU(s))")
    newest = max(o.stat().st_mtime for o in objs)
    if force or not LIB.exists() or LIB.stat().st_mtime < newest:
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o",
                str(LIB) + ".tmp", f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
                f"-Wl,-rpath,{tlib}"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            print(r.stderr[-6000:], file=sys.stderr)
            raise RuntimeError("tiresias_amd link failed")
        os.replace(str(LIB) + ".tmp", LIB)
    return LIB


def build_sched_core(force: bool = False) -> Path:
    """Native event-engine core (pure C++17 + pybind11, no GPU code)."""
    import pybind11

    src = CSRC / "sched_core" / "sched_core.cpp"
    out = PKG / ("_sched_core" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    deps = [src, CSRC / "sched_core" / "engine.h"]
    if not force and out.exists() and out.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return out
    cxx = shutil.which("g++") or shutil.which("c++") or _hipcc()
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{pybind11.get_include()}",
           f"-I{sysconfig.get_paths()['include']}", str(src), "-o", str(out) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr[-6000:], file=sys.stderr)
        raise RuntimeError("sched_core build failed")
    os.replace(str(out) + ".tmp", out)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    p = build(force=a.force, jobs=a.j, verbose=a.v)
    print(p)
    print(build_sched_core(force=a.force))


if __name__ == "__main__":
    main()
