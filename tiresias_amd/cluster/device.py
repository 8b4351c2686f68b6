"""Real-device backend: what the live runtime knows about the GPUs it owns.

The reference's ``Device`` (``infra/device.py:4-58``) is a pure model — memory
is a configured capacity and utilisation is *sampled* from N(avg, (max-avg)/2)
per call (``device.py:30-36``). On the real MI355X node the runtime instead
reads:

* HBM capacity / free bytes from the HIP runtime (``torch.cuda.mem_get_info``,
  i.e. ``hipMemGetInfo``) — per device, no model;
* GPU activity (%) and VRAM use from ``amd-smi metric`` (JSON), falling back to
  ``rocm-smi --showuse --showmemuse --json``; absent both, ``None`` (never a
  synthetic number);
* the xGMI link matrix (``amd-smi topology``) when available, so the placement
  engine can tell directly-linked GPU pairs.

``probe_cluster_spec()`` turns the local node into a ``ClusterSpec`` (one node,
N GPUs, measured HBM), and ``DeviceMonitor`` samples utilisation/memory for
the runtime's gpu.csv rows.
"""
from __future__ import annotations

import json
import shutil
import subprocess
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

from ..config import ClusterSpec


@dataclass
class DeviceInfo:
    index: int
    name: str
    total_mb: float
    free_mb: float
    util_pct: Optional[float] = None
    vram_used_mb: Optional[float] = None


def _run_json(cmd: List[str], timeout: float = 10.0):
    exe = shutil.which(cmd[0]) or f"/opt/rocm/bin/{cmd[0]}"
    try:
        r = subprocess.run([exe] + cmd[1:], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired):
        return None
    if r.returncode != 0 or not r.stdout.strip():
        return None
    try:
        return json.loads(r.stdout)
    except json.JSONDecodeError:
        return None


def _num(v) -> Optional[float]:
    """amd-smi values are numbers, strings, or {"value": x, "unit": u}."""
    if isinstance(v, dict):
        v = v.get("value")
    try:
        return float(str(v).strip().rstrip("%"))
    except (TypeError, ValueError):
        return None


def smi_utilization() -> Dict[int, Dict[str, Optional[float]]]:
    """{gpu index: {"util_pct", "vram_used_mb"}} from amd-smi (or rocm-smi)."""
    out: Dict[int, Dict[str, Optional[float]]] = {}
    d = _run_json(["amd-smi", "metric", "--usage", "--mem-usage", "--json"])
    if isinstance(d, dict):
        d = d.get("gpu_data", d.get("gpus", [d]))
    if isinstance(d, list):
        for i, g in enumerate(d):
            if not isinstance(g, dict):
                continue
            idx = int(_num(g.get("gpu", i)) or i)
            use = g.get("usage", {}) or {}
            mem = g.get("mem_usage", {}) or {}
            out[idx] = {"util_pct": _num(use.get("gfx_activity", use.get("gfx_usage"))),
                        "vram_used_mb": _num(mem.get("used_vram"))}
        if out:
            return out
    d = _run_json(["rocm-smi", "--showuse", "--showmemuse", "--json"])
    if isinstance(d, dict):
        for k, g in d.items():
            if not k.startswith("card"):
                continue
            idx = int(k[4:])
            out[idx] = {"util_pct": _num(g.get("GPU use (%)")), "vram_used_mb": None}
    return out


def xgmi_links() -> Optional[List[List[int]]]:
    """Hop matrix between local GPUs from ``amd-smi topology`` (None if absent)."""
    d = _run_json(["amd-smi", "topology", "--json"])
    if not isinstance(d, list):
        return None
    n = len(d)
    hops = [[0] * n for _ in range(n)]
    for i, g in enumerate(d):
        links = g.get("links", []) if isinstance(g, dict) else []
        for j, l in enumerate(links[:n]):
            hops[i][j] = int(_num(l.get("num_hops", 0)) or 0) if isinstance(l, dict) else 0
    return hops


def probe_devices(with_smi: bool = True) -> List[DeviceInfo]:
    import torch

    if not torch.cuda.is_available():
        return []
    smi = smi_utilization() if with_smi else {}
    out = []
    for i in range(torch.cuda.device_count()):
        free, total = torch.cuda.mem_get_info(i)
        s = smi.get(i, {})
        out.append(DeviceInfo(i, torch.cuda.get_device_name(i), total / 2 ** 20, free / 2 ** 20,
                              s.get("util_pct"), s.get("vram_used_mb")))
    return out


def probe_cluster_spec(base: Optional[ClusterSpec] = None) -> ClusterSpec:
    """The local node as a one-node cluster (measured GPU count and HBM)."""
    spec = base or ClusterSpec.mi355x_node()
    devs = probe_devices(with_smi=False)
    if not devs:
        return spec
    return ClusterSpec(**{**spec.__dict__, "num_switch": 1, "num_node_p_switch": 1,
                          "num_gpu_p_node": len(devs),
                          "gpu_memory_mb": min(d.total_mb for d in devs)})


class DeviceMonitor:
    """Samples the local GPUs at most every ``period`` seconds.

    ``sample()`` probes synchronously (tools, one-off queries). A training
    worker instead calls ``start()`` once and then ``sample_own()`` every
    round: the ``amd-smi`` subprocess (hundreds of ms) runs on a daemon
    thread and only HIP's mem-info of the worker's OWN device is read inline
    (microseconds, and no HIP context is created on the other GPUs), so
    monitoring never stalls the scheduling loop or the GPU."""

    def __init__(self, period: float = 5.0, with_smi: bool = True, device_index: Optional[int] = None):
        self.period = period
        self.with_smi = with_smi
        self.device_index = device_index
        self._last = 0.0
        self._cache: List[DeviceInfo] = []
        self._smi: Dict[int, dict] = {}
        self._thread = None
        self._stop = threading.Event()

    def sample(self, force: bool = False) -> List[DeviceInfo]:
        now = time.monotonic()
        if force or not self._cache or now - self._last >= self.period:
            self._cache = probe_devices(self.with_smi)
            self._last = now
        return self._cache

    # ------------------------------------------------ background (workers)
    def start(self) -> "DeviceMonitor":
        if self.with_smi and self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="tam-smi", daemon=True)
            self._thread.start()
        return self

    def _loop(self):
        while not self._stop.is_set():
            try:
                self._smi = smi_utilization()
            except Exception:                     # a missing/broken CLI is not fatal
                self._smi = {}
            self._stop.wait(self.period)

    def stop(self):
        self._stop.set()

    def sample_own(self) -> Optional[DeviceInfo]:
        import torch

        i = self.device_index
        if i is None or not torch.cuda.is_available():
            return None
        free, total = torch.cuda.mem_get_info(i)
        s = self._smi.get(i, {})
        return DeviceInfo(i, "", total / 2 ** 20, free / 2 ** 20, s.get("util_pct"),
                          s.get("vram_used_mb"))
