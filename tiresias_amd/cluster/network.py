"""Communication / interference cost models used by the simulator to turn a
placement into a progress rate.

The reference adds ``(model_size/bandwidth + cross_nodes*latency) *
iterations * 2`` seconds to a job's duration (``core/network/
network_service.py:3-39``) but crashes (defect D3: ``Job.ps_count``,
``model_size``, ``iterations`` do not exist). Here the same quantities give a
*rate*: per iteration, compute time c = duration / iterations and the
all-reduce of S bytes across k nodes costs a ring's 2(k-1)/k * S / bw plus
2(k-1) latencies on the inter-node links; rate = c / (c + comm). A gang
inside one node (xGMI on MI355X) pays nothing extra.

Measured costs (``--skew_profile``, written by ``profiler/comm.py`` from real
DDP bucket syncs of each model on a consolidated vs a spread gang over the
emulated inter-node link) replace the analytic formula for the models they
cover: ``measured_spread_rate``.

Interference: a task sharing a GPU runs at 1/(1 + factor) (reference
``infra/interference.py:1``, FACTOR = 0.2; the reference never applies it,
defect D6).
"""
from __future__ import annotations

from typing import Optional

from ..profiler.skew import model_profile


def allreduce_seconds(bytes_: float, nodes: int, bw_mbps: float, latency: float) -> float:
    if nodes <= 1:
        return 0.0
    k = nodes
    return 2.0 * (k - 1) / k * (bytes_ / 2 ** 20) / bw_mbps + 2.0 * (k - 1) * latency


def network_rate(job, nodes: int, bw_mbps: float, latency: float,
                 default_iter_s: float = 0.25) -> float:
    if nodes <= 1:
        return 1.0
    spec = job.spec
    try:
        mb = model_profile(spec.model).total_mb if spec.model else 100.0
    except KeyError:
        mb = 100.0
    iters = spec.iterations
    c = spec.duration / iters if iters and iters > 0 else default_iter_s
    comm = allreduce_seconds(mb * 2 ** 20, nodes, bw_mbps, latency)
    return c / (c + comm) if c > 0 else 1.0


def measured_spread_rate(slowdown_2: float, nodes: int) -> float:
    """Progress rate of a gang spread over ``nodes`` nodes from the MEASURED
    iteration slowdown of the same model spread over 2 (virtual) nodes. The
    extra per-iteration time is inter-node all-reduce traffic, which a ring
    scales by 2(k-1)/k: overhead_k = (slowdown_2 - 1) * 2(k-1)/k (= the
    measured overhead at k = 2)."""
    if nodes <= 1:
        return 1.0
    over = max(0.0, slowdown_2 - 1.0) * 2.0 * (nodes - 1) / nodes
    return 1.0 / (1.0 + over)


def interference_rate(shared: bool, factor: float) -> float:
    return 1.0 / (1.0 + factor) if shared else 1.0
