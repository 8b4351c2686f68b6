"""MILP placement (scipy / HiGHS).

The reference sketches a CPLEX model that minimises the maximum per-node
network traffic of a PS/worker job subject to GPU/CPU capacity
(``/root/reference/core/lp.py:2-44``) but its ``placement()`` is a stub and
the module does not import. For all-reduce gangs every node that holds part
of the gang carries the same ring traffic, so minimising the max traffic is
minimising the number of nodes spanned; ties are broken towards nodes that
are already partly used (best fit, keeps whole nodes free).

    min  sum_n y_n + eps * sum_n frag_n * x_n
    s.t. sum_n x_n = W                  (all workers placed)
         x_n <= cap_n * y_n             (GPU / CPU / mem capacity of node n)
         x_n in Z>=0, y_n in {0,1}
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..cluster.topology import Cluster, Plan
from ..core.job import Job
from .schemes import Placement, _Scratch


class LPPlacement(Placement):
    name = "lp"

    def plan(self, cluster: Cluster, job: Job) -> Optional[Plan]:
        from scipy.optimize import Bounds, LinearConstraint, milp

        t = job.tasks[0]
        nodes = list(cluster.nodes)
        N = len(nodes)
        W = len(job.tasks)
        cap = []
        for nid in nodes:
            n = cluster.nodes[nid]
            c = min(n.num_free_gpus() // max(1, t.gpu), n.cpu_free() // max(1, t.cpu),
                    n.mem_free() // max(1, t.mem))
            cap.append(max(0, c))
        if sum(cap) < W:
            return None
        frag = np.array([cluster.nodes[nid].num_free_gpus() / cluster.nodes[nid].gpu_count for nid in nodes])
        # variables: x_0..x_{N-1}, y_0..y_{N-1}
        c = np.concatenate([1e-3 * frag, np.ones(N)])
        A_sum = np.concatenate([np.ones(N), np.zeros(N)])[None, :]
        A_link = np.hstack([np.eye(N), -np.diag(cap)])
        cons = [LinearConstraint(A_sum, W, W), LinearConstraint(A_link, -np.inf, 0)]
        integrality = np.ones(2 * N)
        bounds = Bounds(np.zeros(2 * N), np.concatenate([np.array(cap, float), np.ones(N)]))
        res = milp(c, constraints=cons, integrality=integrality, bounds=bounds)
        if not res.success:
            return None
        x = np.round(res.x[:N]).astype(int)
        s = _Scratch(cluster)
        plan: Plan = []
        it = iter(job.tasks)
        for nid, k in zip(nodes, x):
            for _ in range(k):
                task = next(it)
                devs = s.try_task(nid, task)
                if devs is None:
                    return None
                plan.append((nid, devs))
        return plan if len(plan) == W else None
