"""Bucketed gradient all-reduce over RCCL (xGMI), overlapped with backward.

The arena's flat fp32 grad buffer is cut into buckets at parameter
boundaries, walking the weight-decayed params from the LAST registered one
backwards (backward produces those grads first), plus the no-decay region
(norm params / biases) as the final buckets. Backward kernels call
``Param.grad_ready()`` after accumulating; when every use of every param in a
bucket has reported, that bucket's ``all_reduce`` is issued asynchronously
(RCCL runs it on its own stream, ordered after the producing kernels) while
the remaining backward kernels keep the CUs busy. ``finish()`` flushes any
unlaunched bucket and makes the compute stream wait for the reductions (a
device-side wait, the host is not blocked). The 1/world average is folded
into the optimizer kernel's gradient scale, so the reduction is a pure SUM in
place: no copies, no extra elementwise pass.

Bucket size: xGMI is point-to-point (7 links / GPU, ~153 GB/s each); RCCL's
ring/tree all-reduce over 8 ranks reaches its bus-bandwidth plateau at a few
tens of MB per call, so the default is 32 MB — large enough to amortise the
per-collective launch latency, small enough that the first bucket starts
early in backward.

Uses of a param (tied embeddings report twice) are learned on the first
iteration, which reduces every bucket at the end instead of overlapping.

Timing: on a GPU every step records three hipEvents on the
compute stream -- first bucket launched, backward done (``finish`` entry),
all reductions joined -- and ``poll_timing`` turns completed steps into
``exposed_s`` (the compute stream waiting on communication) and ``span_s``
(first bucket to last reduction), never blocking the host.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops.arena import Arena, Param
from .gang import as_comm, comm_size


class GradBucketer:
    """``group``: a gang comm (``parallel/gang.py``: flat RCCL for a
    consolidated gang, hierarchical intra-node RCCL + throttled host-staged
    inter-node exchange for a spread one) or a plain process group."""

    def __init__(self, arena: Arena, group=None, bucket_mb: float = 32.0, overlap: bool = True):
        self.arena = arena
        self.comm = as_comm(group) if dist.is_initialized() else None
        self.group = group
        self.world = comm_size(self.comm) if self.comm is not None else 1
        self.overlap = overlap
        elems = max(1, int(bucket_mb * (1 << 20) // 4))
        decay = [p for p in arena.params if p.decay]
        nodecay = [p for p in arena.params if not p.decay]
        self.buckets: List[List[Param]] = []
        for plist in (list(reversed(decay)), list(reversed(nodecay))):
            cur, size = [], 0
            for p in plist:
                cur.append(p)
                size += p.numel
                if size >= elems:
                    self.buckets.append(cur)
                    cur, size = [], 0
            if cur:
                self.buckets.append(cur)
        self.bucket_of: Dict[int, int] = {}
        self.ranges = []
        for bi, ps in enumerate(self.buckets):
            lo = min(p.offset for p in ps)
            hi = max(p.offset + p.numel for p in ps)
            hi = min(arena.numel, (hi + 63) // 64 * 64)
            self.ranges.append((lo, hi))
            for p in ps:
                self.bucket_of[id(p)] = bi
        self.uses: Optional[Dict[int, int]] = None
        self._seen: Dict[int, int] = {}
        self._pending: List[int] = []
        self._launched: List[bool] = []
        self._works = []
        self.bytes_reduced = 0
        self._timed = self.world > 1 and arena.grad.is_cuda
        self._ev_first = None
        self._ev_open: List[tuple] = []          # (first, bwd_done, joined) per step, not yet read
        self._acc = {"exposed_s": 0.0, "span_s": 0.0, "steps": 0}
        arena.on_grad_ready = self._on_ready
        self._reset()

    def _reset(self):
        self._seen = {}
        self._launched = [False] * len(self.buckets)
        self._works = []
        if self.uses is not None:
            self._pending = [sum(self.uses.get(id(p), 0) for p in ps) for ps in self.buckets]

    def _launch(self, bi: int):
        if self._launched[bi]:
            return
        self._launched[bi] = True
        lo, hi = self.ranges[bi]
        view = self.arena.grad[lo:hi]
        if self.world > 1:
            if self._timed and self._ev_first is None:
                self._ev_first = torch.cuda.Event(enable_timing=True)
                self._ev_first.record()
            self._works.append(self.comm.start(view))
        self.bytes_reduced += view.numel() * 4

    def _on_ready(self, p: Param):
        k = id(p)
        self._seen[k] = self._seen.get(k, 0) + 1
        if self.uses is None or not self.overlap:
            return
        bi = self.bucket_of.get(k)
        if bi is None:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            # launch in bucket order only: every rank must issue collectives in
            # the same sequence, so an out-of-order completion waits for the
            # earlier buckets (which backward normally finishes first anyway)
            for b in range(len(self.buckets)):
                if self._launched[b]:
                    continue
                if self._pending[b] == 0:
                    self._launch(b)
                else:
                    break

    def finish(self) -> None:
        """Flush unlaunched buckets and order the compute stream after them."""
        if self.uses is None:
            self.uses = dict(self._seen)
        bwd = None
        if self._timed:
            bwd = torch.cuda.Event(enable_timing=True)
            bwd.record()
        for b in range(len(self.buckets)):
            self._launch(b)
        if self._works:
            self.comm.finish(self._works)
            if self._timed:
                done = torch.cuda.Event(enable_timing=True)
                done.record()
                self._ev_open.append((self._ev_first if self._ev_first is not None else bwd, bwd, done))
        self._ev_first = None
        self._reset()

    def poll_timing(self) -> dict:
        """Measured communication seconds of the steps whose events have
        completed since the last poll: ``exposed_s`` (backward done -> all
        reductions joined) and ``span_s`` (first bucket -> joined)."""
        keep = []
        for first, bwd, done in self._ev_open:
            if done.query():
                self._acc["exposed_s"] += bwd.elapsed_time(done) / 1e3
                self._acc["span_s"] += first.elapsed_time(done) / 1e3
                self._acc["steps"] += 1
            else:
                keep.append((first, bwd, done))
        self._ev_open = keep
        out, self._acc = self._acc, {"exposed_s": 0.0, "span_s": 0.0, "steps": 0}
        return out

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world
