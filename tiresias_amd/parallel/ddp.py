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

Sharded mode (``shard=True``, ZeRO-1/2 style; consolidated gangs only --
a spread gang's hierarchical transport keeps the all-reduce): each bucket's
main part (a multiple of ``world`` x 16 elements) is REDUCE-SCATTERED in
place instead of all-reduced, so member ``p`` (its position in the gang)
holds the summed gradient of slice ``p`` of every bucket; the few tail
elements past the last full slice, and the buckets of norm parameters the
kernels read in fp32, are all-reduced (replicated). The optimizer then runs
on the member's slices (+ the replicated tails) only -- 1/world of the
arena's optimizer traffic per member -- and the updated bf16 shadow slices
are ALL-GATHERED back into every member's compute copy. Per parameter and
step a member sends (W-1)/W x (4 + 2) bytes instead of 2(W-1)/W x 4 (25 %
fewer; ``wire="bf16"`` exchanges the gradient in bf16 -- an all-to-all of
bf16 slices summed in fp32 by the owning member, so no partial sum is
rounded to bf16 -- (W-1)/W x 4, half).
The fp32 master and the optimizer state are then SHARDED: only this
member's slices are current. ``consolidate()`` all-gathers them so every
member holds the full state again -- required before anything reads the
job's state (a preemption's P2P move or spill, a snapshot); the live
runtime issues it as a plan action when it suspends such a gang.

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


def check_disjoint(ranges: List[tuple]) -> None:
    """Bucket ranges must not overlap: an element in two buckets is reduced
    twice (W x the mean) and, sharded, updated by two owners."""
    last = -1
    for lo, hi in sorted(ranges):
        if lo < last:
            raise AssertionError(f"overlapping DDP bucket ranges at {lo} (< {last}): {sorted(ranges)}")
        last = hi


class GradBucketer:
    """``group``: a gang comm (``parallel/gang.py``: flat RCCL for a
    consolidated gang, hierarchical intra-node RCCL + throttled host-staged
    inter-node exchange for a spread one) or a plain process group."""

    def __init__(self, arena: Arena, group=None, bucket_mb: float = 32.0, overlap: bool = True,
                 shard: bool = False, wire: str = "fp32"):
        self.arena = arena
        self.comm = as_comm(group) if dist.is_initialized() else None
        self.group = group
        self.world = comm_size(self.comm) if self.comm is not None else 1
        self.overlap = overlap
        # sharded data parallelism only over a flat (consolidated) gang
        self.shard = bool(shard and self.world > 1 and getattr(self.comm, "sharding", False))
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"wire must be fp32 or bf16, not {wire!r}")
        self.wire = wire if self.shard else "fp32"
        self.position = self.comm.position if self.shard else 0
        self.dirty = False                       # sharded master / optimizer state (consolidate())
        elems = max(1, int(bucket_mb * (1 << 20) // 4))
        # A bucket must be ONE contiguous arena range. The arena is laid out
        # as [store_grad | other decay | no-decay] (ops/arena.py::Arena._order),
        # each region in registration order, so buckets are cut per region,
        # walking it from its highest offset down (backward produces the
        # last-registered params' gradients first). Walking all decay params
        # in registration order instead would let one bucket's [min, max)
        # span the other region and reduce those gradients twice.
        regions = ([p for p in arena.params if p.store_grad],
                   [p for p in arena.params if p.decay and not p.store_grad],
                   [p for p in arena.params if not p.decay])
        self.buckets: List[List[Param]] = []
        for plist in regions:
            cur, size = [], 0
            for p in sorted(plist, key=lambda q: q.offset, reverse=True):
                cur.append(p)
                size += p.numel
                if size >= elems:
                    self.buckets.append(cur)
                    cur, size = [], 0
            if cur:
                self.buckets.append(cur)
        self.bucket_of: Dict[int, int] = {}
        self.ranges = []
        self.slices = []          # sharded: per bucket (slice length s, main-part end lo + W*s)
        for bi, ps in enumerate(self.buckets):
            lo = min(p.offset for p in ps)
            hi = max(p.offset + p.numel for p in ps)
            hi = min(arena.numel, (hi + 63) // 64 * 64)
            self.ranges.append((lo, hi))
            # buckets holding params the kernels read in fp32 (norm params:
            # Param.fp32_compute) stay replicated -- every member needs their
            # updated master, and they are tiny
            sl = ((hi - lo) // self.world) // 16 * 16 if (self.shard and not any(p.fp32_compute for p in ps)) else 0
            self.slices.append((sl, lo + self.world * sl))
            for p in ps:
                self.bucket_of[id(p)] = bi
        check_disjoint(self.ranges)
        self._wbufs: List[Optional[torch.Tensor]] = []     # bf16 wire staging, per bucket
        self._rbufs: List[Optional[torch.Tensor]] = []     # bf16 all-to-all receive, per bucket
        self.uses: Optional[Dict[int, int]] = None
        self._seen: Dict[int, int] = {}
        self._pending: List[int] = []
        self._launched: List[bool] = []
        self._works = []
        self.bytes_reduced = 0
        # bytes this member SENDS (ring algorithms): all-reduce 2(W-1)/W x n,
        # reduce-scatter / all-gather (W-1)/W x n each
        self.wire_bytes = 0.0
        self._timed = self.world > 1 and arena.grad.is_cuda
        self._ev_first = None
        self._ev_open: List[tuple] = []          # (first, bwd_done, joined) per step, not yet read
        self._acc = {"exposed_s": 0.0, "span_s": 0.0, "steps": 0}
        self._bytes_acc = [0.0, 0]               # wire bytes / steps since the last poll
        # deferred shadow all-gathers (sharded): bucket -> work, joined at the
        # bucket's first parameter read in the next forward
        self._gathers: Dict[int, object] = {}
        self._gather_ev = None                   # [issued, last joined] on the compute stream
        self._gather_waits: List[tuple] = []     # (before, after) each join's wait
        self._gather_open: List[tuple] = []
        self._gacc = {"gather_exposed_s": 0.0, "gather_window_s": 0.0, "gather_steps": 0}
        arena.on_grad_ready = self._on_ready
        self._reset()

    def _reset(self):
        self._step_w0 = self.wire_bytes
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
            if self.shard:
                self._launch_shard(bi, lo, hi)
                return
            self._works.append(self.comm.start(view))
            self.wire_bytes += 2.0 * (self.world - 1) / self.world * view.numel() * 4
        self.bytes_reduced += view.numel() * 4

    def _launch_shard(self, bi: int, lo: int, hi: int) -> None:
        sl, mid = self.slices[bi]
        W, p = self.world, self.position
        g = self.arena.grad
        if sl > 0:
            if self.wire == "bf16":
                # bf16 on the wire, fp32 accumulation: cast the main part and
                # ALL-TO-ALL it (member j receives every member's copy of
                # slice j: the same (W-1)/W x n x 2 bytes as a bf16
                # reduce-scatter), then finish() sums the W received copies
                # in fp32 into this member's slice of the fp32 grad. A bf16
                # reduce-scatter would round every partial sum to bf16.
                buf = self._wire_buf(self._wbufs, bi, mid - lo)
                buf.copy_(g[lo:mid])
                recv = self._wire_buf(self._rbufs, bi, mid - lo)
                self._works.append(self.comm.all_to_all(recv, buf))
                self.bytes_reduced += (mid - lo) * 2
                self.wire_bytes += (W - 1) / W * (mid - lo) * 2
            else:
                self._works.append(self.comm.reduce_scatter(g[lo + p * sl:lo + (p + 1) * sl], g[lo:mid]))
                self.bytes_reduced += (mid - lo) * 4
                self.wire_bytes += (W - 1) / W * (mid - lo) * 4
        if hi > mid:                                  # tail: replicated
            self._works.append(self.comm.start(g[mid:hi]))
            self.bytes_reduced += (hi - mid) * 4
            self.wire_bytes += 2.0 * (W - 1) / W * (hi - mid) * 4

    def _wire_buf(self, pool: List[Optional[torch.Tensor]], bi: int, n: int) -> torch.Tensor:
        # one bf16 staging buffer per in-flight bucket (distinct memory: the
        # exchanges of several buckets are in flight together)
        while len(pool) <= bi:
            pool.append(None)
        b = pool[bi]
        if b is None or b.numel() < n:
            b = torch.empty(n, dtype=torch.bfloat16, device=self.arena.grad.device)
            pool[bi] = b
        return b[:n]

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
            if self.shard and self.wire == "bf16":
                g, p, W = self.arena.grad, self.position, self.world
                for bi, (sl, _) in enumerate(self.slices):
                    if sl > 0:
                        lo = self.ranges[bi][0]
                        copies = self._rbufs[bi][:W * sl].view(W, sl)
                        torch.sum(copies, dim=0, dtype=torch.float32, out=g[lo + p * sl:lo + (p + 1) * sl])
            if self._timed:
                done = torch.cuda.Event(enable_timing=True)
                done.record()
                self._ev_open.append((self._ev_first if self._ev_first is not None else bwd, bwd, done))
        self._ev_first = None
        if self.world > 1:
            self._bytes_acc[0] += self.wire_bytes - self._step_w0
            self._bytes_acc[1] += 1
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
        gkeep = []
        for (iss, end), waits in self._gather_open:
            if end.query():
                self._gacc["gather_window_s"] += iss.elapsed_time(end) / 1e3
                self._gacc["gather_exposed_s"] += sum(a.elapsed_time(b) for a, b in waits) / 1e3
                self._gacc["gather_steps"] += 1
            else:
                gkeep.append(((iss, end), waits))
        self._gather_open = gkeep
        out, self._acc = self._acc, {"exposed_s": 0.0, "span_s": 0.0, "steps": 0}
        out.update(self._gacc)
        self._gacc = {"gather_exposed_s": 0.0, "gather_window_s": 0.0, "gather_steps": 0}
        # wire bytes of the steps finished since the last poll (the sharded
        # all-gather of a step counts with the NEXT step's finish)
        out["bytes"], out["bytes_steps"] = self._bytes_acc
        self._bytes_acc = [0.0, 0]
        return out

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    # ------------------------------------------------------------ sharded mode
    def owned_ranges(self) -> List[tuple]:
        """Arena ranges whose summed gradient this member holds after
        finish(): its slice of every bucket plus every (replicated) tail."""
        out = []
        for (lo, hi), (sl, mid) in zip(self.ranges, self.slices):
            if sl > 0:
                a = lo + self.position * sl
                out.append((a, a + sl))
            if hi > mid:
                out.append((mid, hi))
        return sorted(out)

    def gather_shadow(self, defer: bool = True) -> None:
        """After the sharded optimizer step: every member's updated bf16
        slices into every member's compute copy (all-gather per bucket).

        ``defer`` (default): the gathers are issued in FORWARD order (the
        buckets were cut walking backward order, so reversed) and not
        joined here: the next forward's first read of a parameter
        (``Param.w``) joins only that parameter's bucket, so the later
        buckets' gathers overlap the forward's first layers.
        ``join_gather()`` joins whatever is still pending (before anything
        else reads the shadow: consolidate, a move, a snapshot)."""
        self.join_gather()
        sh, p = self.arena.shadow, self.position
        works: Dict[int, object] = {}
        for bi in reversed(range(len(self.ranges))):
            lo = self.ranges[bi][0]
            sl, mid = self.slices[bi]
            if sl > 0:
                works[bi] = self.comm.all_gather(sh[lo:mid], sh[lo + p * sl:lo + (p + 1) * sl])
                self.wire_bytes += (self.world - 1) / self.world * (mid - lo) * 2
        self.dirty = True
        if not works:
            return
        if not defer:
            self.comm.finish(list(works.values()))
            return
        self._gathers = works
        if self._timed:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._gather_ev = [ev, None]
        self.arena.on_param_use = self._before_use

    def _before_use(self, p: Param) -> None:
        bi = self.bucket_of.get(id(p))
        w = self._gathers.pop(bi, None) if bi is not None else None
        if w is not None:
            a = None
            if self._timed:
                a = torch.cuda.Event(enable_timing=True)
                a.record()
            self.comm.finish([w])
            if a is not None:
                b = torch.cuda.Event(enable_timing=True)
                b.record()
                self._gather_waits.append((a, b))
        if not self._gathers:
            self._close_gather()

    def _close_gather(self) -> None:
        self.arena.on_param_use = None
        if self._timed and self._gather_ev is not None:
            # issue -> last join on the compute stream: the forward work the
            # gathers overlapped with, plus their exposed waits
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            self._gather_ev[1] = end
            self._gather_open.append((self._gather_ev, self._gather_waits))
        self._gather_ev, self._gather_waits = None, []

    def join_gather(self) -> None:
        """Join every pending shadow all-gather (compute stream waits)."""
        if self._gathers:
            works = list(self._gathers.values())
            self._gathers = {}
            self.comm.finish(works)
            self._close_gather()

    def consolidate(self, state: List[torch.Tensor]) -> int:
        """All-gather the sharded fp32 buffers (master + optimizer state) so
        every member holds the full job state again; collective over the
        gang. Returns bytes gathered per member."""
        self.join_gather()
        if not self.dirty:
            return 0
        p, works, nb = self.position, [], 0
        for buf in state:
            for (lo, _), (sl, mid) in zip(self.ranges, self.slices):
                if sl > 0:
                    works.append(self.comm.all_gather(buf[lo:mid], buf[lo + p * sl:lo + (p + 1) * sl]))
                    nb += (mid - lo - sl) * buf.element_size()
        self.comm.finish(works)
        self.dirty = False
        return nb
