"""One job's training engine on one GPU rank (a DDP gang member).

A ``Trainer`` owns the job's flat parameter arena, optimizer state, static
synthetic batch, the bucketed all-reduce (when the gang spans >1 GPU) and an
optional hipGraph of forward+backward. It is what the cluster executor
time-slices: ``run(iters)`` advances the job, ``state_tensors()`` exposes the
four flat buffers a preemption checkpoints, ``release()`` frees HBM.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import torch

from ..models import MODELS, make_model, samples_per_batch, synthetic_batch
from ..ops import _lib
from ..ops import functional as Fx
from ..ops.arena import Arena
from ..parallel.ddp import GradBucketer
from ..parallel.gang import comm_size


class Trainer:
    def __init__(self, model: str, device, batch: Optional[int] = None, group=None, seed: int = 0,
                 data_seed: Optional[int] = None, use_graph: bool = False, bucket_mb: float = 32.0,
                 model_kwargs: Optional[dict] = None, lr: Optional[float] = None,
                 overlap_wgrad: Optional[bool] = None, branches: Optional[bool] = None,
                 ddp_shard: bool = False, ddp_wire: str = "fp32"):
        self.model_name = model
        self.spec = MODELS[model]
        self.device = torch.device(device)
        if self.device.type == "cuda":
            _lib.load(required=True)
        self.batch = batch or self.spec.batch
        self.arena = Arena(self.device, seed=seed)
        self.model = make_model(model, self.arena, **(model_kwargs or {}))
        self.arena.materialize()
        n = self.arena.numel
        self.opt = self.spec.opt
        self.lr = lr if lr is not None else self.spec.lr
        if self.opt == "sgd":
            self.opt_state = [torch.zeros(n, dtype=torch.float32, device=self.device)]
        else:
            self.opt_state = [torch.zeros(n, dtype=torch.float32, device=self.device),
                              torch.zeros(n, dtype=torch.float32, device=self.device)]
        self.step_count = 0
        self.data = synthetic_batch(model, self.batch, self.device,
                                    seed=seed if data_seed is None else data_seed)
        self.group = group
        self.ddp = None
        self._bucket_mb = bucket_mb
        # sharded data parallelism (parallel/ddp.py): reduce-scatter + 1/N
        # optimizer + bf16 shadow all-gather; master / optimizer state sharded
        # until consolidate()
        self.ddp_shard, self.ddp_wire = ddp_shard, ddp_wire
        if group is not None and comm_size(group) > 1:
            self.ddp = GradBucketer(self.arena, group, bucket_mb=bucket_mb, shard=ddp_shard, wire=ddp_wire)
        from ..utils import debug

        # kernel debug mode synchronises after every op: not capturable
        self._want_graph = use_graph and self.device.type == "cuda" and debug.level() == 0
        self.use_graph = self._want_graph and self.ddp is None   # graphs for 1-GPU jobs only
        self._graph = None
        self._g_loss = None
        self._g_written = []     # store_grad params the captured backward writes
        self._warm = 0           # eager steps done before graph capture
        self.capture_s = 0.0     # host seconds spent capturing the hipGraph
        self._side = None
        self._ws = None                 # weight-gradient stream (1-GPU jobs)
        self._defer_n = 0               # problems the last backward deferred
        self.overlap_wgrad = self.spec.overlap_wgrad if overlap_wgrad is None else overlap_wgrad
        # grouped weight gradients (TAM_GROUP_WGRAD=0 turns them off for A/B runs)
        self.group_wgrad = self.spec.group_wgrad and os.environ.get("TAM_GROUP_WGRAD", "1") != "0"
        # model-declared branch streams (see _fwd_bwd); None = the model's default
        self.branches = getattr(self.model, "branch_default", False) if branches is None else branches
        self._bs: List = []
        self.last_loss: Optional[torch.Tensor] = None
        # weight init and the synthetic batch were queued on the stream that
        # built the trainer; a step issued from another stream (GPU sharing
        # runs each job on its own stream) must wait for them first
        self._ready = None
        if self.device.type == "cuda":
            self._ready = torch.cuda.Event()
            self._ready.record(torch.cuda.current_stream(self.device))

    # ------------------------------------------------------------ one step
    def _fwd_bwd(self) -> torch.Tensor:
        d = self.data
        # 1-GPU jobs: weight gradients on their own stream, concurrent with
        # the input-gradient chain (ops/functional.py::set_wgrad_stream)
        ws = None
        if self.device.type == "cuda" and self.ddp is None and self.overlap_wgrad:
            if self._ws is None:
                # (stream priorities were measured: no gain in graph replay)
                self._ws = torch.cuda.Stream(self.device)
            ws = self._ws
        Fx.set_wgrad_stream(ws)
        # independent model branches on their own streams (1-GPU jobs;
        # ops/functional.py::on_branch), joined before the optimizer
        nb = getattr(self.model, "branch_streams", 0) if self.branches else 0
        if self.device.type == "cuda" and self.ddp is None and nb:
            if len(self._bs) < nb:
                self._bs = [torch.cuda.Stream(self.device) for _ in range(nb)]
            Fx.set_branch_streams(self._bs)
        group = (self.device.type == "cuda" and self.ddp is None and self.group_wgrad)
        if group:
            # the backward's weight gradients as ONE grouped launch at its end
            # (an early flush on a side stream measured slower: ResNet-50 9.07
            # vs 8.89 ms, Transformer 5.41 vs 5.30; removed in round 6)
            Fx.defer_wgrad(True)
        try:
            if self.spec.kind == "image":
                logits = self.model.forward(d["x"])
            else:
                logits = self.model.forward(d)
            labels = d["labels"]
            rows = labels.numel()
            # time-major logits [T,B,V] read the [B,T] labels in place
            loss, dlog = Fx.softmax_xent(logits, labels, smoothing=self.spec.smoothing,
                                         ignore_index=-100, normalizer=rows,
                                         labels_time_major=getattr(self.model, "logits_time_major", False))
            logits.backward(dlog)
            if group:
                Fx.flush_wgrad()
                self._defer_n = Fx.deferred_count()
        finally:
            if group:
                Fx.defer_wgrad(False, discard=True)
            Fx.set_wgrad_stream(None)
            Fx.set_branch_streams(None)
        if ws is not None:
            torch.cuda.current_stream(self.device).wait_stream(ws)   # join before the optimizer
        if self.device.type == "cuda" and self.ddp is None and nb:
            for s in self._bs:
                torch.cuda.current_stream(self.device).wait_stream(s)
        return loss

    def _opt_step(self):
        A = self.arena
        gscale = self.ddp.grad_scale if self.ddp is not None else 1.0
        self.step_count += 1
        sharded = self.ddp is not None and self.ddp.shard
        if sharded:
            # a shadow all-gather of the previous step still in flight (a
            # bucket whose params the forward never read through Param.w)
            # would overwrite this member's slice after the optimizer below
            # writes it: join them all first (free when already joined)
            self.ddp.join_gather()
            # this member's slices (+ replicated tails), split at the
            # decay / no-decay boundary; the gradient is reset as a whole below
            regions = []
            for a, b in self.ddp.owned_ranges():
                if a < A.n_decay:
                    regions.append((a, min(b, A.n_decay), self.spec.wd))
                if b > A.n_decay:
                    regions.append((max(a, A.n_decay), b, 0.0))
        elif self.device.type == "cuda":
            # store_grad params: every step's first gradient write stores
            # (Fx.grad_mode), so their region is not zeroed -- except a param
            # nothing wrote this step (its buffer holds an older gradient).
            # ONE launch over the whole arena: the store / decay / no-decay
            # regions are passed as bounds (zero_from, wd_until)
            for p in A.params:
                if p.store_grad and p.gw_epoch != A.grad_epoch:
                    p.grad.zero_()
            A.grad_epoch += 1
            T = _lib.ops()
            guard = self.model.err if self.uses_persist else None
            zf = A.n_store if Fx.STORE_GRAD else 0
            if self.opt == "sgd":
                T.sgd_step(A.master, A.grad, self.opt_state[0], A.shadow, self.lr, 0.9, self.spec.wd, gscale, False,
                           True, guard, zf, A.n_decay)
            else:
                T.adam_step(A.master, A.grad, self.opt_state[0], self.opt_state[1], A.shadow, self.lr, 0.9, 0.98,
                            1e-9, self.spec.wd, self.step_count, gscale, True, guard, zf, A.n_decay)
            if self.uses_persist:
                _lib.ops().lstm_guard_step(self.model.err)
            return
        else:
            regions = [(0, A.n_decay, self.spec.wd), (A.n_decay, A.numel, 0.0)]
        A.grad_epoch += 1
        for reg in regions:
            lo, hi, wd = reg[:3]
            zero = (reg[3] if len(reg) > 3 else True) and not sharded
            if hi <= lo:
                continue
            w, g, wb = A.master[lo:hi], A.grad[lo:hi], A.shadow[lo:hi]
            if self.device.type == "cuda":
                T = _lib.ops()
                # GNMT: a step whose persistent recurrence timed out (this
                # job's own timeout word) only resets the gradient
                guard = self.model.err if self.uses_persist else None
                if self.opt == "sgd":
                    T.sgd_step(w, g, self.opt_state[0][lo:hi], wb, self.lr, 0.9, wd, gscale, False, zero, guard)
                else:
                    T.adam_step(w, g, self.opt_state[0][lo:hi], self.opt_state[1][lo:hi], wb, self.lr,
                                0.9, 0.98, 1e-9, wd, self.step_count, gscale, zero, guard)
            else:
                _cpu_opt(self.opt, w, g, self.opt_state, lo, hi, wb, self.lr, wd, gscale, self.step_count)
        if sharded:
            A.grad.zero_()                 # the slices of the other members held local partials
            self.ddp.gather_shadow()
        if self.uses_persist:
            # a guarded step -> the job's skipped-step count (persist_skipped)
            _lib.ops().lstm_guard_step(self.model.err)

    def enable_graph(self) -> None:
        """Turn hipGraph capture on for a trainer built without it (a pooled
        trainer now running a long job): two eager warm steps, then capture."""
        from ..utils import debug

        if self.device.type != "cuda" or debug.level() != 0 or self.ddp is not None:
            return
        self._want_graph = True
        self.use_graph = True
        self._graph = None
        self._warm = 0

    @property
    def uses_persist(self) -> bool:
        """The model runs the persistent-grid LSTM kernels (GNMT) -- unless
        they are off for good (a barrier timeout) or for now (its GPU is
        shared with another persistent-grid job, ``set_persist_shared``)."""
        return (self.device.type == "cuda" and bool(getattr(self.model, "persist", False))
                and not getattr(self, "_persist_shared", False))

    def set_persist_shared(self, shared: bool) -> None:
        """While another job's persistent LSTM grids may run on the same GPU
        (GPU sharing in one worker, or another rank of the one-GPU rehearsal),
        take the per-step recurrence: two different persistent kernels cannot
        be guaranteed co-resident. Back to the persistent grids once the job
        runs alone (a change re-captures the step graph)."""
        shared = bool(shared)
        if shared != getattr(self, "_persist_shared", False):
            self._persist_shared = shared
            if hasattr(self.model, "shared"):   # models with persistent grids only
                self.model.shared = shared
                self._graph = None
                self._g_loss = None

    def persist_skipped(self, reset: bool = True) -> int:
        """Steps of THIS job whose persistent recurrence timed out since the
        last reset (their weight update was skipped; they are not progress).
        A host read: call after the round's synchronize."""
        if not self.uses_persist:
            return 0
        n = int(self.model.err[1].item())
        if reset and n:
            self.model.err.zero_()
        return n

    def disable_persist(self) -> None:
        """After a persistent-barrier timeout: the per-step recurrence for the
        rest of the job (a captured graph baked the persistent kernels in, so
        it is re-captured)."""
        if hasattr(self.model, "persist"):
            self.model.persist = False
        self._graph = None
        self._g_loss = None

    def step(self) -> torch.Tensor:
        if self.uses_persist:
            # co-residency rule of THIS job's persistent grids (lstm.hip,
            # passed with every launch): a DDP gang's RCCL kernels run next to
            # the recurrence -> keep CUs free for them; a 1-GPU job may share
            # its GPU with one more grid
            self.model.residency = (1, 64) if self.ddp is not None else (2, 0)
        if self._ready is not None:
            torch.cuda.current_stream(self.device).wait_event(self._ready)
            self._ready = None
        if self.use_graph and self._graph is None and self._warm < 2:
            # the first two steps are REAL steps run eagerly on a side stream
            # (allocator pools, library handles/workspaces, GEMM route tuning
            # happen outside capture); no work is thrown away
            s = self._side or torch.cuda.Stream(self.device)
            self._side = s
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                loss = self._fwd_bwd()
                self._opt_step()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._warm += 1
            self.last_loss = loss
            return loss
        if self.use_graph:
            loss = self._graph_step()
        else:
            loss = self._fwd_bwd()
            if self.ddp is not None:
                self.ddp.finish()
        self._opt_step()
        self.last_loss = loss
        return loss

    def _graph_step(self) -> torch.Tensor:
        if self._graph is None:
            # capture fwd+bwd once (capture itself runs no kernels), then
            # replay. Driven directly rather than through torch.cuda.graph(),
            # whose entry does gc.collect() + empty_cache(): in a long-lived
            # worker holding many jobs that costs ~20 ms and hands cached
            # blocks back to the driver, a fixed cost every job would pay
            # on its first graph step (JCT of short jobs)
            s = self._side or torch.cuda.Stream(self.device)
            self._side = s
            cur = torch.cuda.current_stream(self.device)
            s.wait_stream(cur)
            tc = time.perf_counter()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                g.capture_begin()
                try:
                    self._g_loss = self._fwd_bwd()
                finally:
                    g.capture_end()
            cur.wait_stream(s)
            self._graph = g
            self.capture_s += time.perf_counter() - tc
            # the gradient writes baked into the graph (store-mode firsts
            # included) happen on every replay: _opt_step must see them
            A = self.arena
            self._g_written = [p for p in A.params if p.store_grad and p.gw_epoch == A.grad_epoch]
        self._graph.replay()
        for p in self._g_written:
            p.gw_epoch = self.arena.grad_epoch
        return self._g_loss

    def run(self, iters: int) -> float:
        """Run ``iters`` steps; returns wall seconds (device-synchronised)."""
        t0 = time.perf_counter()
        for _ in range(iters):
            self.step()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    def samples_per_step(self) -> int:
        return samples_per_batch(self.model_name, self.batch)

    # ------------------------------------------------------------ state
    def consolidate(self) -> int:
        """Sharded data parallelism: all-gather the master / optimizer-state
        slices so this member holds the job's full state (collective over
        the gang; every member calls it). Returns bytes gathered."""
        if self.ddp is None or not self.ddp.shard:
            return 0
        return self.ddp.consolidate([self.arena.master] + list(self.opt_state))

    @property
    def state_sharded(self) -> bool:
        return self.ddp is not None and self.ddp.shard and self.ddp.dirty

    def state_tensors(self) -> Dict[str, torch.Tensor]:
        if self.state_sharded:
            raise RuntimeError("trainer state is sharded across its gang: consolidate() first")
        st = {"master": self.arena.master, "shadow": self.arena.shadow}
        for i, t in enumerate(self.opt_state):
            st[f"opt{i}"] = t
        for k, v in self.model.buffers().items():
            st["buf." + k] = v
        return st

    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.state_tensors().values())

    # ------------------------------------------------------------ host spill
    def _spill_buffers(self):
        bufs = [self.arena.master] + list(self.opt_state)
        bufs += [v for v in self.model.buffers().values()]
        return bufs

    def offload(self, engine) -> int:
        """Spill the job's state to pinned host DRAM through the native
        checkpoint engine (D2H on its low-priority side stream, ordered after
        the work already queued on this stream) and release the HBM by
        shrinking the flat buffers' storages to zero bytes (every parameter
        view shares those storages, so nothing else changes). The host NEVER
        waits for the copy: each spilled buffer is record_stream()-ed on the
        engine's side stream before it is freed, so the caching allocator
        reuses that HBM only once the D2H has drained. The bf16 shadow and
        the grad buffer are not saved (the shadow is rebuilt from the master
        on restore, the grad buffer is zero between steps). Returns bytes
        spilled."""
        if getattr(self, "_spilled", None):
            return 0
        if self.state_sharded:
            # only this member's slices of master / optimizer state are
            # current: spilling them would lose the job (consolidate() first)
            raise RuntimeError("trainer state is sharded across its gang: consolidate() before offload()")
        self._release_host_copies()
        self._graph = None
        self._g_loss = None
        self.last_loss = None
        handles, nbytes = [], 0
        self._save_counted = False
        for b in self._spill_buffers():
            handles.append((b, engine.spill(b), b.untyped_storage().nbytes()))
            nbytes += b.numel() * b.element_size()
        if self.device.type == "cuda":
            side = torch.cuda.ExternalStream(engine.stream_handle(), device=self.device)
            for b, _, _ in handles:
                b.record_stream(side)
        for b in [self.arena.master, self.arena.shadow, self.arena.grad] + list(self.opt_state):
            b.untyped_storage().resize_(0)
        self._spilled = handles
        self._engine = engine
        return nbytes

    def restore(self) -> int:
        """Re-allocate the HBM and copy the state back (H2D on the engine's
        side stream; the compute stream waits on its event, the host does not)."""
        handles = getattr(self, "_spilled", None)
        if not handles:
            return 0
        A = self.arena
        for b, n in ((A.master, A.numel * 4), (A.shadow, A.numel * 2), (A.grad, A.numel * 4)):
            b.untyped_storage().resize_(n)
        for t in self.opt_state:
            t.untyped_storage().resize_(t.numel() * 4)
        nbytes = 0
        for b, h, _ in handles:
            self._engine.restore(h, b)
            nbytes += b.numel() * b.element_size()
        A.grad.zero_()
        A.shadow.copy_(A.master.to(torch.bfloat16))
        if hasattr(self._engine, "copy_ms"):
            self._restored = handles      # host copies released by ckpt_poll once the H2D is done
        else:
            for _, h, _ in handles:
                self._engine.release(h)
        self._spilled = None
        return nbytes

    def ckpt_poll(self) -> dict:
        """Measured device copy seconds of spills / restores completed since
        the last poll ({"save_s", "restore_s"}); releases the host copies of
        restores that finished. Never blocks (in-flight copies are picked up
        by a later poll)."""
        out = {"save_s": 0.0, "restore_s": 0.0}
        eng = getattr(self, "_engine", None)
        if eng is None or not hasattr(eng, "copy_ms"):
            return out
        for which in ("_spilled", "_restored"):
            hs = getattr(self, which, None) or []
            if hs and not getattr(self, "_save_counted", False):
                ms = [eng.copy_ms(h, 0) for _, h, _ in hs]
                if all(m >= 0 for m in ms):
                    out["save_s"] += sum(ms) / 1e3
                    self._save_counted = True
        restored = getattr(self, "_restored", None) or []
        if restored and getattr(self, "_save_counted", False):
            ms = [eng.copy_ms(h, 1) for _, h, _ in restored]
            if all(m >= 0 for m in ms):
                out["restore_s"] += sum(ms) / 1e3
                for _, h, _ in restored:
                    eng.release(h)
                self._restored = None
        return out

    def reset(self, seed: int, data_seed: Optional[int] = None, init: bool = True) -> "Trainer":
        """Turn this (finished job's) trainer into a FRESH job of the same
        model/batch/gang: weights re-initialised from ``seed``, optimizer state
        and step count zeroed, a new synthetic batch, BN statistics reset.
        Every buffer keeps its address, so the captured hipGraph, the DDP
        bucketer and the caching-allocator blocks are reused: a job start
        costs a few init kernels instead of allocation + warm-up + capture
        (the worker's warm pool, ``cluster_runtime.Worker``). ``init=False``
        skips the weight init (the state is about to be overwritten by a P2P
        receive)."""
        if getattr(self, "_spilled", None):
            raise RuntimeError("reset of a spilled trainer")
        if self.ddp is not None:
            # fresh state (re-initialised identically on every member, or
            # about to be overwritten whole by a P2P receive)
            self.ddp.dirty = False
        if init:
            self.arena.reinit(seed)
            for t in self.opt_state:
                t.zero_()
            for k, v in self.model.buffers().items():
                if k.endswith(".var"):
                    v.fill_(1.0)
                else:
                    v.zero_()
        fresh = synthetic_batch(self.model_name, self.batch, self.device,
                                seed=seed if data_seed is None else data_seed)
        for k, v in fresh.items():
            self.data[k].copy_(v)
        self.step_count = 0
        self.last_loss = None
        if self.device.type == "cuda":
            self._ready = torch.cuda.Event()
            self._ready.record(torch.cuda.current_stream(self.device))
        return self

    def rebind(self, group) -> None:
        """Move the job to a new DDP gang (after a preemption resumed it on
        different GPUs): new communicator, fresh bucketer."""
        # sharded state survives only a re-created communicator over the SAME
        # rank set (same member positions); anything else needs consolidate()
        dirty = self.state_sharded
        old_ranks = tuple(getattr(self.ddp.comm, "ranks", ())) if self.ddp is not None else ()
        new_ranks = tuple(getattr(group, "ranks", ())) if group is not None else ()
        if dirty and old_ranks != new_ranks:
            raise RuntimeError(f"sharded trainer state on {old_ranks} cannot move to {new_ranks}: "
                               "consolidate() first")
        # shadow all-gathers still pending on the old communicator (deferred
        # to the next forward) are abandoned: a broken gang may never finish
        # them; the new bucketer re-gathers below
        regather = self.ddp is not None and bool(self.ddp._gathers)
        if self.ddp is not None:
            self.ddp._gathers = {}
        self.group = group
        self.arena.on_grad_ready = None
        self.arena.on_param_use = None
        self.ddp = None
        # an interrupted step (a peer died mid-collective) may have left
        # partial gradients: the new gang starts from clean ones
        self.arena.grad.zero_()
        self.broken = False
        if group is not None and comm_size(group) > 1:
            self.ddp = GradBucketer(self.arena, group, bucket_mb=self._bucket_mb, shard=self.ddp_shard,
                                    wire=self.ddp_wire)
            self.ddp.dirty = dirty and self.ddp.shard
            if regather and self.ddp.dirty:
                # every member's own shadow slices are current (its optimizer
                # wrote them); rebuild the rest over the new communicator
                self.ddp.gather_shadow(defer=False)
        self.use_graph = self._want_graph and self.ddp is None
        self._graph = None

    def hbm_bytes(self) -> int:
        """Device bytes this trainer pins: state buffers + batch (the graph's
        private activation pool is not visible here)."""
        n = self.arena.numel * (4 + 2 + 4) + sum(t.numel() * 4 for t in self.opt_state)
        n += sum(v.numel() * v.element_size() for v in self.data.values())
        return n

    def _release_host_copies(self) -> None:
        eng = getattr(self, "_engine", None)
        for which in ("_restored", "_spilled"):
            for _, h, _ in getattr(self, which, None) or []:
                eng.release(h)
            setattr(self, which, None)

    def release(self) -> None:
        self._release_host_copies()
        self._graph = None
        self._g_loss = None
        self.last_loss = None                    # may alias the graph's output
        self.arena.on_grad_ready = None


def _cpu_opt(opt, w, g, state, lo, hi, wb, lr, wd, gscale, step):
    gg = g * gscale
    if opt == "sgd":
        m = state[0][lo:hi]
        d = gg + wd * w
        m.mul_(0.9).add_(d)
        w.sub_(lr * m)
    else:
        m, v = state[0][lo:hi], state[1][lo:hi]
        m.mul_(0.9).add_(0.1 * gg)
        v.mul_(0.98).add_(0.02 * gg * gg)
        mh = m / (1 - 0.9 ** step)
        vh = v / (1 - 0.98 ** step)
        w.sub_(lr * (mh / (vh.sqrt() + 1e-9) + wd * w))
    g.zero_()
    wb.copy_(w.to(torch.bfloat16))
