"""Flat parameter arena: the MI355X-native parameter store of one job.

Every job owns exactly four device buffers::

    master  fp32 [N]   optimizer-owned weights
    shadow  bf16 [N]   compute copy every kernel reads (rewritten by the fused
                       optimizer step, never by a separate cast pass)
    grad    fp32 [N]   backward kernels ACCUMULATE straight into it (conv wgrad
                       split-K atomics, GEMM epilogues, BN/LN reductions) --
                       except a GEMM that writes a weight's gradient FIRST in a
                       step, which stores; the bucketed all-reduce reduces it in
                       place; the optimizer step zeroes it (not the leading
                       store_grad params, whose first write always stores)
    state   fp32 [k*N] optimizer state (momentum / Adam m,v)

so a checkpoint is four memcpys, a preemption spill is one contiguous D2H per
buffer, a DDP bucket is a contiguous slice, and the optimizer is one launch.

Layout: weight-decayed params first (in registration = forward order; the
store_grad ones leading), then the no-decay params (norm scales/shifts,
biases). Every param is padded to
64 elements so each view starts 256-B aligned (16-B vector loads).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import torch

_ALIGN = 64


@dataclass
class Param:
    name: str
    shape: tuple
    init: str = "normal"
    std: float = 0.02
    decay: bool = True
    fp32_compute: bool = False     # kernels read the fp32 master (norm params)
    # every step's FIRST write of the gradient is a full-tensor store (a GEMM
    # in store mode, ops/functional.py::grad_mode): the optimizer step then
    # skips zeroing it (Arena layout: these params lead the decay region)
    store_grad: bool = False
    gw_epoch: int = -1             # Arena.grad_epoch of the last gradient write
    offset: int = 0
    numel: int = 0
    # views (set by Arena.materialize); the bf16 shadow view is ``w`` (a
    # property: a first read may first join a pending all-gather of it)
    _w: Optional[torch.Tensor] = field(default=None, repr=False)
    master: Optional[torch.Tensor] = None   # fp32 master view
    grad: Optional[torch.Tensor] = None     # fp32 grad view
    arena: Optional["Arena"] = field(default=None, repr=False)

    @property
    def w(self) -> Optional[torch.Tensor]:
        """bf16 shadow view. While a sharded gang's shadow all-gather is in
        flight (parallel/ddp.py GradBucketer.gather_shadow) the arena's
        ``on_param_use`` hook orders this read after the gather of THIS
        parameter's bucket only (the next forward overlaps the rest)."""
        a = self.arena
        if a is not None and a.on_param_use is not None:
            a.on_param_use(self)
        return self._w

    @w.setter
    def w(self, t: Optional[torch.Tensor]) -> None:
        self._w = t

    @property
    def value(self) -> torch.Tensor:
        """The tensor kernels consume (fp32 master for norm params, bf16 shadow otherwise)."""
        return self.master if self.fp32_compute else self.w

    def grad_ready(self) -> None:
        if self.arena is not None and self.arena.on_grad_ready is not None:
            self.arena.on_grad_ready(self)


def _padded(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class Arena:
    def __init__(self, device: torch.device | str = "cpu", seed: int = 0):
        self.device = torch.device(device)
        self.params: List[Param] = []
        self.seed = seed
        self.master = self.shadow = self.grad = None
        self.numel = 0
        self.n_decay = 0
        self.n_store = 0          # [0, n_store): the store_grad params
        self.grad_epoch = 0       # optimizer steps taken (ops/functional.py::grad_mode)
        self.on_grad_ready: Optional[Callable[[Param], None]] = None
        # set while a deferred shadow all-gather is pending (Param.w)
        self.on_param_use: Optional[Callable[[Param], None]] = None
        # autograd anchor: every param-consuming op takes it as an input so
        # outputs require grad even when the data input does not.
        self.token = torch.zeros(1, device=self.device, requires_grad=True)

    # ----------------------------------------------------------------- build
    def add(self, name: str, shape: Sequence[int], init: str = "normal", std: float = 0.02,
            decay: bool = True, fp32_compute: bool = False, store_grad: bool = False) -> Param:
        p = Param(name=name, shape=tuple(int(s) for s in shape), init=init, std=std, decay=decay,
                  fp32_compute=fp32_compute, store_grad=store_grad and decay)
        p.numel = int(math.prod(p.shape))
        p.arena = self
        self.params.append(p)
        return p

    def _order(self) -> List[Param]:
        return ([p for p in self.params if p.store_grad] + [p for p in self.params if p.decay and not p.store_grad]
                + [p for p in self.params if not p.decay])

    def layout(self) -> List[Param]:
        """Assign every param its arena offset (no allocation); returns the
        params in arena order."""
        off = 0
        order = self._order()
        for p in order:
            p.offset = off
            off += _padded(p.numel)
            if p.decay:
                self.n_decay = off
            if p.store_grad:
                self.n_store = off
        self.numel = max(off, _ALIGN)
        return order

    def materialize(self) -> "Arena":
        order = self.layout()
        dev = self.device
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.shadow = torch.zeros(self.numel, dtype=torch.bfloat16, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        for p in order:
            p.master = self.master[p.offset:p.offset + p.numel].view(p.shape)
            p.w = self.shadow[p.offset:p.offset + p.numel].view(p.shape)
            p.grad = self.grad[p.offset:p.offset + p.numel].view(p.shape)
        self.reinit(self.seed)
        return self

    def reinit(self, seed: int) -> None:
        """(Re-)initialise every parameter in place from ``seed``: the buffers
        keep their addresses, so a hipGraph captured over them stays valid
        (warm trainer reuse, ``executor/trainer.py::Trainer.reset``). Runs on
        the device itself: a 138M-param VGG-16 job starts in milliseconds
        instead of seconds of host RNG + H2D copy."""
        self.seed = seed
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        for p in self._order():
            self._init_into(p, g)
        self.shadow.copy_(self.master.to(torch.bfloat16))
        self.grad.zero_()

    @staticmethod
    def _init_into(p: Param, g: torch.Generator) -> None:
        t = p.master
        if p.init == "zeros":
            t.zero_()
        elif p.init == "ones":
            t.fill_(1.0)
        elif p.init == "kaiming":
            # fan_in over all dims but the first (conv [K,R,S,C], linear [out,in])
            fan_in = max(1, p.numel // p.shape[0])
            t.normal_(0.0, math.sqrt(2.0 / fan_in), generator=g)
        elif p.init == "xavier":
            fan_in = max(1, p.numel // p.shape[0])
            a = math.sqrt(6.0 / (fan_in + p.shape[0]))
            t.uniform_(-a, a, generator=g)
        elif p.init == "uniform":
            t.uniform_(-p.std, p.std, generator=g)
        else:
            t.normal_(0.0, p.std, generator=g)

    # ----------------------------------------------------------------- state
    def zero_grad(self) -> None:
        self.grad.zero_()

    def state_bytes(self) -> int:
        return self.numel * (4 + 2 + 4)

    def named(self):
        return {p.name: p for p in self.params}

    def sync_shadow(self) -> None:
        self.shadow.copy_(self.master.to(torch.bfloat16))
