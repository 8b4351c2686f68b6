"""Autograd-aware ops over the HIP kernel library.

Conventions (MI355X-first):
  * activations are bf16; convolutions are NHWC ([N,H,W,C], C % 8 == 0);
  * parameters come from an :class:`~tiresias_amd.ops.arena.Arena`; backward
    kernels ACCUMULATE weight gradients directly into the arena's flat fp32
    grad buffer (no per-param grad tensors, no copies before the all-reduce)
    and then call ``param.grad_ready()`` so the DDP bucketer can launch the
    bucket's RCCL all-reduce while backward continues;
  * ReLU is fused into the producing kernel's epilogue; its backward mask is
    applied by the *consumer's* input-gradient epilogue when the consumer is
    told ``in_relu=True`` (no separate relu-backward pass).

On GPU tensors every op runs the hand-written gfx950 kernels (the library is
required and loaded eagerly); on CPU tensors the ops run an fp32 PyTorch
reference of the same math (CPU test-suite, gloo rehearsals, numerics refs).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import _lib
from .arena import Param

BF16 = torch.bfloat16


def _T():
    return _lib.ops()


def _cpu_gemm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return a.float() @ b.float()


# ============================================================ weight-gradient stream
# Weight gradients (dW = dY^T X, bias colsums, embedding scatter-adds) are off
# the backward critical path: nothing downstream in the backward pass reads
# them. When a trainer installs a side stream here, those kernels are issued
# on it -- forked from the compute stream right after dY exists, BEFORE the
# input-gradient kernel is launched -- so on the GPU they run concurrently with
# the dgrad / BN / LSTM-recurrence chain (latency-bound small GEMMs and
# memory-bound BN kernels fill each other's idle CUs). Inside a hipGraph
# capture the fork/join becomes parallel graph branches. Every writer of a
# given grad buffer must then sit on this stream (tied embedding/projection),
# and the trainer joins it before the optimizer (Trainer._fwd_bwd). Gangs
# (DDP) leave it unset: their bucket all-reduces follow grad_ready() on the
# compute stream.
_WGRAD_STREAM = None


def set_wgrad_stream(stream) -> None:
    global _WGRAD_STREAM
    _WGRAD_STREAM = stream


class _OnWgrad:
    def __init__(self, *tensors, stream=None):
        self.s = (stream or _WGRAD_STREAM) if tensors[0].is_cuda else None
        self.ts = tensors
        self.ctx = None

    def __enter__(self):
        if self.s is None:
            return self
        self.s.wait_stream(torch.cuda.current_stream(self.ts[0].device))
        for t in self.ts:
            t.record_stream(self.s)        # not recycled by the compute stream meanwhile
        self.ctx = torch.cuda.stream(self.s)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


# ============================================================ grouped weight gradients
# A trainer may DEFER every eligible Linear weight gradient of a backward pass
# (dW = dY^T X, db = colsum(dY)) and issue them together as ONE grouped
# launch (csrc/kernels/gemm_grouped.hip): the per-layer dW GEMMs of
# Transformer-base (512..2048 x 512 x 4096) each underfill the 256 CUs, while
# the ~60 of a step fill it as one grid. dY / X stay alive until the flush
# (a few MB each). ``TAM_WGRAD_GROUP_CHUNK`` = n > 0 flushes every n deferred
# layers instead of once at the end (A/B of overlap vs. fill).
_DEFER_WGRAD: Optional[list] = None
_DEFER_CHUNK = int(os.environ.get("TAM_WGRAD_GROUP_CHUNK", "0") or 0)
_GROUP_OK: dict = {}
_DEFER_COUNT = 0


def defer_wgrad(on: bool, discard: bool = False) -> None:
    """Start (True) or stop (False) deferring Linear weight gradients; stopping
    with problems still pending is a programming error (flush first) unless
    ``discard`` (an aborted step)."""
    global _DEFER_WGRAD, _DEFER_COUNT
    _DEFER_COUNT = 0
    if not on and _DEFER_WGRAD and not discard:
        raise RuntimeError("defer_wgrad(False) with unflushed weight gradients")
    if not on:
        _DEFER_LNRED.clear()               # (an aborted step: its partial rows are dropped)
    if not on and _DEFER_WGRAD:
        for it in _DEFER_WGRAD:            # dropped writes: the next one must store (grad_mode)
            it[2].gw_epoch = -1
    _DEFER_WGRAD = [] if on else None


# a weight gradient this big fills the chip on its own, on the 256^2 route
# (~770-880 TF/s) -- inside the grouped launch (128^2 tiles, ~460 TF/s) it
# would run slower: the vocab-sized classifier gradients stay per-layer
GROUP_MAX_MNK = float(os.environ.get("TAM_GROUP_MAX_MNK", str(float(1 << 35))))


def _group_ok(M: int, N: int, K: int) -> bool:
    key = (M, N, K)
    ok = _GROUP_OK.get(key)
    if ok is None:
        ok = bool(_T().gemm_wgrad_grouped_ok(M, N, K)) and float(M) * N * K <= GROUP_MAX_MNK
        _GROUP_OK[key] = ok
    return ok


def defer_problems(probs) -> bool:
    """Defer a layer's weight-gradient problems [(dY, X, w, b, mode), ...]
    into the backward's grouped launch when deferral is on (a model's own
    grouped call, e.g. the LSTM's dW_hh / dW_ih); False: issue them now."""
    if _DEFER_WGRAD is None:
        return False
    for it in probs:
        if any(p[2] is it[2] for p in _DEFER_WGRAD):
            flush_wgrad()            # a second write of the same weight: the pending one first
            break
    for it in probs:
        _DEFER_WGRAD.append(tuple(it))
        _deferred()
    return True


def deferred_count() -> int:
    """Problems deferred so far in this backward (flushed or not)."""
    return _DEFER_COUNT


def _deferred(pending_flush: bool = True) -> None:
    """After appending one deferred problem: count it; flush when a chunk is
    full."""
    global _DEFER_COUNT
    _DEFER_COUNT += 1
    if _DEFER_CHUNK and len(_DEFER_WGRAD) >= _DEFER_CHUNK:
        flush_wgrad()


def flush_wgrad() -> int:
    """Issue every deferred weight gradient as one grouped launch (on the
    weight-gradient stream when one is installed), then signal grad_ready.
    Returns the number of problems flushed."""
    if _DEFER_LNRED:
        lnr = list(_DEFER_LNRED)
        _DEFER_LNRED.clear()
        _T().col_reduce_acc_batch([e[0] for e in lnr], [e[1] for e in lnr], [e[2].grad for e in lnr],
                                  [e[3].grad for e in lnr])
        for _, _, g, b in lnr:
            g.grad_ready()
            b.grad_ready()
    pend = _DEFER_WGRAD
    if not pend:
        return 0
    items = list(pend)
    pend.clear()
    dys = [it[0] for it in items]
    with _OnWgrad(*dys, *[it[1] for it in items]):
        empty = torch.empty(0, dtype=torch.float32, device=dys[0].device)
        # it[5] (when present): the 2-D view of a conv weight's gradient
        _T().gemm_wgrad_grouped(dys, [it[1] for it in items], [it[5] if len(it) > 5 else it[2].grad for it in items],
                                [it[3].grad if it[3] is not None else empty for it in items],
                                [it[4] for it in items])
    for it in items:
        it[2].grad_ready()
        if it[3] is not None:
            it[3].grad_ready()
    return len(items)


# ============================================================ branch streams
# Independent sub-graphs of a model (GNMT: the forward and reverse halves of
# the bidirectional encoder layer; the first decoder layer, which reads only
# the target embedding, vs the whole encoder stack) are issued on their own
# streams. Their per-timestep recurrences are latency-bound (<= 256
# workgroups per kernel), so two of them co-run on the CUs; inside a hipGraph
# capture the fork/join become parallel branches. Autograd runs each
# Function's backward on its forward's stream, so the backward branches
# overlap too. Every gradient buffer has ONE writer stream, and the trainer
# joins all branch streams before the optimizer (Trainer._fwd_bwd). Gangs
# leave them unset: a bucket all-reduce is ordered after the current stream
# only.
_BRANCH_STREAMS: list = []


def set_branch_streams(streams) -> None:
    global _BRANCH_STREAMS
    _BRANCH_STREAMS = list(streams or [])


class on_branch:
    """``with on_branch(i, *inputs):`` issue the block on branch stream ``i``
    (forked from the current stream; no-op when no branch streams are set)."""

    def __init__(self, i: int, *inputs):
        self.s = _BRANCH_STREAMS[i] if i < len(_BRANCH_STREAMS) and inputs[0].is_cuda else None
        self.ts = inputs
        self.ctx = None

    def __enter__(self):
        if self.s is None:
            return self
        self.s.wait_stream(torch.cuda.current_stream(self.ts[0].device))
        for t in self.ts:
            t.record_stream(self.s)        # not recycled by the forking stream meanwhile
        self.ctx = torch.cuda.stream(self.s)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


def join_branch(i: int, *outputs):
    """Order the current stream after branch ``i`` and hand it ``outputs``."""
    if i < len(_BRANCH_STREAMS) and outputs[0].is_cuda:
        cur = torch.cuda.current_stream(outputs[0].device)
        cur.wait_stream(_BRANCH_STREAMS[i])
        for t in outputs:
            t.record_stream(cur)
    return outputs if len(outputs) > 1 else outputs[0]


# ============================================================ Linear
# first gradient write of a step stores (grad_mode); 0: always accumulate
# into the optimizer-zeroed buffer (A/B and the equivalence test)
STORE_GRAD = os.environ.get("TAM_STORE_GRAD", "1") != "0"


def grad_mode(p: Param) -> int:
    """Epilogue mode of a GEMM that writes p's whole gradient: 0 (store) for
    the first write since the last optimizer step (the buffer's content is
    dead: zeroed, or a store_grad param's stale gradient), 1 (accumulate)
    after it. The store skips the fp32 read of C (4 B per weight) and lets the
    optimizer skip zeroing store_grad params (another 4 B). Only the writers
    that call this may write such a param's gradient (a bias / BN / conv
    accumulation into it would be lost); under hipGraph capture the decision
    is taken once, at capture, like every other host-side choice."""
    A = p.arena
    first = p.gw_epoch != A.grad_epoch
    p.gw_epoch = A.grad_epoch
    return 0 if (first and STORE_GRAD) else 1


class _Linear(Function):
    @staticmethod
    def forward(ctx, x, token, w: Param, b: Optional[Param], relu: bool, in_relu: bool,
                mask_own_relu: bool):
        M = x.shape[0]
        out = w.shape[0]
        if x.is_cuda:
            y = torch.empty(M, out, dtype=BF16, device=x.device)
            _T().gemm(x, True, w.w, True, y, 0, b.w if b is not None else None, relu, None, 1.0, False)
        else:
            yf = _cpu_gemm_f32(x, w.w.t())
            if b is not None:
                yf = yf + b.w.float()
            if relu:
                yf = yf.clamp_min(0)
            y = yf.to(BF16)
        ctx.w, ctx.b, ctx.relu, ctx.in_relu, ctx.mask_own = w, b, relu, in_relu, mask_own_relu
        ctx.save_for_backward(x, y if (relu and mask_own_relu) else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        dy = dy.contiguous()
        if y is not None:
            if dy.is_cuda:
                dyr = torch.empty_like(dy)
                _T().relu_backward(dy, y, dyr)
                dy = dyr
            else:
                dy = (dy.float() * (y.float() > 0)).to(BF16)
        dx = None
        deferred = False
        if dy.is_cuda:
            if (_DEFER_WGRAD is not None and x.dim() == 2 and w.grad.is_contiguous()
                    and _group_ok(w.shape[0], w.shape[1], x.shape[0])):
                if any(it[2] is w for it in _DEFER_WGRAD):
                    flush_wgrad()      # a second use of w: its pending write goes first
                # issued by flush_wgrad, AFTER writers that run in between
                # (a tied embedding's scatter-add): only a store_grad weight,
                # which nothing else writes, may store there
                if w.store_grad:
                    mode = grad_mode(w)
                else:
                    w.gw_epoch = w.arena.grad_epoch
                    mode = 1
                _DEFER_WGRAD.append((dy, x, w, b, mode))
                deferred = True
            else:
                if _DEFER_WGRAD is not None and any(it[2] is w for it in _DEFER_WGRAD):
                    # w also has a deferred (possibly store-mode) write pending:
                    # issue it first, or its later store would overwrite this
                    # accumulation
                    flush_wgrad()
                with _OnWgrad(dy, x):
                    # the bias gradient colsum(dy) rides on the weight-gradient
                    # GEMM's own A loads (fused on the igemm route, else a pass)
                    _T().gemm(dy, False, x, False, w.grad, grad_mode(w), None, False, None, 1.0, True,
                              b.grad if b is not None else None)
        if ctx.needs_input_grad[0]:
            if dy.is_cuda:
                dx = torch.empty_like(x)
                wk = weight_kmajor(w)
                if wk is not None:
                    _T().gemm(dy, True, wk, True, dx, 0, None, False, x if ctx.in_relu else None, 1.0, False)
                else:
                    _T().gemm(dy, True, w.w, False, dx, 0, None, False, x if ctx.in_relu else None, 1.0, False)
            else:
                dxf = _cpu_gemm_f32(dy, w.w)
                if ctx.in_relu:
                    dxf = dxf * (x.float() > 0)
                dx = dxf.to(BF16)
        if not dy.is_cuda:
            w.grad += _cpu_gemm_f32(dy.t(), x)
            if b is not None:
                b.grad += dy.float().sum(0)
        if deferred:
            _deferred()
        else:
            w.grad_ready()
            if b is not None:
                b.grad_ready()
        return dx, None, None, None, None, None, None


def linear(x: torch.Tensor, w: Param, b: Optional[Param] = None, relu: bool = False,
           in_relu: bool = False, mask_own_relu: bool = True) -> torch.Tensor:
    """y = x W^T (+b) (relu). x: [..., in] bf16 -> [..., out].

    in_relu: x is a ReLU output; mask the input-gradient by (x > 0).
    mask_own_relu: apply this layer's own ReLU mask in backward (set False when
    the consumer was built with in_relu=True, which already masks).
    """
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    y = _Linear.apply(x2, w.arena.token, w, b, relu, in_relu, mask_own_relu)
    return y.view(*shp[:-1], w.shape[0])


# ============================================================ Conv2d (NHWC)
def _conv_out(h: int, k: int, s: int, p: int, d: int = 1) -> int:
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


# (the BatchNorm-backward reduction of a consumer_masks BN computed in the
# consumer conv's dgrad epilogue measured neutral on ResNet-50 -- 23 of 53
# bn_bwd_reduce launches gone, -127 us, the dgrad convs +165 us -- and its
# model plumbing was removed in round 6; profiles/r6/bn_fold.md)


# relu BNs whose backward applies the ReLU mask itself keep it as 1 bit per
# output (bn_forward ymask) instead of re-reading the bf16 output
BN_RELU_BITMASK = True

# shards of a BatchNorm statistics accumulator (csrc/include/tam/common.h
# BN_SHARDS; the ops check the size): fp64 [BN_SHARDS][2C]
BN_SHARDS = 16


def _bn_sums(ws, C: int, device) -> torch.Tensor:
    """fp64 [BN_SHARDS * 2C] BatchNorm statistics accumulator: the caller's
    zeroed workspace slice, or a fresh zeroed tensor."""
    if ws is not None:
        return ws
    return torch.zeros(BN_SHARDS * 2 * C, dtype=torch.float64, device=device)


class _Conv(Function):
    @staticmethod
    def forward(ctx, x, token, w: Param, b: Optional[Param], stride: int, pad: int, relu: bool,
                in_relu: bool, mask_own_relu: bool, bn_stats=False):
        N, H, W, C = x.shape
        K, R, S, _ = w.shape
        P, Q = _conv_out(H, R, stride, pad), _conv_out(W, S, stride, pad)
        part = None
        if x.is_cuda:
            y = torch.empty(N, P, Q, K, dtype=BF16, device=x.device)
            if bn_stats is not False and bn_stats is not None:
                # BatchNorm sums from the conv epilogue (no stats pass): fp64
                # atomics into the BN's zeroed workspace
                sums = _bn_sums(bn_stats if isinstance(bn_stats, torch.Tensor) else None, K, x.device)
                done = _T().conv_fwd(x, w.w, y, stride, pad, 1, b.w if b is not None else None, relu, sums)
                part = sums if done else None
            else:
                _T().conv_fwd(x, w.w, y, stride, pad, 1, b.w if b is not None else None, relu)
        else:
            yf = F.conv2d(x.float().permute(0, 3, 1, 2), w.w.float().permute(0, 3, 1, 2),
                          b.w.float() if b is not None else None, stride=stride, padding=pad)
            if relu:
                yf = yf.clamp_min(0)
            y = yf.permute(0, 2, 3, 1).contiguous().to(BF16)
        ctx.w, ctx.b, ctx.stride, ctx.pad, ctx.in_relu = w, b, stride, pad, in_relu
        ctx.save_for_backward(x, y if (relu and mask_own_relu) else None)
        ctx.part = part
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        w, b, st, pd = ctx.w, ctx.b, ctx.stride, ctx.pad
        dy = dy.contiguous()
        if y is not None:
            if dy.is_cuda:
                dyr = torch.empty_like(dy)
                _T().relu_backward(dy, y, dyr)
                dy = dyr
            else:
                dy = (dy.float() * (y.float() > 0)).to(BF16)
        dx = None
        deferred = False
        if dy.is_cuda:
            K, R, S, C = w.shape
            Mr = dy.numel() // K
            if (_DEFER_WGRAD is not None and R == 1 and S == 1 and st == 1 and pd == 0 and b is None
                    and w.grad.is_contiguous() and not any(it[2] is w for it in _DEFER_WGRAD)
                    and _group_ok(K, C, Mr)):
                # a 1x1 / stride-1 conv's dW = dY^T X is a plain GEMM over the
                # output pixels: deferred into the backward's grouped launch
                # (K-split there: ResNet-50's are 128..2048 x 128..2048 x
                # 3136..200704), accumulating into the optimizer-zeroed buffer
                w.gw_epoch = w.arena.grad_epoch
                _DEFER_WGRAD.append((dy.view(Mr, K), x.view(Mr, C), w, None, 1, w.grad.view(K, C)))
                deferred = True
            else:
                with _OnWgrad(dy, x) as ow:
                    # the bias gradient colsum(dy) rides on the wgrad kernel's dY reads;
                    # the LDS-heavy patch-staged wgrad only off the side stream
                    # accumulate into the optimizer-zeroed buffer: a store-mode first
                    # write costs a zero pass of dW on the fp32-atomic split paths
                    # (ResNet-50: 29 more zero launches per step when conv weights
                    # were store_grad), the optimizer's bulk zeroing does not
                    _T().conv_wgrad(dy, x, w.grad, st, pd, 1, 1, b.grad if b is not None else None,
                                    ow.s is None)
            if ctx.needs_input_grad[0]:
                dx = torch.empty_like(x)
                wt = getattr(w, "wt", None)
                if wt is not None:       # re-laid once per step (prepare_conv_wt)
                    _T().conv_dgrad_pre(dy, w.w, wt, dx, st, pd, 1, x if ctx.in_relu else None)
                else:
                    wt = torch.empty_like(w.w)
                    _T().conv_dgrad(dy, w.w, wt, dx, st, pd, 1, x if ctx.in_relu else None)
        else:
            xf = x.float().permute(0, 3, 1, 2).requires_grad_(ctx.needs_input_grad[0])
            wf = w.w.float().permute(0, 3, 1, 2).requires_grad_(True)
            with torch.enable_grad():
                yf = F.conv2d(xf, wf, stride=st, padding=pd)
                grads = torch.autograd.grad(yf, [xf, wf] if ctx.needs_input_grad[0] else [wf],
                                            dy.float().permute(0, 3, 1, 2))
            if ctx.needs_input_grad[0]:
                dxf = grads[0].permute(0, 2, 3, 1)
                if ctx.in_relu:
                    dxf = dxf * (x.float() > 0)
                dx = dxf.contiguous().to(BF16)
            w.grad += grads[-1].permute(0, 2, 3, 1)
            if b is not None:
                b.grad += dy.float().sum((0, 1, 2))
        if deferred:
            _deferred()
        else:
            w.grad_ready()
            if b is not None:
                b.grad_ready()
        return dx, None, None, None, None, None, None, None, None, None


# the re-laid weights are first read by the backward's dgrad. A side-stream
# re-lay beside the forward measured slower in hipGraph replay (ResNet-50
# 9.02-9.03 vs 8.88 ms, VGG-16 6.65 vs 6.61-6.62 ms: a fork / join costs more
# than the 60 us launch it hides) and was removed in round 6.


def prepare_conv_wt(params: List[Param]) -> None:
    """Re-lay every conv weight [K,R,S,C] -> [C,R,S,K] (the dgrad operand) in
    ONE launch per step, into per-parameter buffers kept across steps (the
    dgrad then skips its own transpose). Call at the start of the forward:
    the weights are final for the step then. No-op on CPU."""
    if not params or not params[0].w.is_cuda:
        return
    for p in params:
        if getattr(p, "wt", None) is None or p.wt.device != p.w.device:
            p.wt = torch.empty_like(p.w)
    _T().conv_weight_t_batch([p.w for p in params], [p.wt for p in params])



# TAM_KMAJOR_DGRAD=0: the models' input gradients on the KN GEMM, no
# per-step K-major weight copies (A/B)
KMAJOR_DGRAD = os.environ.get("TAM_KMAJOR_DGRAD", "1") != "0"


def prepare_weight_t(params: List[Param]) -> None:
    """K-major copies ``p.wk`` [in, out] of 2-D weights [out, in], all in ONE
    launch (the batched conv-weight re-lay, as 1x1 kernels), for the input
    gradients dX = dY . W: with W K-major they run on the KK GEMM instead of
    the slower KN form (GNMT's LSTM input and classifier gradients, e.g.
    3200 x 2048 x 4096 KN 85 us vs KK 65 us + an 8 us re-lay,
    profiles/r6/kn_vs_kk.json; GNMT step 9.93-9.97 -> 9.73-9.80 ms). Valid for the current optimizer step only
    (``p.wk_epoch``); call at the start of the forward. No-op on CPU."""
    if not params or not params[0].w.is_cuda:
        return
    ws, wts = [], []
    for p in params:
        O, I = p.shape
        if getattr(p, "wk", None) is None or p.wk.device != p.w.device:
            p.wk = torch.empty(I, O, dtype=BF16, device=p.w.device)
        ws.append(p.w.view(O, 1, 1, I))
        wts.append(p.wk)
        p.wk_epoch = p.arena.grad_epoch
    _T().conv_weight_t_batch(ws, wts)


def weight_kmajor(p: Param) -> Optional[torch.Tensor]:
    """p's K-major copy when prepare_weight_t made one for this step."""
    wk = getattr(p, "wk", None)
    return wk if wk is not None and getattr(p, "wk_epoch", None) == p.arena.grad_epoch else None


def conv2d(x: torch.Tensor, w: Param, b: Optional[Param] = None, stride: int = 1, pad: int = 0,
           relu: bool = False, in_relu: bool = False, mask_own_relu: bool = True,
           bn_stats=False) -> torch.Tensor:
    """NHWC conv, weights [K,R,S,C]. ``bn_stats``: the output feeds a
    BatchNorm -- its per-channel sums come from the conv epilogue (where the
    conv path supports it) and ride on the output tensor. True, or the BN's
    zeroed fp64 forward workspace (``BNWorkspace.fwd``) to accumulate into."""
    if not x.is_contiguous():
        x = x.contiguous()
    y = _Conv.apply(x, w.arena.token, w, b, stride, pad, relu, in_relu, mask_own_relu, bn_stats)
    if bn_stats is not False and bn_stats is not None and y.is_cuda and y.grad_fn is not None:
        part = getattr(y.grad_fn, "part", None)
        if part is not None:
            y._tam_bnpart = part
    return y


# ============================================================ BatchNorm (NHWC)
class GradSlot:
    """A second upstream gradient of a BN output, parked by a residual tap
    (``residual_split``) instead of being summed by autograd; the producing
    BN's backward adds it while loading dy (bn_backward ``addend``), so the
    residual-branch sum is never materialised (no separate add kernel)."""

    __slots__ = ("stash",)

    def __init__(self):
        self.stash = None


class _Tap(Function):
    @staticmethod
    def forward(ctx, y, slot: GradSlot):
        ctx.slot = slot
        return y.view_as(y)

    @staticmethod
    def backward(ctx, g):
        if ctx.slot.stash is not None:           # a second tap: fall back to autograd's sum
            return g, None
        ctx.slot.stash = g.contiguous()
        return None, None


def residual_split(y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(y for the main branch, y for a second consumer): a residual tap when
    y's producer is a BN (the sum happens in its backward), else a fan-out
    whose two gradients one launch of ours sums (e.g. the max-pool output
    feeding the first bottleneck's conv1 and its downsample conv)."""
    slot = getattr(y, "_tam_slot", None)
    if not (y.is_cuda and torch.is_grad_enabled() and y.requires_grad):
        return y, y
    if slot is not None:
        return y, _Tap.apply(y, slot)
    return fanout(y, 2)


class _BN(Function):
    @staticmethod
    def forward(ctx, x, res, token, g: Param, b: Param, run_mean, run_var, relu: bool, eps: float,
                momentum: float, training: bool, slot: Optional[GradSlot] = None,
                consumer_masks: bool = False, ws=None):
        C = x.shape[-1]
        # consumer_masks: the only consumer (a conv with in_relu) already zeroes
        # the gradient where y <= 0 in its dgrad epilogue -- the backward here
        # neither re-reads y nor keeps it alive
        bwd_relu = relu and not consumer_masks
        ymask = None
        if x.is_cuda:
            y = torch.empty_like(x)
            if training:
                mean = torch.empty(C, dtype=torch.float32, device=x.device)
                rstd = torch.empty_like(mean)
                if bwd_relu and BN_RELU_BITMASK:
                    # the backward's ReLU mask as 1 bit per output (1/16 of y's bytes)
                    ymask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
                part = getattr(x, "_tam_bnpart", None)
                if part is not None:       # sums accumulated by the producing conv
                    _T().bn_forward(x, res, y, g.master, b.master, run_mean, run_var, mean, rstd, eps,
                                    momentum, relu, part, True, ymask)
                else:
                    _T().bn_forward(x, res, y, g.master, b.master, run_mean, run_var, mean, rstd, eps,
                                    momentum, relu, ws.fwd if ws is not None else None, False, ymask)
            else:
                rstd_i = torch.rsqrt(run_var + eps)
                scale = g.master * rstd_i
                shift = b.master - run_mean * scale
                mean, rstd = run_mean, rstd_i
                y = _bn_infer_gpu(x, res, scale, shift, relu)
        else:
            xf = x.float().reshape(-1, C)
            if training:
                mean = xf.mean(0)
                var = xf.var(0, unbiased=False)
                if run_mean is not None:
                    n = xf.shape[0]
                    run_mean.mul_(1 - momentum).add_(momentum * mean)
                    run_var.mul_(1 - momentum).add_(momentum * var * n / max(n - 1, 1))
            else:
                mean, var = run_mean, run_var
            rstd = torch.rsqrt(var + eps)
            yf = (xf - mean) * rstd * g.master + b.master
            if res is not None:
                yf = yf + res.float().reshape(-1, C)
            if relu:
                yf = yf.clamp_min(0)
            y = yf.reshape(x.shape).to(BF16)
        ctx.g, ctx.b, ctx.relu, ctx.has_res = g, b, bwd_relu, res is not None
        ctx.bitmask = ymask is not None
        ctx.slot = slot
        ctx.bws = ws.bwd if ws is not None else None
        ctx.save_for_backward(x, (ymask if ymask is not None else y) if bwd_relu else None, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd = ctx.saved_tensors
        g, b = ctx.g, ctx.b
        dy = dy.contiguous()
        C = x.shape[-1]
        add = None
        if ctx.slot is not None:
            add, ctx.slot.stash = ctx.slot.stash, None
        if dy.is_cuda:
            dx = torch.empty_like(x)
            dres = torch.empty_like(x) if ctx.has_res and (ctx.relu or add is not None) else None
            if ctx.bitmask:
                _T().bn_backward(dy, None, x, mean, rstd, g.master, dx, dres, g.grad, b.grad, ctx.relu, add,
                                 ctx.bws, False, y)
            else:
                _T().bn_backward(dy, y, x, mean, rstd, g.master, dx, dres, g.grad, b.grad, ctx.relu, add,
                                 ctx.bws, False)
            if ctx.has_res and dres is None:
                dres = dy
        else:
            dyf = dy.float().reshape(-1, C)
            if add is not None:
                dyf = dyf + add.float().reshape(-1, C)
            if ctx.relu:
                dyf = dyf * (y.float().reshape(-1, C) > 0)
            xh = (x.float().reshape(-1, C) - mean) * rstd
            M = dyf.shape[0]
            sdy = dyf.sum(0)
            sdyx = (dyf * xh).sum(0)
            g.grad += sdyx
            b.grad += sdy
            dxf = g.master * rstd * (dyf - sdy / M - xh * sdyx / M)
            dx = dxf.reshape(x.shape).to(BF16)
            dres = dyf.reshape(x.shape).to(BF16) if ctx.has_res else None
        g.grad_ready()
        b.grad_ready()
        return dx, dres, None, None, None, None, None, None, None, None, None, None, None, None


def _bn_infer_gpu(x, res, scale, shift, relu):
    # inference-only path (not on the training hot path)
    yf = x.float() * scale + shift
    if res is not None:
        yf = yf + res.float()
    if relu:
        yf = yf.clamp_min(0)
    return yf.to(BF16)


class BNWorkspace:
    """fp64 statistics accumulators of one BatchNorm layer: ``fwd``
    [BN_SHARDS][2C] (sum | sum of squares of x) and ``bwd`` [BN_SHARDS][2C]
    (sum(d) | sum(d * xhat)),
    slices of one model-wide buffer that the model zeroes ONCE per training
    step (``zero_()``, a single memset node in the captured graph). The
    producing conv's epilogue, or the BN's own reduction pass, accumulates
    into them with device-scope atomics; the apply passes derive the
    per-channel coefficients in their prologue (no finalize launches)."""

    def __init__(self, buf: torch.Tensor, off: int, C: int):
        n = BN_SHARDS * 2 * C
        self.fwd = buf[off:off + n]
        self.bwd = buf[off + n:off + 2 * n]


def bn_workspaces(channels: dict, device) -> Tuple[torch.Tensor, dict]:
    """One zero-initialised fp64 buffer for every BN of a model
    ({key: C} -> (buffer, {key: BNWorkspace}))."""
    per = {k: 2 * BN_SHARDS * 2 * c for k, c in channels.items()}
    buf = torch.zeros(max(sum(per.values()), 1), dtype=torch.float64, device=device)
    out, off = {}, 0
    for k, c in channels.items():
        out[k] = BNWorkspace(buf, off, c)
        off += per[k]
    return buf, out


def batchnorm(x: torch.Tensor, g: Param, b: Param, run_mean: Optional[torch.Tensor] = None,
              run_var: Optional[torch.Tensor] = None, relu: bool = False,
              residual: Optional[torch.Tensor] = None, eps: float = 1e-5, momentum: float = 0.1,
              training: bool = True, consumer_masks: bool = False,
              ws: Optional[BNWorkspace] = None) -> torch.Tensor:
    """y = relu(BN(x) + residual) over the last (channel) dim of an NHWC tensor.

    ``consumer_masks``: y has exactly one consumer, a ``conv2d(..., in_relu=True)``
    whose dgrad applies the ReLU backward mask (reading y once there instead of
    twice in this BN's backward passes).
    ``ws``: this layer's statistics workspace, zeroed since its last use
    (None: zeroed temporaries per call)."""
    if not x.is_contiguous():
        x = x.contiguous()
    if residual is not None and not residual.is_contiguous():
        residual = residual.contiguous()
    slot = GradSlot() if (x.is_cuda and training and torch.is_grad_enabled()) else None
    y = _BN.apply(x, residual, g.arena.token, g, b, run_mean, run_var, relu, eps, momentum,
                  training, slot, consumer_masks and relu and residual is None,
                  ws if (x.is_cuda and training) else None)
    if slot is not None:
        y._tam_slot = slot
    return y


# ============================================================ LayerNorm
# (a side-stream column reduce of the LN weight gradients beside the next
# input-gradient GEMM measured much slower in hipGraph replay -- Transformer
# 5.49-5.57 vs 5.18 ms, 32 fork / join pairs per step -- and was removed in
# round 6; the reduces are batched into the backward's flush instead)


# while weight gradients are deferred (trainer group_wgrad), a LayerNorm's
# dgamma / dbeta column reduce is deferred too and every one of the backward
# runs in ONE batched launch at the flush (Transformer-base: 32 reduce
# launches per step -> 1); TAM_LN_DEFER=0 for A/B
LN_DEFER = os.environ.get("TAM_LN_DEFER", "1") != "0"
_DEFER_LNRED: list = []
# (deferring slab-split conv weight-gradient reduces into the same flush
# measured neutral in graph replay and held the DDP buckets back; removed in
# round 6)


def _ln_backward(dy, x, g: Param, b: Param, mean, rstd, dx, addend=None) -> bool:
    """LN backward; returns True when dgamma / dbeta were deferred to the
    flush (their grad_ready() then comes from flush_wgrad)."""
    deferred = _DEFER_WGRAD is not None and LN_DEFER
    if not deferred:
        _T().ln_backward(dy, x, g.master, mean, rstd, dx, g.grad, b.grad, addend)
        return False
    D = x.shape[-1]
    ws = torch.empty(_LN_MAX_BLOCKS * 2 * D, dtype=torch.float32, device=x.device)
    nblk = _T().ln_backward_split(dy, x, g.master, mean, rstd, dx, ws, addend)
    _DEFER_LNRED.append((ws, nblk, g, b))
    return True


_LN_MAX_BLOCKS = 512        # csrc/include/tam/kernels.h LN_MAX_BLOCKS


class _LN(Function):
    @staticmethod
    def forward(ctx, x, token, g: Param, b: Param, eps: float):
        D = x.shape[-1]
        rows = x.numel() // D
        if x.is_cuda:
            y = torch.empty_like(x)
            mean = torch.empty(rows, dtype=torch.float32, device=x.device)
            rstd = torch.empty_like(mean)
            _T().ln_forward(x, g.master, b.master, y, mean, rstd, eps)
        else:
            xf = x.float().reshape(rows, D)
            mean = xf.mean(1)
            rstd = torch.rsqrt(xf.var(1, unbiased=False) + eps)
            y = (((xf - mean[:, None]) * rstd[:, None]) * g.master + b.master).reshape(x.shape).to(BF16)
        ctx.g, ctx.b = g, b
        ctx.save_for_backward(x, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        g, b = ctx.g, ctx.b
        dy = dy.contiguous()
        D = x.shape[-1]
        if dy.is_cuda:
            dx = torch.empty_like(x)
            if _ln_backward(dy, x, g, b, mean, rstd, dx):
                return dx, None, None, None, None
        else:
            rows = x.numel() // D
            xh = (x.float().reshape(rows, D) - mean[:, None]) * rstd[:, None]
            dyf = dy.float().reshape(rows, D)
            g.grad += (dyf * xh).sum(0)
            b.grad += dyf.sum(0)
            gd = dyf * g.master
            dxf = rstd[:, None] * (gd - gd.mean(1, keepdim=True) - xh * (gd * xh).mean(1, keepdim=True))
            dx = dxf.reshape(x.shape).to(BF16)
        g.grad_ready()
        b.grad_ready()
        return dx, None, None, None, None


def layernorm(x: torch.Tensor, g: Param, b: Param, eps: float = 1e-5) -> torch.Tensor:
    if not x.is_contiguous():
        x = x.contiguous()
    return _LN.apply(x, g.arena.token, g, b, eps)


class _LNSkip(_LN):
    """Pre-LN residual tap: returns (x, LN(x)). The residual stream leaves
    through this Function instead of being consumed twice, so autograd does
    not sum the two incoming gradients with an extra elementwise kernel: the
    LN backward kernel adds the skip gradient in its epilogue."""

    @staticmethod
    def forward(ctx, x, token, g: Param, b: Param, eps: float):
        # an unused skip output (the stack's final LN) arrives as None, not
        # as a zero-filled tensor autograd would launch a fill kernel for
        ctx.set_materialize_grads(False)
        y = _LN.forward(ctx, x, token, g, b, eps)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, dskip, dy):
        x, mean, rstd = ctx.saved_tensors
        g, b = ctx.g, ctx.b
        if dy is None:
            return dskip, None, None, None, None
        dy = dy.contiguous()
        if dy.is_cuda:
            dx = torch.empty_like(x)
            if not _ln_backward(dy, x, g, b, mean, rstd, dx, dskip.contiguous() if dskip is not None else None):
                g.grad_ready()
                b.grad_ready()
            return dx, None, None, None, None
        dx = _LN.backward(ctx, dy)[0]
        if dskip is not None:
            dx = (dx.float() + dskip.float()).to(BF16)
        return dx, None, None, None, None


def layernorm_skip(x: torch.Tensor, g: Param, b: Param, eps: float = 1e-5):
    """(x, layernorm(x)) for ``x + f(layernorm(x))`` blocks; see _LNSkip."""
    if not x.is_contiguous():
        x = x.contiguous()
    return _LNSkip.apply(x, g.arena.token, g, b, eps)


class _AddLNSkip(Function):
    """(s, LN(s)) with s = x + r: the residual add of a pre-LN block fused
    into the next LayerNorm's forward (one kernel writes s and LN(s)); the
    backward is _LNSkip's (dskip summed in the LN backward kernel) and hands
    ds to both addends."""

    @staticmethod
    def forward(ctx, x, r, token, g: Param, b: Param, eps: float):
        ctx.set_materialize_grads(False)         # see _LNSkip.forward
        D = x.shape[-1]
        rows = x.numel() // D
        if x.is_cuda:
            sm = torch.empty_like(x)
            y = torch.empty_like(x)
            mean = torch.empty(rows, dtype=torch.float32, device=x.device)
            rstd = torch.empty_like(mean)
            _T().ln_forward(x, g.master, b.master, y, mean, rstd, eps, r, sm)
        else:
            sm = (x.float() + r.float()).to(BF16)
            sf = sm.float().reshape(rows, D)
            mean = sf.mean(1)
            rstd = torch.rsqrt(sf.var(1, unbiased=False) + eps)
            y = (((sf - mean[:, None]) * rstd[:, None]) * g.master + b.master).reshape(x.shape).to(BF16)
        ctx.g, ctx.b = g, b
        ctx.save_for_backward(sm, mean, rstd)
        return sm, y

    @staticmethod
    def backward(ctx, dskip, dy):
        ds = _LNSkip.backward(ctx, dskip, dy)[0]
        return ds, ds, None, None, None, None


def add_layernorm_skip(x: torch.Tensor, r: torch.Tensor, g: Param, b: Param, eps: float = 1e-5):
    """(x + r, layernorm(x + r)) in one kernel: ``layernorm_skip(add(x, r))``."""
    if not x.is_contiguous():
        x = x.contiguous()
    if not r.is_contiguous():
        r = r.contiguous()
    return _AddLNSkip.apply(x, r, g.arena.token, g, b, eps)


# ============================================================ pooling
class _MaxPool(Function):
    @staticmethod
    def forward(ctx, x, k: int, s: int, p: int):
        N, H, W, C = x.shape
        P, Q = _conv_out(H, k, s, p), _conv_out(W, k, s, p)
        if x.is_cuda:
            y = torch.empty(N, P, Q, C, dtype=BF16, device=x.device)
            idx = torch.empty(N, P, Q, C, dtype=torch.uint8, device=x.device)
            _T().maxpool_forward(x, y, idx, k, k, s, p)
            ctx.save_for_backward(idx)
        else:
            y = F.max_pool2d(x.float().permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1).contiguous().to(BF16)
            ctx.save_for_backward(x)
        ctx.cfg = (k, s, p, x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        (saved,) = ctx.saved_tensors
        k, s, p, shape = ctx.cfg
        dy = dy.contiguous()
        if dy.is_cuda:
            dx = torch.empty(shape, dtype=BF16, device=dy.device)
            _T().maxpool_backward(dy, saved, dx, k, k, s, p)
        else:
            # overlapping windows (3x3/s2) route several outputs to one input:
            # the gradient must SUM them (max_unpool2d would overwrite)
            xf = saved.float().permute(0, 3, 1, 2).requires_grad_(True)
            with torch.enable_grad():
                yf = F.max_pool2d(xf, k, s, p)
                (g,) = torch.autograd.grad(yf, [xf], dy.float().permute(0, 3, 1, 2))
            dx = g.permute(0, 2, 3, 1).contiguous().to(BF16)
        return dx, None, None, None


def maxpool2d(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    return _MaxPool.apply(x.contiguous(), k, s, p)


class _AvgPool(Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        if x.is_cuda:
            y = torch.empty(N, C, dtype=BF16, device=x.device)
            _T().avgpool_forward(x, y)
        else:
            y = x.float().mean((1, 2)).to(BF16)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        dy = dy.contiguous()
        if dy.is_cuda:
            dx = torch.empty(ctx.shape, dtype=BF16, device=dy.device)
            _T().avgpool_backward(dy, dx)
        else:
            dx = (dy.float()[:, None, None, :] / (H * W)).expand(N, H, W, C).contiguous().to(BF16)
        return dx


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    return _AvgPool.apply(x.contiguous())


# ============================================================ loss
def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0,
                 ignore_index: Optional[int] = -100,
                 normalizer: Optional[int] = None,
                 labels_time_major: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused softmax cross-entropy. Returns (mean loss, dlogits) WITHOUT autograd:
    the loss is the graph sink, so the training step calls
    ``logits.backward(dlogits)`` directly (no extra scale pass over the logits).

    ``normalizer``: number of non-ignored rows when known statically (keeps the
    step free of host syncs, i.e. capturable in a hipGraph); otherwise counted.
    ``labels_time_major``: logits are [T,B,V] while labels stay [B,T] -- the
    kernel reads label (b, t) for logits row t * B + b (no transposed copy).
    The mean loss is one reduction kernel of ours (no torch reduce / scale).
    """
    V = logits.shape[-1]
    l2 = logits.reshape(-1, V).contiguous()
    rows = l2.shape[0]
    tm_b = labels.shape[0] if labels_time_major else 0
    ign = ignore_index if ignore_index is not None else -(1 << 62)
    if normalizer is None:
        normalizer = max(1, int((labels != ign).sum().item()))
    n = normalizer
    if l2.is_cuda:
        lab = labels.reshape(-1).contiguous()
        loss_rows = torch.empty(rows, dtype=torch.float32, device=l2.device)
        dlog = torch.empty_like(l2)
        _T().softmax_xent(l2.detach(), lab, dlog, loss_rows, smoothing, 1.0 / n, ign, tm_b)
        loss = torch.empty((), dtype=torch.float32, device=l2.device)
        _T().sum_scale(loss_rows, loss, 1.0 / n)
        return loss, dlog.view(logits.shape)
    lab = (labels.t() if labels_time_major else labels).reshape(-1)
    lf = l2.detach().float()
    logp = torch.log_softmax(lf, -1)
    valid = (lab != ign)
    safe = torch.where(valid, lab, torch.zeros_like(lab))
    nll = -logp.gather(1, safe[:, None])[:, 0]
    smooth = -logp.mean(1)
    lrow = ((1 - smoothing) * nll + smoothing * smooth) * valid
    loss = lrow.sum() / n
    p = logp.exp()
    tgt = torch.zeros_like(p).scatter_(1, safe[:, None], 1.0) * (1 - smoothing) + smoothing / V
    dlog = ((p - tgt) * valid[:, None] / n).to(BF16)
    return loss, dlog.view(logits.shape)


# ============================================================ embedding
class _Embed(Function):
    """time_major: ids [B,S] -> out [S,B,D], the kernel reading ids (b, s) for
    row s * B + b (no transposed copy of the ids, forward or backward)."""

    @staticmethod
    def forward(ctx, ids, token, table: Param, scale: float, time_major: bool = False, pos=None):
        D = table.shape[1]
        tm_b = ids.shape[0] if time_major else 0
        oshape = (ids.shape[1], ids.shape[0], D) if time_major else (*ids.shape, D)
        flat = ids.reshape(-1).contiguous()
        if flat.is_cuda:
            out = torch.empty(flat.numel(), D, dtype=BF16, device=flat.device)
            _T().embedding_forward(table.w, flat, out, scale, tm_b, pos)
        else:
            if time_major:
                flat = ids.t().reshape(-1)
            out = table.w.float()[flat] * scale
            if pos is not None:
                # bf16 rounding of the scaled row first, as the separate add did
                out = out.to(BF16).float().view(*oshape) + (pos.float()[:, None] if time_major else pos.float())
            out = out.to(BF16)
        ctx.table, ctx.scale, ctx.tm_b = table, scale, tm_b
        ctx.save_for_backward(flat)
        return out.view(*oshape)

    @staticmethod
    def backward(ctx, dout):
        (flat,) = ctx.saved_tensors
        t = ctx.table
        d2 = dout.reshape(-1, t.shape[1]).contiguous()
        t.gw_epoch = t.arena.grad_epoch       # written (accumulated) this step: see grad_mode
        if d2.is_cuda:
            with _OnWgrad(d2, flat):           # the table may be tied to a projection
                _T().embedding_backward(d2, flat, t.grad, ctx.scale, ctx.tm_b)
        else:
            t.grad.index_add_(0, flat, d2.float() * ctx.scale)
        t.grad_ready()
        return None, None, None, None, None, None


def embedding(ids: torch.Tensor, table: Param, scale: float = 1.0, time_major: bool = False,
              pos: Optional[torch.Tensor] = None) -> torch.Tensor:
    """table[ids] * scale (+ pos[position], a constant [S][D] table added in
    the same kernel)."""
    return _Embed.apply(ids, table.arena.token, table, scale, time_major, pos)


# ============================================================ attention
def _attn_ref(q, k, v, causal, scale, kv_len):
    # q [B,Sq,H,64], k/v [B,Sk,H,64] -> o [B,Sq,H,64], lse [B,H,Sq]
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) * scale
    Sq, Sk = s.shape[-2], s.shape[-1]
    mask = torch.zeros(Sq, Sk, dtype=torch.bool, device=s.device)
    if causal:
        mask = torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device), 1)
    s = s.masked_fill(mask, float("-inf"))
    if kv_len is not None:
        km = torch.arange(Sk, device=s.device)[None, :] >= kv_len[:, None].to(s.device)
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None])
    o = (p @ vf).permute(0, 2, 1, 3)
    return o, lse


class _Attn(Function):
    """q_src: [B,Sq,nq*H*64], kv_src: [B,Sk,nkv*H*64]; q at slot q_slot of q_src,
    k / v at slots k_slot / v_slot of kv_src (self-attention passes the same
    packed qkv tensor for both, slots 0/1/2). Gradients come back packed."""

    @staticmethod
    def forward(ctx, q_src, kv_src, H: int, q_slot: int, nq: int, k_slot: int, v_slot: int,
                nkv: int, causal: bool, kv_len, kv_hold=None, tm: bool = False):
        # tm: q_src / kv_src / the output are time-major [S,B,.] (GNMT's
        # recurrent layout); the kernels take batch and token strides, so the
        # [B,S,H,64] views are transposes and no layout copy is made
        same = q_src is kv_src
        ctx.tm = tm
        # kv_hold: several attention calls read different slots of ONE packed
        # K/V tensor (the decoder's batched cross-attention projection); they
        # write their slots into one shared gradient buffer and only the call
        # that ran first (backward runs last) returns it -- no zero-fill, no
        # autograd sum of per-layer full-size gradients
        ctx.kv_hold = kv_hold
        ctx.kv_idx = None
        if kv_hold is not None:
            ctx.kv_idx = kv_hold["n"]
            kv_hold["n"] += 1
        qv, kvv, B, Sq, Sk = _attn_views(q_src, kv_src, H, nq, nkv, q_slot, tm)
        kv_, vv = kvv[:, :, k_slot], kvv[:, :, v_slot]
        scale = 1.0 / math.sqrt(64)
        if q_src.is_cuda:
            ob = torch.empty((Sq, B, H, 64) if tm else (B, Sq, H, 64), dtype=BF16, device=q_src.device)
            o = ob.transpose(0, 1) if tm else ob
            lse = torch.empty(B, H, Sq, dtype=torch.float32, device=q_src.device)
            _T().attn_forward(qv, kv_, vv, o, lse, causal, scale, kv_len)
        else:
            of, lse = _attn_ref(qv, kv_, vv, causal, scale, kv_len)
            ob = (of.transpose(0, 1) if tm else of).to(BF16).contiguous()
        ctx.cfg = (same, H, q_slot, nq, k_slot, v_slot, nkv, causal, scale)
        ctx.save_for_backward(q_src, kv_src, ob, lse, kv_len)
        return ob.view(Sq, B, H * 64) if tm else ob.view(B, Sq, H * 64)

    @staticmethod
    def backward(ctx, do):
        q_src, kv_src, ob, lse, kv_len = ctx.saved_tensors
        same, H, q_slot, nq, k_slot, v_slot, nkv, causal, scale = ctx.cfg
        tm = ctx.tm
        qv, kvv, B, Sq, Sk = _attn_views(q_src, kv_src, H, nq, nkv, q_slot, tm)
        if tm:
            o = ob.transpose(0, 1)
            do = do.contiguous().view(Sq, B, H, 64).transpose(0, 1)
        else:
            o = ob
            do = do.contiguous().view(B, Sq, H, 64)
        alloc = torch.empty_like if q_src.is_cuda else torch.zeros_like
        dq_src = alloc(q_src)
        hold = ctx.kv_hold
        if hold is not None:
            if hold.get("buf") is None:
                hold["buf"] = alloc(kv_src)
            dkv_src = hold["buf"]
        else:
            dkv_src = dq_src if same else alloc(kv_src)
        dqv, dkvv, _, _, _ = _attn_views(dq_src, dkv_src, H, nq, nkv, q_slot, tm)
        if q_src.is_cuda:
            dq_acc = torch.empty(B, Sq, H, 64, dtype=torch.float32, device=q_src.device)
            delta = torch.empty(B, H, Sq, dtype=torch.float32, device=q_src.device)
            _T().attn_backward(qv, kvv[:, :, k_slot], kvv[:, :, v_slot], o, do, lse, dqv,
                               dkvv[:, :, k_slot], dkvv[:, :, v_slot], dq_acc, delta, causal, scale,
                               kv_len)
        else:
            qf = qv.float().requires_grad_(True)
            kf = kvv[:, :, k_slot].float().requires_grad_(True)
            vf = kvv[:, :, v_slot].float().requires_grad_(True)
            with torch.enable_grad():
                of, _ = _attn_ref(qf, kf, vf, causal, scale, kv_len)
                gq, gk, gv = torch.autograd.grad(of, [qf, kf, vf], do.float())
            dqv.copy_(gq.to(BF16))
            dkvv[:, :, k_slot].copy_(gk.to(BF16))
            dkvv[:, :, v_slot].copy_(gv.to(BF16))
        if same:
            return dq_src, None, None, None, None, None, None, None, None, None, None, None
        if hold is not None and ctx.kv_idx != 0:
            dkv_src = None                 # slots written; the first caller returns the buffer
        return dq_src, dkv_src, None, None, None, None, None, None, None, None, None, None


def _attn_views(q_src, kv_src, H, nq, nkv, q_slot, tm):
    """[B,S,H,64] views of the packed q / kv sources (transposes of the
    time-major tensors when tm) and (B, Sq, Sk)."""
    if tm:
        Sq, B, _ = q_src.shape
        Sk = kv_src.shape[0]
        qv = q_src.view(Sq, B, nq, H, 64)[:, :, q_slot].transpose(0, 1)
        kvv = kv_src.view(Sk, B, nkv, H, 64).transpose(0, 1)
    else:
        B, Sq, _ = q_src.shape
        Sk = kv_src.shape[1]
        qv = q_src.view(B, Sq, nq, H, 64)[:, :, q_slot]
        kvv = kv_src.view(B, Sk, nkv, H, 64)
    return qv, kvv, B, Sq, Sk


def self_attention(qkv: torch.Tensor, heads: int, causal: bool = False,
                   kv_len: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv: [B,S,3*H*64] packed projection output -> [B,S,H*64]."""
    qkv = qkv.contiguous()
    return _Attn.apply(qkv, qkv, heads, 0, 3, 1, 2, 3, causal, kv_len, None)


def cross_attention(q: torch.Tensor, kv: torch.Tensor, heads: int,
                    kv_len: Optional[torch.Tensor] = None, k_slot: int = 0, v_slot: int = 1,
                    nkv: int = 2, kv_hold: Optional[dict] = None, time_major: bool = False) -> torch.Tensor:
    """q: [B,Sq,H*64], kv: [B,Sk,nkv*H*64] (K at slot k_slot, V at v_slot)
    -> [B,Sq,H*64]; time_major: q [Sq,B,.], kv [Sk,B,.] -> [Sq,B,H*64] with
    no layout copies. Calls sharing one packed kv pass the same ``kv_hold``
    dict (``{"n": 0}``, fresh per forward); see _Attn."""
    if time_major:
        q, kv = q.contiguous(), kv.contiguous()
    return _Attn.apply(q, kv, heads, 0, 1, k_slot, v_slot, nkv, False, kv_len, kv_hold, time_major)


# ============================================================ residual add
class _Add(Function):
    @staticmethod
    def forward(ctx, a, b):
        if a.is_cuda and a.numel() % 8 == 0:
            y = torch.empty_like(a)
            _T().add(a.contiguous(), b.contiguous(), y)
            return y
        return (a.float() + b.float()).to(BF16)

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return _Add.apply(a, b)


# ======================================== last-dim concat and gradient fan-in
def _rows_ok(*ts) -> bool:
    return all(t.is_cuda and t.dtype == BF16 and t.size(-1) % 8 == 0 and t.stride(-1) == 1 for t in ts)


class _Cat2(Function):
    """[..., Ca] ++ [..., Cb] -> [..., Ca+Cb] in ONE launch of ours (rows_sum:
    a copy job per part); the backward hands out the two column slices of
    the gradient as views (consumers read them at their row pitch)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.ca = a.shape[-1]
        if _rows_ok(a, b):
            a, b = a.contiguous(), b.contiguous()
            out = torch.empty(*a.shape[:-1], a.shape[-1] + b.shape[-1], dtype=BF16, device=a.device)
            _T().rows_sum([out[..., :ctx.ca], out[..., ctx.ca:]], [a, b], [1, 1])
            return out
        return torch.cat([a, b], -1)

    @staticmethod
    def backward(ctx, dy):
        return dy[..., :ctx.ca], dy[..., ctx.ca:]


def cat2(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return _Cat2.apply(a, b)


class _Fanout(Function):
    """x used by n consumers: n aliases whose gradients are summed by ONE
    launch of ours (rows_sum, up to 4 pitched inputs) instead of autograd's
    pairwise accumulation adds."""

    @staticmethod
    def forward(ctx, x, n: int):
        ctx.n = n
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *gs):
        gs = [g for g in gs if g is not None]
        if not gs:
            return None, None
        if len(gs) == 1:
            return gs[0], None
        if len(gs) <= 4 and _rows_ok(*gs):
            out = torch.empty(gs[0].shape, dtype=BF16, device=gs[0].device)
            _T().rows_sum([out], gs, [len(gs)])
            return out, None
        acc = gs[0].float()
        for g in gs[1:]:
            acc = acc + g.float()
        return acc.to(gs[0].dtype), None


def fanout(x: torch.Tensor, n: int) -> Tuple[torch.Tensor, ...]:
    return _Fanout.apply(x, n)
