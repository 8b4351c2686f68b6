"""GNMT-style LSTM seq2seq (Wu et al. 2016, as in the MLPerf GNMT reference:
hidden 1024, 4 encoder layers with a bidirectional first layer and residual
connections from layer 3, 4 decoder layers, attention from the first decoder
layer's output fed to every later layer) on the tiresias_amd kernels.

Attention is multi-head scaled dot-product (16 heads x 64) so it runs on the
flash-attention kernel; training uses teacher forcing, so the first decoder
layer runs over the whole target sequence before attention (exactly GNMT's
data flow).

The LSTM layer is one autograd Function over the whole sequence:
  * the input projection X W_ih^T + b for ALL timesteps is one MFMA GEMM
    (fp32 gate pre-activations);
  * per step: h_{t-1} W_hh^T accumulated in place into that step's gate slice
    (GEMM epilogue mode=accumulate) + the fused cell kernel;
  * backward per step: fused cell backward, dh_{t-1} += dG_t W_hh accumulated
    in place; the weight gradients are two large GEMMs over all timesteps.
The per-step loop is launch-bound; on MI355X both recurrences run as ONE
persistent kernel per layer-direction (lstm.hip, grid barrier per timestep,
W_hh slices resident in VGPRs), the per-step path remaining the fallback.
"""
from __future__ import annotations

import os

import torch
from torch.autograd import Function

from ..ops import _lib
from ..ops import functional as Fx
from ..ops.arena import Arena, Param

BF16 = torch.bfloat16


def _T():
    return _lib.ops()


FUSED_STEP = False
# whole-sequence persistent recurrence kernels (lstm.hip: lstm_seq_forward /
# lstm_seq_backward): one launch per layer-direction per pass instead of two
# per timestep; they decline (return False) for shapes / residency they do not
# cover and the per-step path runs
PERSIST = True
# LSTM weight gradients (dW_hh, dW_ih, the bias column sums) of a layer as
# one grouped launch (csrc/kernels/gemm_grouped.hip) instead of two routed
# GEMMs with split-K slab reduces + a column-sum pass; 0: the per-GEMM path
LSTM_GROUPED_WGRAD = os.environ.get("TAM_LSTM_GROUPED", "1") != "0"
# ...and, when the trainer defers weight gradients (ModelSpec.group_wgrad),
# every layer's problems join the backward's ONE grouped launch instead of
# one launch per layer (TAM_LSTM_DEFER=0: per-layer launches, A/B)
LSTM_DEFER_WGRAD = os.environ.get("TAM_LSTM_DEFER", "1") != "0"
_SYNCS: list = []          # recent barrier/error words (tests read the error flags)


def _sync_words(B: int) -> int:
    return 32 * (4 * (B // 16) + 1)


def _sync(dev, B: int, m=None):
    """(sync words, zeroed) of one persistent launch: [0] error flag, up to 4
    arrival counters per batch tile (own 128-B line each). A slice of the
    model's per-step pool (zeroed by ONE fill at the start of the forward,
    GNMT.forward) when one is left, else a fresh buffer the kernel launcher
    zeroes (stream-ordered). Only buffers of launches that ran are kept for
    persist_errors (_ran)."""
    pool = getattr(m, "_sync_pool", None)
    n = _sync_words(B)
    if pool is not None and m._sync_next + n <= pool.numel() and m._sync_B == B:
        t = pool[m._sync_next:m._sync_next + n]
        m._sync_next += n
        return t, True
    return torch.empty(n, dtype=torch.int32, device=dev), False


def _ran(ok: bool, t: torch.Tensor) -> bool:
    if ok:
        _SYNCS.append(t)
        del _SYNCS[:-64]
    return ok


def persist_errors() -> int:
    """Number of recent persistent launches whose grid barrier timed out."""
    return sum(int(t[0].item()) for t in _SYNCS)


class PersistTimeout(RuntimeError):
    """A persistent LSTM grid barrier timed out during the last round's
    steps: those steps computed on hidden states / gradients that had not
    arrived. Raised by ``check_device_errors`` after the round's
    synchronize; the model has already switched to the per-step path."""


def device_timeouts(reset: bool = True) -> int:
    """Sticky device-wide count of persistent-barrier timeouts since the last
    reset (lstm.hip ``g_pl_timeouts``). Host read: call after a synchronize
    (the worker does, once per round -- never per step)."""
    return int(_T().lstm_persist_timeouts(reset))


class _LSTMLayer(Function):
    @staticmethod
    def forward(ctx, x, token, w_ih: Param, w_hh: Param, b: Param, reverse: bool, m=None):
        # m: the owning model (GNMT) -- its persist flag, its own timeout
        # word (err) and its co-residency rule (residency) go with every
        # persistent launch; None: persistent with the process defaults
        persist = (m.persist and not m.shared) if m is not None else True
        T, B, I = x.shape
        Hd = w_hh.shape[1]
        dev = x.device
        x2 = x.reshape(T * B, I)
        G = torch.empty(T * B, 4 * Hd, dtype=torch.float32, device=dev)
        Hs = torch.empty(T, B, Hd, dtype=BF16, device=dev)
        Cs = torch.empty(T, B, Hd, dtype=torch.float32, device=dev)
        act = torch.empty(T, B, 5 * Hd, dtype=torch.float32, device=dev)
        steps = range(T - 1, -1, -1) if reverse else range(T)
        if dev.type == "cuda":
            _T().gemm(x2, True, w_ih.w, True, G, 0, b.w, False, None, 1.0, False)
            Gv = G.view(T, B, 4 * Hd)
            sy, zeroed = _sync(dev, B, m)
            ran = PERSIST and persist and _ran(_T().lstm_seq_forward(Gv, w_hh.w, Hs, Cs, act, reverse, sy,
                                                                     *_pl_args(m), zeroed), sy)
            steps = [] if ran else steps
            prev = None
            # the fused per-timestep kernel (lstm_step_forward) ties GEMM + cell +
            # launch boundary on MI355X (12.8 us vs 8.4 + 2.8 us: its 4-units-per-WG
            # split re-reads h_{t-1} in every CU, 4x the split-K GEMM's L2 traffic),
            # so it is opt-in
            fused = FUSED_STEP and B % 16 == 0 and Hd % 256 == 0
            for t in steps:
                if fused:
                    # one launch per timestep: recurrent MFMA GEMM + cell (lstm.hip)
                    _T().lstm_step_forward(Gv[t], w_hh.w, Hs[prev] if prev is not None else None,
                                           Cs[prev] if prev is not None else None, Cs[t], Hs[t], act[t])
                else:
                    if prev is not None:
                        _T().gemm(Hs[prev], True, w_hh.w, True, Gv[t], 1, None, False, None, 1.0, True)
                    _T().lstm_cell_forward(Gv[t], Cs[prev] if prev is not None else None, Cs[t], Hs[t],
                                           None, act[t])
                prev = t
        else:
            G = x2.float() @ w_ih.w.float().t() + b.w.float()
            Gv = G.view(T, B, 4 * Hd)
            prev = None
            for t in steps:
                g = Gv[t].clone()
                if prev is not None:
                    g += Hs[prev].float() @ w_hh.w.float().t()
                i, f, gg, o = g.chunk(4, 1)
                i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
                c = f * (Cs[prev] if prev is not None else 0) + i * gg
                tc = torch.tanh(c)
                Cs[t] = c
                Hs[t] = (o * tc).to(BF16)
                act[t] = torch.cat([i, f, gg, o, tc], 1)
                prev = t
        ctx.save_for_backward(x, Hs, Cs, act)
        ctx.p = (w_ih, w_hh, b, reverse, m)
        return Hs

    @staticmethod
    def backward(ctx, dH):
        x, Hs, Cs, act = ctx.saved_tensors
        w_ih, w_hh, b, reverse, m = ctx.p
        persist = (m.persist and not m.shared) if m is not None else True
        T, B, I = x.shape
        Hd = Hs.shape[2]
        dev = x.device
        dG = torch.empty(T, B, 4 * Hd, dtype=BF16, device=dev)
        order = list(range(T - 1, -1, -1) if reverse else range(T))
        rev_order = order[::-1]
        if dev.type == "cuda":
            sy, zeroed = _sync(dev, B, m)
            # the persistent kernel reads dH as it comes (bf16); only the
            # per-step path needs the fp32 accumulator it updates in place
            ran = PERSIST and persist and _ran(
                _T().lstm_seq_backward(act, Cs, _pitched(dH), w_hh.w, dG, reverse, sy, *_pl_args(m), zeroed),
                sy)
            if not ran:                            # per-step path: cell-state gradient carry
                dHf = dH.float().contiguous()
                dc = torch.zeros(B, Hd, dtype=torch.float32, device=dev)
                dc2 = torch.empty_like(dc)
            for k, t in enumerate([] if ran else rev_order):
                prev = rev_order[k + 1] if k + 1 < T else None   # the step that ran before t
                _T().lstm_cell_backward(act[t], Cs[prev] if prev is not None else None, dHf[t], dc,
                                        None, dc2, dG[t])
                dc, dc2 = dc2, dc
                if prev is not None:
                    _T().gemm(dG[t], True, w_hh.w, False, dHf[prev], 1, None, False, None, 1.0, True)
            dG2 = dG.view(T * B, 4 * Hd)
            # dW_hh = sum_t dG_t^T h_{t-1} over the steps with a predecessor:
            # row-shifted views of dG and Hs (no zero-padded h_{t-1} copy)
            Hs2 = Hs.view(T * B, Hd)
            if reverse:
                dGh, Hp = dG2[:(T - 1) * B], Hs2[B:]
            else:
                dGh, Hp = dG2[B:], Hs2[:(T - 1) * B]
            x2 = x.reshape(T * B, I)
            grouped = (LSTM_GROUPED_WGRAD and T > 1 and x2.is_contiguous() and Fx._group_ok(4 * Hd, Hd, (T - 1) * B)
                       and Fx._group_ok(4 * Hd, I, T * B))
            if grouped and LSTM_DEFER_WGRAD and Fx.defer_problems(
                    [(dGh, Hp, w_hh, None, Fx.grad_mode(w_hh)), (dG2, x2, w_ih, b, Fx.grad_mode(w_ih))]):
                # into the backward's ONE grouped launch (trainer group_wgrad):
                # grad_ready() is signalled by the flush
                grouped = None
            with Fx._OnWgrad(dG2, Hs, x):        # overlaps the next layer's recurrence
                if grouped is None:
                    pass
                elif grouped:
                    # dW_hh, dW_ih and the bias colsum in ONE launch (no split-K
                    # slabs, no separate column-sum passes)
                    empty = torch.empty(0, dtype=torch.float32, device=dev)
                    _T().gemm_wgrad_grouped([dGh, dG2], [Hp, x2], [w_hh.grad, w_ih.grad], [empty, b.grad],
                                            [Fx.grad_mode(w_hh), Fx.grad_mode(w_ih)])
                else:
                    if T > 1:
                        _T().gemm(dGh, False, Hp, False, w_hh.grad, Fx.grad_mode(w_hh), None, False, None, 1.0, True)
                    # bias gradient colsum(dG) fused into the weight-gradient GEMM
                    # where it runs on the igemm, else a pass inside the op
                    _T().gemm(dG2, False, x2, False, w_ih.grad, Fx.grad_mode(w_ih), None, False, None, 1.0, True,
                              b.grad)
            dx = None
            if ctx.needs_input_grad[0]:
                dx = torch.empty(T * B, I, dtype=BF16, device=dev)
                wk = Fx.weight_kmajor(w_ih)             # K-major W_ih copy of this step (KK GEMM)
                if wk is not None:
                    _T().gemm(dG2, True, wk, True, dx, 0, None, False, None, 1.0, False)
                else:
                    _T().gemm(dG2, True, w_ih.w, False, dx, 0, None, False, None, 1.0, False)
                dx = dx.view(T, B, I)
        else:
            dHf = dH.float().contiguous()          # dh accumulator (fp32), updated in place
            Whh = w_hh.w.float()
            dGf = torch.empty(T, B, 4 * Hd)
            dc = torch.zeros(B, Hd, dtype=torch.float32, device=dev)
            for k, t in enumerate(rev_order):
                prev = rev_order[k + 1] if k + 1 < T else None
                i, f, gg, o, tc = act[t].chunk(5, 1)
                dh = dHf[t]
                dcc = dh * o * (1 - tc * tc) + dc
                cp = Cs[prev] if prev is not None else torch.zeros_like(dc)
                di = dcc * gg * i * (1 - i)
                df = dcc * cp * f * (1 - f)
                dg_ = dcc * i * (1 - gg * gg)
                do = dh * tc * o * (1 - o)
                g4 = torch.cat([di, df, dg_, do], 1)
                dGf[t] = g4
                dG[t] = g4.to(BF16)
                dc = dcc * f
                if prev is not None:
                    dHf[prev] += dG[t].float() @ Whh
            Hprev = torch.zeros_like(Hs)
            if T > 1:
                if reverse:
                    Hprev[:-1] = Hs[1:]
                else:
                    Hprev[1:] = Hs[:-1]
            dG2 = dG.view(T * B, 4 * Hd).float()
            w_hh.grad += dG2.t() @ Hprev.view(T * B, Hd).float()
            w_ih.grad += dG2.t() @ x.reshape(T * B, I).float()
            b.grad += dG2.sum(0)
            dx = (dG2 @ w_ih.w.float()).to(BF16).view(T, B, I) if ctx.needs_input_grad[0] else None
        if not (dev.type == "cuda" and grouped is None):
            w_ih.grad_ready()
            w_hh.grad_ready()
            b.grad_ready()
        return dx, None, None, None, None, None, None


# TAM_LSTM_PITCHED=0: gather every non-contiguous dH (A/B)
LSTM_PITCHED_DH = os.environ.get("TAM_LSTM_PITCHED", "1") != "0"


def _pitched(dH: torch.Tensor) -> torch.Tensor:
    """dH as the persistent backward reads it: a [T,B,H] column slice of a
    wider gradient (the backward of the decoder / encoder feature concats
    hands the layer output's gradient as such a view) is read in place at
    its row pitch; anything else is made contiguous."""
    T, B, H = dH.shape
    if LSTM_PITCHED_DH and dH.stride(2) == 1 and dH.stride(1) >= H and dH.stride(0) == B * dH.stride(1):
        return dH
    return dH.contiguous()


def _pl_args(m):
    """(job_err, grids, reserved_cus) of a persistent launch for model m."""
    if m is None:
        return (None, -1, 0)
    g, r = m.residency
    return (m.err if (m.err is not None and m.err.is_cuda) else None, g, r)


def lstm(x, p, reverse=False, model=None):
    """x: [T,B,I] bf16 -> [T,B,H] bf16."""
    return _LSTMLayer.apply(x.contiguous(), p[0].arena.token, p[0], p[1], p[2], reverse, model)


class GNMT:
    name = "gnmt"
    branch_streams = 2          # independent recurrences that CAN be issued concurrently
    # ...but not by default: each per-timestep split-K recurrence GEMM already
    # spreads over all 256 CUs, so two co-running recurrences contend (CUs,
    # 2 x 8 MB of W_hh through the 4 MB per-XCD L2s): measured on MI355X,
    # hipGraph step 15.5 ms one stream vs 16.3 ms with branches
    branch_default = False
    # forward returns [T,B,V]; the trainer transposes the [B,T] labels to match
    logits_time_major = True
    # whole-sequence persistent recurrences; off for the rest of the job
    # after a barrier timeout (Worker.run reads the job's own err words)
    persist = True
    # ...and off while another job's persistent grids may share the GPU
    # (Trainer.set_persist_shared)
    shared = False

    def __init__(self, arena: Arena, vocab: int = 32000, hidden: int = 1024, enc_layers: int = 4,
                 dec_layers: int = 4, heads: int = 16):
        assert hidden == heads * 64
        A = arena
        H = hidden
        self.arena, self.H, self.heads, self.vocab = arena, H, heads, vocab
        self.src_emb = A.add("src_emb", (vocab, H), init="uniform", std=0.1)
        self.tgt_emb = A.add("tgt_emb", (vocab, H), init="uniform", std=0.1)

        def lstm_p(n, i):
            return (A.add(n + ".w_ih", (4 * H, i), init="uniform", std=0.1, store_grad=True),
                    A.add(n + ".w_hh", (4 * H, H), init="uniform", std=0.1, store_grad=True),
                    A.add(n + ".b", (4 * H,), init="zeros", decay=False))

        self.enc = [lstm_p("enc0.fw", H), lstm_p("enc0.bw", H), lstm_p("enc1", 2 * H)]
        self.enc += [lstm_p(f"enc{i}", H) for i in range(2, enc_layers)]
        self.dec = [lstm_p("dec0", H)] + [lstm_p(f"dec{i}", 2 * H) for i in range(1, dec_layers)]
        # weights whose gradient is one GEMM per step (store_grad: stored, not
        # accumulated into a zeroed buffer)
        self.att_q = A.add("att.q", (H, H), init="xavier", store_grad=True)
        self.att_kv = A.add("att.kv", (2 * H, H), init="xavier", store_grad=True)
        self.cls_w = A.add("cls.w", (vocab, 2 * H), init="uniform", std=0.1, store_grad=True)
        self.cls_b = A.add("cls.b", (vocab,), init="zeros", decay=False)
        self.training = True
        # this job's persistent-LSTM words: [0] barrier timeouts of the current
        # step (the optimizer's guard), [1] steps whose update was skipped
        self.err = torch.zeros(2, dtype=torch.int32, device=arena.device)
        # co-residency rule of this job's persistent grids (grids that must
        # fit at once, CUs reserved for RCCL): set by the trainer per job
        self.residency = (2, 0)

    def forward(self, batch):
        src, tgt_in = batch["src"], batch["tgt_in"]       # [B,S] token ids
        if src.is_cuda and PERSIST and self.persist and not self.shared:
            # the sync words of every persistent launch of this step (forward
            # and backward of each layer-direction) zeroed by one fill instead
            # of one zeroing kernel per launch
            B = src.shape[0]
            n = 2 * (len(self.enc) + len(self.dec)) * _sync_words(B)
            self._sync_pool = torch.empty(n, dtype=torch.int32, device=src.device)
            _T().zero_(self._sync_pool)
            self._sync_next, self._sync_B = 0, B
        # time-major activations [T,B,H]
        # branch 1: the first decoder layer (+ attention query) reads only the
        # target embedding, so it runs alongside the whole encoder stack;
        # branch 0: the reverse half of the bidirectional layer alongside the
        # forward half (ops/functional.py::on_branch; no-op without streams)
        # everything stays time-major [T,B,.]: the attention kernels take
        # batch / token strides and the logits come out [T,B,V] with the
        # labels transposed to match (logits_time_major), so no activation
        # or gradient is ever re-laid between the recurrences and attention
        if src.is_cuda and Fx.KMAJOR_DGRAD:
            # K-major copies of the weights whose input gradient is a KN GEMM
            # (every W_ih, the classifier), one launch: their dX run as KK
            Fx.prepare_weight_t([p[0] for p in self.enc + self.dec] + [self.cls_w])
        # the embeddings read the [B,S] ids time-major in place; every tensor
        # with several consumers goes through Fx.fanout (its gradients summed
        # by one launch of ours) and every feature concat through Fx.cat2, so
        # the step runs no torch elementwise / concat / copy kernels
        with Fx.on_branch(1, tgt_in):
            y = Fx.embedding(tgt_in, self.tgt_emb, time_major=True)
            d0 = lstm(y, self.dec[0], model=self)                    # [T,B,H]
            d0q, d0 = Fx.fanout(d0, 2)
            q = Fx.linear(d0q, self.att_q)                           # [T,B,H]
        x = Fx.embedding(src, self.src_emb, time_major=True)
        xb, x = Fx.fanout(x, 2)
        with Fx.on_branch(0, xb):
            bw = lstm(xb, self.enc[1], reverse=True, model=self)
        fw = lstm(x, self.enc[0], model=self)
        bw = Fx.join_branch(0, bw)
        h = lstm(Fx.cat2(fw, bw), self.enc[2], model=self)
        for p in self.enc[3:]:                           # residual from layer 3 on
            hi, h = Fx.fanout(h, 2)
            h = Fx.add(h, lstm(hi, p, model=self))
        kv = Fx.linear(h, self.att_kv)                   # [S,B,2H]
        d0, q = Fx.join_branch(1, d0, q)
        ctxv = Fx.cross_attention(q, kv, self.heads, time_major=True)   # [T,B,H]
        cs = Fx.fanout(ctxv, len(self.dec))              # the decoder layers' inputs + the classifier's
        h = d0
        for i, p in enumerate(self.dec[1:]):
            if i >= 1:
                hi, h = Fx.fanout(h, 2)
                h = Fx.add(h, lstm(Fx.cat2(hi, cs[i]), p, model=self))
            else:
                h = lstm(Fx.cat2(h, cs[i]), p, model=self)
        out = Fx.cat2(h, cs[-1])                         # [T,B,2H]
        return Fx.linear(out, self.cls_w, self.cls_b)    # [T,B,V] (logits_time_major)

    def buffers(self):
        return {}
