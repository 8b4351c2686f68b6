"""Transformer-base (Vaswani et al.: d=512, 8 heads, FFN 2048, 6+6 layers)
on the tiresias_amd kernels.

MI355X-first layout decisions:
  * one fused QKV projection per self-attention ([B,S,3,H,64] packed) read in
    place by the flash-attention kernel (no split/permute copies) and
    gradients written back packed;
  * cross-attention K/V from one fused [d -> 2d] projection of the encoder
    output;
  * pre-LN residual blocks with every residual add fused into the next
    LayerNorm's kernel; FFN bias+ReLU fused into the first GEMM's epilogue
    and the ReLU backward into the second GEMM's dgrad epilogue;
  * tied source/target embedding + output projection; the loss is the fused
    softmax-xent kernel with label smoothing 0.1.
Dropout is omitted (synthetic-data throughput workload).
"""
from __future__ import annotations

import math

import torch

from ..ops import functional as Fx
from ..ops.arena import Arena


class TransformerBase:
    name = "transformer"

    def __init__(self, arena: Arena, vocab: int = 32000, d: int = 512, heads: int = 8,
                 ffn: int = 2048, enc_layers: int = 6, dec_layers: int = 6, max_len: int = 1024):
        assert d == heads * 64, "kernels are built for head_dim 64"
        A = arena
        self.arena, self.d, self.h, self.vocab = arena, d, heads, vocab
        self.emb = A.add("emb", (vocab, d), init="normal", std=d ** -0.5)
        self.pos = self._sinusoid(max_len, d, arena.device)

        def ln(n):
            return (A.add(n + ".g", (d,), init="ones", decay=False, fp32_compute=True),
                    A.add(n + ".b", (d,), init="zeros", decay=False, fp32_compute=True))

        def lin(n, o, i, bias=True):
            # one dW GEMM per step each (grouped launch, store mode): store_grad
            w = A.add(n + ".w", (o, i), init="xavier", store_grad=True)
            b = A.add(n + ".b", (o,), init="zeros", decay=False) if bias else None
            return (w, b)

        self.enc = []
        for i in range(enc_layers):
            p = f"enc{i}"
            self.enc.append(dict(ln1=ln(p + ".ln1"), qkv=lin(p + ".qkv", 3 * d, d), o=lin(p + ".o", d, d),
                                 ln2=ln(p + ".ln2"), f1=lin(p + ".f1", ffn, d), f2=lin(p + ".f2", d, ffn)))
        self.enc_ln = ln("enc.ln")
        self.dec = []
        for i in range(dec_layers):
            p = f"dec{i}"
            self.dec.append(dict(ln1=ln(p + ".ln1"), qkv=lin(p + ".qkv", 3 * d, d), o=lin(p + ".o", d, d),
                                 ln2=ln(p + ".ln2"), q=lin(p + ".q", d, d),
                                 o2=lin(p + ".o2", d, d), ln3=ln(p + ".ln3"),
                                 f1=lin(p + ".f1", ffn, d), f2=lin(p + ".f2", d, ffn)))
        # every decoder layer's cross-attention K/V projection of the encoder
        # memory as ONE [L*2d, d] GEMM (per-layer xavier bound): one fwd GEMM,
        # one dgrad, one wgrad instead of L each + L-1 gradient sums
        self.dec_kv = (A.add("dec.kv.w", (dec_layers * 2 * d, d), init="uniform",
                             std=math.sqrt(6.0 / (3 * d)), store_grad=True),
                       A.add("dec.kv.b", (dec_layers * 2 * d,), init="zeros", decay=False))
        self.dec_ln = ln("dec.ln")
        self.training = True

    @staticmethod
    def _sinusoid(n, d, dev):
        pos = torch.arange(n, dtype=torch.float32)[:, None]
        i = torch.arange(0, d, 2, dtype=torch.float32)[None, :]
        ang = pos / torch.pow(10000.0, i / d)
        pe = torch.zeros(n, d)
        pe[:, 0::2] = torch.sin(ang)
        pe[:, 1::2] = torch.cos(ang)
        return pe.to(device=dev, dtype=torch.bfloat16)

    def _embed(self, ids):
        # scale + positional table in the embedding kernel (no broadcast copy)
        return Fx.embedding(ids, self.emb, scale=math.sqrt(self.d), pos=self.pos[:ids.shape[1]])

    @staticmethod
    def _ln_skip(x, r, p):
        """(x + r, LN(x + r)) with the residual add fused into the LN kernel,
        or (x, LN(x)) when no residual is pending."""
        if r is None:
            return Fx.layernorm_skip(x, *p)
        return Fx.add_layernorm_skip(x, r, *p)

    def _ffn(self, x, r, L):
        """FFN sub-block: returns (residual stream, pending FFN output)."""
        x, h = self._ln_skip(x, r, L["ln2" if "q" not in L else "ln3"])
        (w1, b1), (w2, b2) = L["f1"], L["f2"]
        h = Fx.linear(h, w1, b1, relu=True, mask_own_relu=False)
        return x, Fx.linear(h, w2, b2, in_relu=True)

    # Each sub-block's output is carried as a PENDING residual r and added by
    # the next LayerNorm's kernel (add_layernorm_skip): no separate add pass.
    def encode(self, src):
        x, r = self._embed(src), None
        for L in self.enc:
            x, h = self._ln_skip(x, r, L["ln1"])
            qkv = Fx.linear(h, *L["qkv"])
            a = Fx.self_attention(qkv, self.h, causal=False)
            r = Fx.linear(a, *L["o"])
            x, r = self._ffn(x, r, L)
        return self._ln_skip(x, r, self.enc_ln)[1]

    def decode(self, tgt, mem):
        x, r = self._embed(tgt), None
        n = len(self.dec)
        kv_all = Fx.linear(mem, *self.dec_kv)          # [B, S, n*2d]
        hold = {"n": 0}
        for i, L in enumerate(self.dec):
            x, h = self._ln_skip(x, r, L["ln1"])
            a = Fx.self_attention(Fx.linear(h, *L["qkv"]), self.h, causal=True)
            x, h = self._ln_skip(x, Fx.linear(a, *L["o"]), L["ln2"])
            q = Fx.linear(h, *L["q"])
            a = Fx.cross_attention(q, kv_all, self.h, k_slot=2 * i, v_slot=2 * i + 1, nkv=2 * n,
                                   kv_hold=hold)
            x, r = self._ffn(x, Fx.linear(a, *L["o2"]), L)
        x = self._ln_skip(x, r, self.dec_ln)[1]
        return Fx.linear(x, self.emb)   # tied output projection -> logits

    def forward(self, batch):
        src, tgt_in = batch["src"], batch["tgt_in"]
        if src.is_cuda and Fx.KMAJOR_DGRAD:
            # K-major copies of every 2-D weight (the Linear weights and the
            # tied embedding / output projection), one launch: the input
            # gradients dX = dY . W run as KK GEMMs (Fx.prepare_weight_t;
            # graph step 4.99-5.03 -> 4.89-4.94 ms, same box)
            Fx.prepare_weight_t([p for p in self.arena.params if len(p.shape) == 2])
        return self.decode(tgt_in, self.encode(src))

    def buffers(self):
        return {}
