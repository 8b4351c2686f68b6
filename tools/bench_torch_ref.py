"""Stock PyTorch-ROCm baseline for the four cluster workloads.

Same architectures, batch sizes and optimizer recipes as ``tiresias_amd.models``
(ResNet-50 v1.5 bs64 SGD, VGG-16 bs32 SGD, Transformer-base 32x128 Adam,
GNMT-8 64x50 Adam), written with ``torch.nn`` and run the way a PyTorch user
would: bf16 autocast, fp32 master weights, channels_last, MIOpen convs,
hipBLASLt GEMMs, SDPA attention, ``nn.LSTM`` (MIOpen RNN), fused
optimizers. This is the comparison point for ``tools/bench_models.py``
(our hand-written kernels): same work per step, different compute path.

  python tools/bench_torch_ref.py --out profiles/torch_ref.json
"""
from __future__ import annotations

import argparse
import json
import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, w, stride, down):
        super().__init__()
        self.c1 = nn.Conv2d(cin, w, 1, bias=False)
        self.b1 = nn.BatchNorm2d(w)
        self.c2 = nn.Conv2d(w, w, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(w)
        self.c3 = nn.Conv2d(w, 4 * w, 1, bias=False)
        self.b3 = nn.BatchNorm2d(4 * w)
        self.down = nn.Sequential(nn.Conv2d(cin, 4 * w, 1, stride, bias=False),
                                  nn.BatchNorm2d(4 * w)) if down else None

    def forward(self, x):
        o = F.relu(self.b1(self.c1(x)))
        o = F.relu(self.b2(self.c2(o)))
        o = self.b3(self.c3(o))
        return F.relu(o + (self.down(x) if self.down is not None else x))


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for si, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for bi in range(n):
                blocks.append(Bottleneck(cin, w, 2 if (bi == 0 and si > 0) else 1, bi == 0))
                cin = 4 * w
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        y = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(y, 1), 1))


class VGG16(nn.Module):
    CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]

    def __init__(self, classes=1000):
        super().__init__()
        layers, cin = [], 3
        for v in self.CFG:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, 1, 1), nn.ReLU(inplace=True)]
                cin = v
        self.features = nn.Sequential(*layers)
        self.cls = nn.Sequential(nn.Linear(512 * 49, 4096), nn.ReLU(True), nn.Linear(4096, 4096),
                                 nn.ReLU(True), nn.Linear(4096, classes))

    def forward(self, x):
        return self.cls(torch.flatten(self.features(x), 1))


class Transformer(nn.Module):
    """Transformer-base, pre-LN, tied embeddings, SDPA attention, no dropout."""

    def __init__(self, vocab=32000, d=512, heads=8, ffn=2048, layers=6):
        super().__init__()
        self.emb = nn.Embedding(vocab, d)
        nn.init.normal_(self.emb.weight, std=d ** -0.5)
        self.d = d
        pos = torch.arange(1024, dtype=torch.float32)[:, None]
        i = torch.arange(0, d, 2, dtype=torch.float32)[None, :]
        pe = torch.zeros(1024, d)
        pe[:, 0::2] = torch.sin(pos / 10000 ** (i / d))
        pe[:, 1::2] = torch.cos(pos / 10000 ** (i / d))
        self.register_buffer("pe", pe)
        self.tf = nn.Transformer(d, heads, layers, layers, ffn, dropout=0.0, batch_first=True,
                                 norm_first=True)

    def forward(self, src, tgt):
        e = lambda t: self.emb(t) * math.sqrt(self.d) + self.pe[: t.shape[1]]
        mask = nn.Transformer.generate_square_subsequent_mask(tgt.shape[1], device=tgt.device)
        h = self.tf(e(src), e(tgt), tgt_mask=mask, tgt_is_causal=True)
        return h @ self.emb.weight.t()


class GNMT(nn.Module):
    """GNMT: bi-LSTM + 3 LSTM encoder layers (residual from 3), 4 decoder
    layers with multi-head attention on the first decoder layer's output."""

    def __init__(self, vocab=32000, H=1024, heads=16):
        super().__init__()
        self.H, self.heads = H, heads
        self.se = nn.Embedding(vocab, H)
        self.te = nn.Embedding(vocab, H)
        self.e0 = nn.LSTM(H, H, bidirectional=True)
        self.e1 = nn.LSTM(2 * H, H)
        self.e2 = nn.LSTM(H, H)
        self.e3 = nn.LSTM(H, H)
        self.d0 = nn.LSTM(H, H)
        self.d = nn.ModuleList([nn.LSTM(2 * H, H) for _ in range(3)])
        self.q = nn.Linear(H, H, bias=False)
        self.kv = nn.Linear(H, 2 * H, bias=False)
        self.cls = nn.Linear(2 * H, vocab)

    def forward(self, src, tgt):
        x = self.se(src.t())                              # [S,B,H]
        h, _ = self.e0(x)
        h, _ = self.e1(h)
        h = h + self.e2(h)[0]
        h = h + self.e3(h)[0]
        y = self.te(tgt.t())
        d0, _ = self.d0(y)                                # [T,B,H]
        B, T, S, nh = d0.shape[1], d0.shape[0], h.shape[0], self.heads
        q = self.q(d0).permute(1, 0, 2).reshape(B, T, nh, -1).transpose(1, 2)
        kv = self.kv(h).permute(1, 0, 2).reshape(B, S, 2, nh, -1)
        k, v = kv[:, :, 0].transpose(1, 2), kv[:, :, 1].transpose(1, 2)
        c = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, T, -1).transpose(0, 1)
        hh = d0
        for i, l in enumerate(self.d):
            o, _ = l(torch.cat([hh, c], 2))
            hh = hh + o if i >= 1 else o
        return self.cls(torch.cat([hh, c], 2)).transpose(0, 1)


SPECS = {
    "resnet50": (ResNet50, 64, "sgd", 0.1, 1e-4),
    "vgg16": (VGG16, 32, "sgd", 0.01, 5e-4),
    "transformer": (Transformer, 32, "adam", 5e-4, 0.0),
    "gnmt": (GNMT, 64, "adam", 1e-3, 0.0),
}


def bench(name, steps, warmup, dev):
    cls, B, opt, lr, wd = SPECS[name]
    torch.manual_seed(0)
    m = cls().to(dev)
    image = name in ("resnet50", "vgg16")
    if image:
        m = m.to(memory_format=torch.channels_last)
        x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev)
        fwd = lambda: F.cross_entropy(m(x), y)
        samples = B
    else:
        S = 128 if name == "transformer" else 50
        src = torch.randint(1, 32000, (B, S), device=dev)
        tgt = torch.randint(1, 32000, (B, S + 1), device=dev)
        ti, lab = tgt[:, :-1].contiguous(), tgt[:, 1:].contiguous()
        sm = 0.1 if name == "transformer" else 0.0
        fwd = lambda: F.cross_entropy(m(src, ti).reshape(-1, 32000).float(), lab.reshape(-1),
                                      label_smoothing=sm)
        samples = B * S
    if opt == "sgd":
        o = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=wd, fused=True)
    else:
        o = torch.optim.Adam(m.parameters(), lr=lr, betas=(0.9, 0.98), eps=1e-9, fused=True)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = fwd()
        loss.backward()
        o.step()
        o.zero_grad(set_to_none=False)
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dict(model=name, batch=B, path="torch eager (autocast bf16, MIOpen/hipBLASLt/SDPA)",
                ms_per_step=dt * 1e3, samples_per_s=samples / dt, loss=float(loss))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16,transformer,gnmt")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    res = []
    for n in a.models.split(","):
        r = bench(n, a.steps, a.warmup, dev)
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        json.dump({"models": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
