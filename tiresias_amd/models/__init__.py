"""Model zoo: the DL workloads the cluster scheduler runs as real jobs.

``MODELS[name]`` gives the builder, default per-GPU batch and the optimizer
recipe; ``make_model(name, arena, **over)`` instantiates it; ``synthetic_batch``
creates a fixed random batch of the right shape (no datasets on the box).
Reference: the simulated model table ``/root/reference/core/models.py:8-26``
and ``model/model_factory.py:19-55`` (sizes only).
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Any, Callable, Dict

import torch

from .cnn import ResNet50, VGG16
from .gnmt import GNMT
from .transformer import TransformerBase


@dataclass
class ModelSpec:
    builder: Callable
    kind: str                      # "image" | "seq2seq"
    batch: int                     # per-GPU batch (images / sentences)
    opt: str                       # "sgd" | "adam"
    lr: float
    wd: float
    kwargs: Dict[str, Any] = field(default_factory=dict)
    image: int = 224
    classes: int = 1000
    seq: int = 128
    vocab: int = 32000
    smoothing: float = 0.0
    # weight gradients on a side stream, overlapping the dgrad chain (measured
    # per model on MI355X, hipGraph replay: VGG-16 7.95 -> 7.59 ms; ResNet-50
    # +3 %, Transformer +2 %, GNMT +20 %: big wgrad GEMMs starve the
    # latency-bound recurrence / small-GEMM chains of CUs)
    overlap_wgrad: bool = False
    # Linear weight gradients deferred and issued as ONE grouped launch per
    # backward (ops/functional.py defer_wgrad; 1-GPU jobs)
    group_wgrad: bool = False


MODELS: Dict[str, ModelSpec] = {
    # the 1x1 / stride-1 conv weight gradients (stages 1-3) as one K-split
    # grouped launch at the end of the backward (ops/functional.py _Conv)
    "resnet50": ModelSpec(ResNet50, "image", 64, "sgd", 0.1, 1e-4, group_wgrad=True),
    # (no layer of VGG-16 is grouped-eligible; deferral here batches the
    # slab-split conv weight-gradient reduces into one launch per backward)
    "vgg16": ModelSpec(VGG16, "image", 32, "sgd", 0.01, 5e-4, group_wgrad=True),
    # weight-gradient side stream: measured per model (profiles/r2/ab_overlap.txt,
    # hipGraph steps): Transformer 7.28 -> 7.14 ms on; ResNet-50 10.65 -> 11.01
    # and GNMT 10.87 -> 11.93 (the persistent recurrence loses its CUs) off.
    # Re-measured at the end of round 4 with the slab-split weight gradients
    # (profiles/r4/*_overlap_ab.log): VGG-16 6.71 on vs 6.62 off (off: the
    # patch-staged 224x224 wgrad runs again), ResNet-50 9.63 on vs 9.19 off
    # (Transformer re-measured too: 5.38 on vs 5.21 off -- the deferred weight
    # gradients are one grouped launch at the end of the backward now)
    "transformer": ModelSpec(TransformerBase, "seq2seq", 32, "adam", 5e-4, 0.0, seq=128,
                             smoothing=0.1, group_wgrad=True),
    # LSTM dW_hh / dW_ih (+ bias column sums) and the attention projections'
    # weight gradients as one grouped launch per backward (models/gnmt.py)
    "gnmt": ModelSpec(GNMT, "seq2seq", 64, "adam", 1e-3, 0.0, seq=50, group_wgrad=True),
    # tiny variants (CPU tests / gloo rehearsals / smoke)
    "resnet_tiny": ModelSpec(ResNet50, "image", 4, "sgd", 0.1, 1e-4,
                             dict(layers=(1, 1, 1, 1), width=8, num_classes=16), image=32, classes=16),
    "vgg_tiny": ModelSpec(VGG16, "image", 4, "sgd", 0.01, 5e-4,
                          dict(cfg=[16, "M", 32, "M"], image=16, fc=64, num_classes=16),
                          image=16, classes=16),
    "transformer_tiny": ModelSpec(TransformerBase, "seq2seq", 4, "adam", 1e-3, 0.0,
                                  dict(vocab=512, d=64, heads=1, ffn=128, enc_layers=1,
                                       dec_layers=1, max_len=64), seq=16, vocab=512, smoothing=0.1),
    "gnmt_tiny": ModelSpec(GNMT, "seq2seq", 4, "adam", 1e-3, 0.0,
                           dict(vocab=512, hidden=64, enc_layers=3, dec_layers=2, heads=1),
                           seq=8, vocab=512),
}

# model family for the reference's model names (core/models.py:20, model_factory.py)
FAMILY = {
    "resnet50": "resnet50", "resnet101": "resnet50", "resnet152": "resnet50",
    "vgg16": "vgg16", "vgg19": "vgg16", "vgg11": "vgg16", "alexnet": "vgg16",
    "inception3": "resnet50", "inception4": "resnet50",
    "transformer": "transformer", "bert": "transformer", "gnmt": "gnmt", "lstm": "gnmt",
}


def make_model(name: str, arena, **over):
    spec = MODELS[name]
    kw = dict(spec.kwargs)
    kw.update(over)
    return spec.builder(arena, **kw)


def synthetic_batch(name: str, batch: int, device, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Fixed random batch generated ON the device (no host RNG / H2D on job start)."""
    spec = MODELS[name]
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    if spec.kind == "image":
        x = torch.zeros(batch, spec.image, spec.image, 8, device=dev, dtype=torch.bfloat16)
        x[..., :3] = torch.randn(batch, spec.image, spec.image, 3, generator=g, device=dev)
        y = torch.randint(0, spec.classes, (batch,), generator=g, device=dev)
        return {"x": x, "labels": y}
    S = spec.seq
    src = torch.randint(1, spec.vocab, (batch, S), generator=g, device=dev)
    tgt = torch.randint(1, spec.vocab, (batch, S + 1), generator=g, device=dev)
    return {"src": src, "tgt_in": tgt[:, :-1].contiguous(), "labels": tgt[:, 1:].contiguous()}


def samples_per_batch(name: str, batch: int) -> int:
    """Throughput unit: images for CNNs, target tokens for seq2seq."""
    spec = MODELS[name]
    return batch if spec.kind == "image" else batch * spec.seq
