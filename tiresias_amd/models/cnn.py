"""ResNet-50 (v1.5) and VGG-16 on the tiresias_amd HIP kernels.

These are the image workloads the Tiresias north star time-slices (the
reference only *models* them: per-tensor gradient sizes in
``/root/reference/core/models.py:8-26`` and checkpoint sizes in
``model/model_factory.py:19-55``). Here they are real training jobs:

* activations NHWC bf16 (channels innermost = the implicit-GEMM K axis);
* the 3-channel RGB input is zero-padded to 8 channels so every conv keeps
  16-byte channel vectors;
* ResNet: BN + residual-add + ReLU fused in one kernel; the residual
  branch's gradient is summed inside the producing BN's backward (a tap, no
  add kernel); the ReLU backward of bn1/bn2 rides in the next conv's dgrad
  epilogue; VGG: conv + bias + ReLU fused in the conv epilogue, the ReLU
  backward fused into the next layer's dgrad epilogue;
* every conv weight is re-laid for dgrad once per step in one launch;
* BN statistics: fp64 sums accumulated by the producing conv's epilogue (or
  the BN's own pass) into per-layer slices of ONE buffer zeroed once per step;
  the apply passes finalize per channel in their prologue (no finalize
  launches);
* all weights live in one flat :class:`Arena` per job.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from ..ops import functional as Fx
from ..ops.arena import Arena


class _BNState:
    def __init__(self, C: int, device):
        self.mean = torch.zeros(C, dtype=torch.float32, device=device)
        self.var = torch.ones(C, dtype=torch.float32, device=device)


class ResNet50:
    """torchvision-style ResNet-50 v1.5 (stride on the 3x3 conv), NHWC."""

    name = "resnet50"

    def __init__(self, arena: Arena, num_classes: int = 1000, layers=(3, 4, 6, 3), width: int = 64,
                 in_ch: int = 8):
        self.arena = arena
        dev = arena.device
        self.training = True
        A = arena
        self.stem = A.add("stem.conv", (width, 7, 7, in_ch), init="kaiming")
        self.stem_bn = (A.add("stem.bn.g", (width,), init="ones", decay=False, fp32_compute=True),
                        A.add("stem.bn.b", (width,), init="zeros", decay=False, fp32_compute=True))
        self.bn_state = {"stem": _BNState(width, dev)}
        self.blocks: List[dict] = []
        cin = width
        for si, (n, w) in enumerate(zip(layers, [width, width * 2, width * 4, width * 8])):
            for bi in range(n):
                stride = 2 if (bi == 0 and si > 0) else 1
                pre = f"s{si}.b{bi}"
                blk = {
                    "stride": stride,
                    "c1": A.add(pre + ".c1", (w, 1, 1, cin), init="kaiming"),
                    "c2": A.add(pre + ".c2", (w, 3, 3, w), init="kaiming"),
                    "c3": A.add(pre + ".c3", (w * 4, 1, 1, w), init="kaiming"),
                }
                for k, c in (("bn1", w), ("bn2", w), ("bn3", w * 4)):
                    # zero-init the last BN gamma of each block (standard trick)
                    blk[k] = (A.add(f"{pre}.{k}.g", (c,), init="zeros" if k == "bn3" else "ones",
                                    decay=False, fp32_compute=True),
                              A.add(f"{pre}.{k}.b", (c,), init="zeros", decay=False, fp32_compute=True))
                    self.bn_state[f"{pre}.{k}"] = _BNState(c, dev)
                if bi == 0:
                    blk["down"] = A.add(pre + ".down", (w * 4, 1, 1, cin), init="kaiming")
                    blk["down_bn"] = (A.add(pre + ".dbn.g", (w * 4,), init="ones", decay=False, fp32_compute=True),
                                      A.add(pre + ".dbn.b", (w * 4,), init="zeros", decay=False, fp32_compute=True))
                    self.bn_state[pre + ".dbn"] = _BNState(w * 4, dev)
                blk["pre"] = pre
                self.blocks.append(blk)
                cin = w * 4
        self.bn_buf, self.bn_ws = Fx.bn_workspaces(
            {k: st.mean.numel() for k, st in self.bn_state.items()}, dev)
        self.fc_w = A.add("fc.w", (num_classes, cin), init="normal", std=0.01)
        self.fc_b = A.add("fc.b", (num_classes,), init="zeros", decay=False)
        self.num_classes = num_classes
        self.in_ch = in_ch

    def _bn(self, x, p, key, relu, res=None, consumer_masks=False):
        st = self.bn_state[key]
        return Fx.batchnorm(x, p[0], p[1], st.mean, st.var, relu=relu, residual=res,
                            training=self.training, consumer_masks=consumer_masks,
                            ws=self.bn_ws[key])

    def _st(self, key):
        # the conv feeding BN `key` accumulates its statistics into the BN's
        # forward workspace (training on GPU), else the BN reduces itself
        return self.bn_ws[key].fwd if (self.training and self.bn_buf.is_cuda) else True

    def conv_params(self):
        out = [self.stem]
        for blk in self.blocks:
            out += [blk["c1"], blk["c2"], blk["c3"]] + ([blk["down"]] if "down" in blk else [])
        return out

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        Fx.prepare_conv_wt(self.conv_params())
        if self.training:
            # every BN accumulator of this step: one zeroing launch of ours
            if self.bn_buf.is_cuda:
                Fx._T().zero_(self.bn_buf)
            else:
                self.bn_buf.zero_()
        y = Fx.conv2d(x, self.stem, stride=2, pad=3, bn_stats=self._st("stem"))
        y = self._bn(y, self.stem_bn, "stem", relu=True)
        y = Fx.maxpool2d(y, 3, 2, 1)
        for blk in self.blocks:
            pre = blk["pre"]
            # the second consumer of y (residual / downsample) goes through a
            # tap: its gradient is summed inside y's producing BN backward (a
            # fan-out summed by our kernel when the producer is the max-pool)
            y, y2 = Fx.residual_split(y)
            idn = y2 if "down" not in blk else None
            # bn1 / bn2 outputs feed exactly one conv each: that conv's dgrad
            # epilogue applies their ReLU backward mask (in_relu)
            o = Fx.conv2d(y, blk["c1"], bn_stats=self._st(pre + ".bn1"))
            o = self._bn(o, blk["bn1"], pre + ".bn1", relu=True, consumer_masks=True)
            o = Fx.conv2d(o, blk["c2"], stride=blk["stride"], pad=1, in_relu=True,
                          bn_stats=self._st(pre + ".bn2"))
            o = self._bn(o, blk["bn2"], pre + ".bn2", relu=True, consumer_masks=True)
            o = Fx.conv2d(o, blk["c3"], in_relu=True, bn_stats=self._st(pre + ".bn3"))
            if "down" in blk:
                idn = Fx.conv2d(y2, blk["down"], stride=blk["stride"],
                                bn_stats=self._st(pre + ".dbn"))
                idn = self._bn(idn, blk["down_bn"], pre + ".dbn", relu=False)
            y = self._bn(o, blk["bn3"], pre + ".bn3", relu=True, res=idn)
        y = Fx.global_avgpool(y)
        return Fx.linear(y, self.fc_w, self.fc_b)

    def buffers(self):
        out = {}
        for k, st in self.bn_state.items():
            out[k + ".mean"] = st.mean
            out[k + ".var"] = st.var
        return out


VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG16:
    """VGG-16 (configuration D), NHWC, conv+bias+ReLU fused; no dropout
    (synthetic-data throughput workload)."""

    name = "vgg16"

    def __init__(self, arena: Arena, num_classes: int = 1000, cfg=VGG16_CFG, in_ch: int = 8,
                 image: int = 224, fc: int = 4096):
        self.arena = arena
        A = arena
        self.layers: List[Tuple[str, object]] = []
        cin = in_ch
        spatial = image
        ci = 0
        for v in cfg:
            if v == "M":
                self.layers.append(("pool", None))
                spatial //= 2
            else:
                w = A.add(f"conv{ci}.w", (v, 3, 3, cin), init="kaiming")
                b = A.add(f"conv{ci}.b", (v,), init="zeros", decay=False)
                self.layers.append(("conv", (w, b)))
                cin = v
                ci += 1
        self.flat = cin * spatial * spatial
        # classifier weights: one dW GEMM per step each (store_grad)
        self.fc = [(A.add("fc0.w", (fc, self.flat), init="normal", std=0.005, store_grad=True),
                    A.add("fc0.b", (fc,), init="zeros", decay=False)),
                   (A.add("fc1.w", (fc, fc), init="normal", std=0.005, store_grad=True),
                    A.add("fc1.b", (fc,), init="zeros", decay=False)),
                   (A.add("fc2.w", (num_classes, fc), init="normal", std=0.005, store_grad=True),
                    A.add("fc2.b", (num_classes,), init="zeros", decay=False))]
        self.num_classes = num_classes
        self.in_ch = in_ch
        self.training = True

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        Fx.prepare_conv_wt([p[0] for kind, p in self.layers if kind == "conv"])
        y = x
        in_relu = False
        n = len(self.layers)
        for i, (kind, p) in enumerate(self.layers):
            if kind == "pool":
                y = Fx.maxpool2d(y, 2, 2, 0)
                continue
            w, b = p
            # this conv's ReLU mask is applied by the consumer (next conv /
            # fc0 dgrad epilogue masks with its relu-output input)
            y = Fx.conv2d(y, w, b, stride=1, pad=1, relu=True, in_relu=in_relu, mask_own_relu=False)
            in_relu = True
        y = y.reshape(y.shape[0], -1)
        (w0, b0), (w1, b1), (w2, b2) = self.fc
        y = Fx.linear(y, w0, b0, relu=True, in_relu=True, mask_own_relu=False)
        y = Fx.linear(y, w1, b1, relu=True, in_relu=True, mask_own_relu=False)
        return Fx.linear(y, w2, b2, in_relu=True)

    def buffers(self):
        return {}
