"""Full-size check of the 64-channel 3x3 weight gradient (VGG-16 224x224 /
112x112, ResNet-50 56x56): the patch-staged kernel and the tap-gather path
vs an fp32 torch reference at the model's batch (the unit tests use small
grids). Prints rel err per path."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

T = _lib.ops()
dev = torch.device("cuda", 0)
for N, H, C, K in ((32, 224, 64, 64), (32, 112, 64, 128), (64, 56, 64, 64), (32, 112, 128, 128)):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, H, H, K, device=dev).to(torch.bfloat16)
    wf = torch.zeros(K, C, 3, 3, device=dev, requires_grad=True)
    gw, = torch.autograd.grad(F.conv2d(x.float().permute(0, 3, 1, 2), wf, padding=1), [wf],
                              dy.float().permute(0, 3, 1, 2))
    ref = gw.permute(0, 2, 3, 1).contiguous()
    row = {"shape": [N, H, H, C, K]}
    for pol in (1, 0):
        T.conv_wgrad_c64_policy(pol)
        dw = torch.zeros(K, 3, 3, C, device=dev)
        T.conv_wgrad(dy, x, dw, 1, 1, 1, 0)
        torch.cuda.synchronize()
        e = ((dw - ref).norm() / ref.norm()).item()
        row["c64" if pol else "gather"] = e
        if e > 1e-3:
            d = (dw - ref).abs()
            row[("c64" if pol else "gather") + "_worst"] = [list(map(int, divmod(int(d.argmax()), 9 * C))), float(d.max())]
    T.conv_wgrad_c64_policy(1)
    print(json.dumps(row), flush=True)
    del x, dy, wf, gw, ref
    torch.cuda.empty_cache()
