"""Bitwise A/B of the persistent LSTM recurrence between two builds
(TAM_LIB_PATH): same inputs, dumps h/c/act (forward) and dG (backward),
plus one GNMT fwd+bwd's loss and gradient, to gpurun_out/lstm_bits_<tag>.pt."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402

_lib.load(required=True)
T = torch.ops.tam
tag = sys.argv[1]
gpu = torch.device("cuda", 0)
out = {}
for (T_, B, Hd, rev) in [(50, 64, 1024, False), (50, 64, 1024, True)]:
    g = torch.Generator().manual_seed(21)
    gx = torch.randn(T_, B, 4 * Hd, generator=g).to(gpu)
    w = (torch.randn(4 * Hd, Hd, generator=g) / Hd ** 0.5).to(torch.bfloat16).to(gpu)
    hs = torch.empty(T_, B, Hd, device=gpu, dtype=torch.bfloat16)
    cs = torch.empty(T_, B, Hd, device=gpu)
    act = torch.empty(T_, B, 5 * Hd, device=gpu)
    sync = torch.zeros(32 * (4 * (B // 16) + 1), dtype=torch.int32, device=gpu)
    assert T.lstm_seq_forward(gx, w, hs, cs, act, rev, sync)
    dH = torch.randn(T_, B, Hd, generator=g).to(gpu)
    dG = torch.empty(T_, B, 4 * Hd, device=gpu, dtype=torch.bfloat16)
    sync.zero_()
    assert T.lstm_seq_backward(act, cs, dH, w, dG, rev, sync)
    torch.cuda.synchronize()
    out[f"rev{int(rev)}"] = dict(hs=hs.cpu(), cs=cs.cpu(), act=act.cpu(), dG=dG.cpu())
from tiresias_amd.executor.trainer import Trainer  # noqa: E402

t = Trainer("gnmt", gpu, seed=3, batch=64)
loss = t._fwd_bwd()
torch.cuda.synchronize()
out["gnmt"] = dict(loss=float(loss), grad=t.arena.grad.cpu(),
                   params=[(p.name, p.offset, p.numel) for p in t.arena.params])
# the same build again in this process: run-to-run determinism of one step
t2 = Trainer("gnmt", gpu, seed=3, batch=64)
t2._fwd_bwd()
torch.cuda.synchronize()
out["gnmt"]["grad_again"] = t2.arena.grad.cpu()
torch.save(out, f"gpurun_out/lstm_bits_{tag}.pt")
print(tag, "loss", float(loss))
