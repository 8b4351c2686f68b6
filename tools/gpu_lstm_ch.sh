#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/lstm_ch_test.log 2>&1 || { tail -30 gpurun_out/lstm_ch_test.log; exit 1; }
tail -1 gpurun_out/lstm_ch_test.log
for ch in 1 2; do
python - <<PY > gpurun_out/lstm_ch$ch.json || exit 1
import json, time, torch
from tiresias_amd.ops import _lib
_lib.load(required=True)
T = torch.ops.tam
T.lstm_seq_policy($ch)
dev = "cuda"
Tn, B, Hd = 50, 64, 1024
gx = torch.randn(Tn, B, 4 * Hd, device=dev); w = (torch.randn(4 * Hd, Hd, device=dev) / 32).bfloat16()
hs = torch.empty(Tn, B, Hd, device=dev, dtype=torch.bfloat16); cs = torch.empty(Tn, B, Hd, device=dev)
act = torch.empty(Tn, B, 5 * Hd, device=dev); sync = torch.zeros(32 * 5, dtype=torch.int32, device=dev)
dH = torch.randn(Tn, B, Hd, device=dev); dG = torch.empty(Tn, B, 4 * Hd, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    assert T.lstm_seq_forward(gx, w, hs, cs, act, False, sync); assert T.lstm_seq_backward(act, cs, dH, w, dG, False, sync)
torch.cuda.synchronize()
def tm(f, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / n * 1e3
fw = tm(lambda: T.lstm_seq_forward(gx, w, hs, cs, act, False, sync))
bw = tm(lambda: T.lstm_seq_backward(act, cs, dH, w, dG, False, sync))
print(json.dumps({"ch": $ch, "fwd_us_per_seq": round(fw, 1), "bwd_us_per_seq": round(bw, 1), "T": Tn, "err": int(sync[0])}))
PY
cat gpurun_out/lstm_ch$ch.json
done
