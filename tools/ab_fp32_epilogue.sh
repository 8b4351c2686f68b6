set -o pipefail
# cross-build A/B of the igemm LDS-staged fp32 epilogue on rank-k weight
# gradients (VGG classifier: K = batch 32): base = tiresias_amd/_C_base.so
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.
cat > /tmp/fp32ep.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from tiresias_amd.ops import _lib
T = _lib.ops(); T.gemm_lib_policy(0)
dev = torch.device("cuda", 0)
for M, N, K in ((4096, 25088, 32), (4096, 4096, 32), (1000, 4096, 32), (2048, 2048, 64)):
    A = torch.randn(K, M, device=dev).to(torch.bfloat16); B = torch.randn(K, N, device=dev).to(torch.bfloat16)
    c = torch.zeros(M, N, device=dev)
    fn = lambda: T.gemm(A, False, B, False, c, 1, None, False, None, 1.0, True)
    for _ in range(3): fn()
    torch.cuda.synchronize()
    c.zero_(); fn(); torch.cuda.synchronize()
    err = float((c - A.float().t() @ B.float()).norm() / (A.float().t() @ B.float()).norm())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(10): fn()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 100)
    print(json.dumps({"lib": sys.argv[1], "shape": f"{M}x{N}x{K} MN f32acc", "us": round(best, 1), "err": err}), flush=True)
PY
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export TAM_LIB_PATH=$PWD/tiresias_amd/_C_base.so; else unset TAM_LIB_PATH; fi
    timeout -k 10 120 python -u /tmp/fp32ep.py $v 2>/dev/null || exit 1
  done
done
