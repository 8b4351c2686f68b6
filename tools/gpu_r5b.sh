#!/bin/bash
# round-5 GPU checks (b): BN kernel numerics + per-layer BN timings + ResNet-50
# step, then the multi-rank shared-GPU tests, the N=2 rehearsal (fill + lazy
# preemption + IPC moves) and the N=1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
run() {
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 4 "gpurun_out/$name.out"; tail -n 4 "gpurun_out/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
run bn_tests 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "bn or batchnorm" --timeout 120 --timeout-method thread -p no:cacheprovider
run bn_bench 200 python tools/bench_bn.py --out gpurun_out/bn_kernels.json
run rn50 200 python tools/bench_models.py --models resnet50 --graph --steps 30 --warmup 5
run mg_tests 300 python -u -m pytest tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
run n2 400 env TAM_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-nopool-replay
run n1 300 python bench.py --steps 5 --warmup 2 --no-nopool-replay
