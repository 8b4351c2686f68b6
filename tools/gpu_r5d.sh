#!/bin/bash
# round-5 GPU (d): grouped K-split weight gradients -- kernel + model tests,
# then the four-model graph bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
run() {
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 6 "gpurun_out/$name.out"; tail -n 4 "gpurun_out/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
run gg_tests 200 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "grouped" --timeout 120 --timeout-method thread -p no:cacheprovider
run gg_model 400 python -u -m pytest tests/test_models_gpu.py -x -v -k "grouped" --timeout 300 --timeout-method thread -p no:cacheprovider
run models 300 python tools/bench_models.py --models resnet50,transformer --graph --steps 30 --warmup 5
