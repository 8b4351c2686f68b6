#!/bin/bash
# round-5 GPU (c): per-call kernel trace of the ResNet-50 graph step (layer
# attribution of BN / igemm time), then the grouped-dW PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rn50_trace -o run -- \
  python3 tools/bench_models.py --models resnet50 --graph --steps 3 --warmup 2 > gpurun_out/rn50_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rn50_trace.log; exit $rc; }
find gpurun_out/rn50_trace -name "*.db" -delete
bash tools/pmc_grouped.sh
