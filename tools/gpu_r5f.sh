#!/bin/bash
# round-5 GPU (f): LayerNorm kernels (operand prefetch) + grouped model tests,
# then the Transformer / ResNet-50 graph steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "layernorm or grouped or transformer" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ln_tests.out 2>&1
rc=$?; tail -4 gpurun_out/ln_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=transformer,resnet50 bash tools/ab_rn50.sh ln
