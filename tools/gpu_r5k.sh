#!/bin/bash
# round-5 GPU (k): batched (deferred) LayerNorm weight-gradient column
# reduces -- tests, then Transformer A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "layernorm or grouped_wgrad_matches or model_grads or model_trains or graph" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/k_tests.out 2>&1
rc=$?; tail -4 gpurun_out/k_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=transformer bash tools/ab_rn50.sh base lndefer0=TAM_LN_DEFER=0
