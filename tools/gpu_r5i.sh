#!/bin/bash
# round-5 GPU (i): LN weight-gradient column reduce on an aux stream (tests +
# Transformer A/B) and the igemm-epilogue BN statistics test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 500 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "layernorm or bn_stats or model_grads or grouped_wgrad_matches or model_trains" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/i_tests.out 2>&1
rc=$?; tail -4 gpurun_out/i_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=transformer bash tools/ab_rn50.sh base lnaux0=TAM_LN_AUX=0
