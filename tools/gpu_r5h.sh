#!/bin/bash
# round-5 GPU (h): GNMT LSTM weight gradients deferred into the backward's
# grouped launch + grouped size cap + igemm-epilogue BN statistics: tests,
# then GNMT / Transformer / ResNet-50 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 500 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "grouped or gnmt or layernorm or bn_stats or batchnorm" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/h_tests.out 2>&1
rc=$?; tail -4 gpurun_out/h_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=resnet50 bash tools/ab_rn50.sh base istats0=TAM_CONV_IGEMM_STATS=0 || exit $?
AB_MODELS=gnmt,transformer bash tools/ab_rn50.sh base defer0=TAM_LSTM_DEFER=0 nocap=TAM_GROUP_MAX_MNK=1e30
