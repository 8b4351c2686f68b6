#!/bin/bash
# round-5 GPU (n): BN apply-grid rule + pitched LSTM dH: numerics (BN, LSTM,
# GNMT/ResNet model tests), BN bench, ResNet-50 / GNMT A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "batchnorm or bn_ or lstm or gnmt or resnet" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/n_tests.out 2>&1
rc=$?; tail -3 gpurun_out/n_tests.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_bn.py --out gpurun_out/bnn_base.json > gpurun_out/bnn_base.log 2>&1 || exit $?
echo "bn $(tail -1 gpurun_out/bnn_base.log)"
AB_MODELS=resnet50 bash tools/ab_rn50.sh base ab2048=TAM_BN_APPLY_BLOCKS=2048 || exit $?
AB_MODELS=gnmt bash tools/ab_rn50.sh base pitch0=TAM_LSTM_PITCHED=0
