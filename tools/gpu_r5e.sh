#!/bin/bash
# round-5 GPU (e): grouped-wgrad model tests (early flush), then ResNet-50 /
# Transformer A/B of the early flush.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -v -k "grouped" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gg_model2.out 2>&1
rc=$?; tail -8 gpurun_out/gg_model2.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=resnet50,transformer bash tools/ab_rn50.sh early early0=TAM_GROUP_EARLY=0
