#!/bin/bash
# round-5 GPU (l): deferred + batched conv weight-gradient slab reduces:
# tests, then ResNet-50 / VGG-16 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "grouped or model_grads or model_trains or graph or wgrad or resnet or vgg" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/l_tests.out 2>&1
rc=$?; tail -4 gpurun_out/l_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=resnet50,vgg16 bash tools/ab_rn50.sh base slab0=TAM_SLAB_DEFER=0
