#!/bin/bash
# round-5 GPU (j): conv weight re-lay on a side stream, A/B (ResNet-50, VGG-16)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_MODELS=resnet50,vgg16 bash tools/ab_rn50.sh base wtside0=TAM_WT_SIDE=0
