#!/bin/bash
# round-5 GPU (u): the grouped weight-gradient launch vs per-GEMM dispatch
# (measured MFMA / hipBLASLt routing per shape), same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_MODELS=transformer,gnmt,resnet50 bash tools/ab_rn50.sh base nogroup=TAM_GROUP_MAX_MNK=1
