#!/bin/bash
# round-5 GPU (w): grouped-launch size cap under the measured library routing
# (problems above the cap go to per-GEMM dispatch), same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_MODELS=gnmt,transformer bash tools/ab_rn50.sh base cap34=TAM_GROUP_MAX_MNK=17179869184 cap33=TAM_GROUP_MAX_MNK=8589934592
