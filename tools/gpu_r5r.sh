#!/bin/bash
# round-5 GPU (r): streaming Adam (U=4 + non-temporal) re-measured inside the
# graph steps, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_MODELS=gnmt,transformer bash tools/ab_rn50.sh base ov3=TAM_OPTIM_VARIANT=3
