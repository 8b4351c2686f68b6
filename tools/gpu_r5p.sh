#!/bin/bash
# round-5 GPU (p): end-of-work checkpoint -- per-call step traces of the
# three models, then the GPU suite, smoke, N=1 bench and the N=2 shared-GPU
# rehearsal (tools/gpu_final.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_trace3.sh || exit $?
bash tools/gpu_final.sh
