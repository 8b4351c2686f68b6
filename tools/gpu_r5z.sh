#!/bin/bash
# round-5 GPU (z): last full GPU suite + smoke on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/z_suite.out 2>&1
rc=$?; tail -3 gpurun_out/z_suite.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/z_smoke.out 2>&1
rc=$?; tail -1 gpurun_out/z_smoke.out; exit $rc
