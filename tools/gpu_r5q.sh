#!/bin/bash
# round-5 GPU (q): attention kernels with one-tile-ahead fetches: numerics,
# then same-box A/B against the previous build (Transformer, GNMT)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "attn or attention or transformer" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.out 2>&1
rc=$?; tail -3 gpurun_out/q_tests.out; [ $rc -eq 0 ] || exit $rc
AB_MODELS=transformer,gnmt bash tools/ab_so.sh
