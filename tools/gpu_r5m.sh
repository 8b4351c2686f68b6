#!/bin/bash
# round-5 GPU (m): channel-slabbed BN reduction passes + BN grid knobs:
# numerics, per-shape BN bench over the knobs, ResNet-50 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "batchnorm or bn_" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/m_tests.out 2>&1
rc=$?; tail -3 gpurun_out/m_tests.out; [ $rc -eq 0 ] || exit $rc
for spec in base slab0=TAM_BN_RED_SLAB=0 rb256=TAM_BN_RED_BLOCKS=256 rb1024=TAM_BN_RED_BLOCKS=1024 ab1024=TAM_BN_APPLY_BLOCKS=1024 ab512=TAM_BN_APPLY_BLOCKS=512; do
  name=${spec%%=*}; envs=${spec#*=}
  [ "$name" = "$spec" ] && envs=""
  timeout -k 10 200 env $envs python tools/bench_bn.py --out gpurun_out/bnm_$name.json > gpurun_out/bnm_$name.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/bnm_$name.log; exit $rc; }
  echo "$name $(tail -1 gpurun_out/bnm_$name.log)"
done
bash tools/ab_rn50.sh base slab0=TAM_BN_RED_SLAB=0
