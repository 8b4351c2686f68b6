#!/bin/bash
# ResNet-50 graph-step A/B over environment knobs: one bench_models run per
# variant (args: "NAME=VAR=VAL[,VAR=VAL]" ...; "base" = no override).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  [ "$name" = "$spec" ] && envs=""
  for rep in 1 2; do
    timeout -k 10 200 env ${envs//,/ } python tools/bench_models.py --models ${AB_MODELS:-resnet50} --graph --steps 30 --warmup 5 \
      > gpurun_out/ab_${name}_$rep.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/ab_${name}_$rep.log; exit $rc; }
    grep -o '"model": "[a-z0-9]*".*"ms_per_step": [0-9.]*' gpurun_out/ab_${name}_$rep.log | sed "s/^/$name $rep /"
  done
done
