#!/bin/bash
# same-box A/B of two builds of the extension: tiresias_amd/_C_old.so (A)
# vs the in-tree _C.so (B), interleaved, AB_MODELS graph steps each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp tiresias_amd/_C.so gpurun_out/_C_new.so
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp tiresias_amd/_C_old.so tiresias_amd/_C.so; else cp gpurun_out/_C_new.so tiresias_amd/_C.so; fi
    timeout -k 10 200 python tools/bench_models.py --models ${AB_MODELS:-transformer} --graph --steps 30 --warmup 5 \
      > gpurun_out/abso_${v}_$rep.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abso_${v}_$rep.log; cp gpurun_out/_C_new.so tiresias_amd/_C.so; exit $rc; }
    grep -o '"model": "[a-z0-9]*".*"ms_per_step": [0-9.]*' gpurun_out/abso_${v}_$rep.log | sed "s/^/$v $rep /"
  done
done
cp gpurun_out/_C_new.so tiresias_amd/_C.so
rm -f gpurun_out/_C_new.so
