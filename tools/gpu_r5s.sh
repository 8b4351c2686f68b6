#!/bin/bash
# round-5 GPU (s): measured MFMA / hipBLASLt routing for plain GEMMs (--lib -1)
# vs our kernels only (--lib 0), both re-tuned from scratch, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TAM_GEMM_ROUTES=0
for rep in 1 2; do
  for lib in 0 -1; do
    timeout -k 10 300 python tools/bench_models.py --models transformer,gnmt,vgg16 --graph --steps 30 --warmup 5 --lib $lib \
      > gpurun_out/lib_${lib}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "lib $lib rc=$rc"; tail -5 gpurun_out/lib_${lib}_$rep.log; exit $rc; }
    grep -o '"model": "[a-z0-9]*".*"ms_per_step": [0-9.]*' gpurun_out/lib_${lib}_$rep.log | sed "s/^/lib$lib $rep /"
    grep "plain-GEMM shapes" gpurun_out/lib_${lib}_$rep.log
  done
done
