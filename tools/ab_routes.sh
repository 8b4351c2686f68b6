#!/bin/bash
# re-tune the GEMM routing table on this tree from the four models' own calls
# (cold process, TAM_GEMM_ROUTES=0, every shape timed over its candidates),
# then a same-box interleaved A/B of the shipped table (old) vs the re-tuned
# one (new): AB_MODELS graph steps, 2 reps. The new table lands in
# gpurun_out/routes_retuned.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=${AB_MODELS:-transformer,gnmt,resnet50,vgg16}
rm -f gpurun_out/routes_retuned.txt
TAM_GEMM_ROUTES=0 timeout -k 10 300 python tools/bench_models.py --models $M --graph --steps 10 --warmup 3 \
  --save_routes gpurun_out/routes_retuned.txt > gpurun_out/retune.log 2>&1 || { tail -5 gpurun_out/retune.log; exit 1; }
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then unset TAM_GEMM_ROUTES; else export TAM_GEMM_ROUTES=gpurun_out/routes_retuned.txt; fi
    timeout -k 10 300 python tools/bench_models.py --models $M --graph --steps 30 --warmup 5 \
      > gpurun_out/abr_${v}_$rep.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/abr_${v}_$rep.log; exit $rc; }
    grep -o '"model": "[a-z0-9]*".*"ms_per_step": [0-9.]*' gpurun_out/abr_${v}_$rep.log | sed "s/^/$v $rep /"
  done
done
