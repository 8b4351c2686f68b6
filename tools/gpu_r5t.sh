#!/bin/bash
# round-5 GPU (t): re-tune the shipped GEMM routing table with the measured
# MFMA / hipBLASLt routing (production default now), then validate with it:
# same-box model A/B against MFMA-only, the GPU suite, the N=1 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
R=profiles/gemm_routes_gfx950_256cu.txt
cp $R gpurun_out/gemm_routes.txt
TAM_GEMM_ROUTES=0 timeout -k 10 400 python tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 10 --warmup 3 \
  --save_routes gpurun_out/gemm_routes.txt > gpurun_out/t_retune.log 2>&1
rc=$?; tail -3 gpurun_out/t_retune.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/gemm_routes.txt $R
AB_MODELS=resnet50,vgg16,transformer,gnmt bash tools/ab_rn50.sh base lib0=TAM_GEMM_LIB=0 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_suite.out 2>&1
rc=$?; tail -3 gpurun_out/t_suite.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/t_bench1.out 2> gpurun_out/t_bench1.err
rc=$?; tail -1 gpurun_out/t_bench1.out | cut -c1-300; exit $rc
