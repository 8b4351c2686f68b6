set -o pipefail
# Cold-start costs: per-model trainer build / first steps in a fresh process
# WITHOUT and WITH the pre-loaded GEMM routing table (the first run writes it).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
export PYTHONPATH=.
TAM_GEMM_ROUTES=gpurun_out/r3/gemm_routes.txt timeout -k 10 300 python -u tools/job_startup.py --save-routes \
  > gpurun_out/r3/startup_noroutes.jsonl 2>gpurun_out/r3/startup_noroutes.err
rc=$?; echo startup1_rc=$rc; [ $rc -eq 0 ] || exit $rc
TAM_GEMM_ROUTES=gpurun_out/r3/gemm_routes.txt timeout -k 10 300 python -u tools/job_startup.py \
  > gpurun_out/r3/startup_routes.jsonl 2>gpurun_out/r3/startup_routes.err
rc=$?; echo startup2_rc=$rc; exit $rc
