set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
export PYTHONPATH=.
timeout -k 10 400 python -u tools/bench_gemm_routes.py --out gpurun_out/r3/gemm_routes_vs_lib.json \
  > gpurun_out/r3/gemm_routes_vs_lib.log 2>&1
rc=$?; echo routes_rc=$rc; exit $rc
