set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r2_v2.log 2>&1; echo pytest_rc=$?
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r2_v3.json 2> gpurun_out/bench_r2_v3.err; echo bench_rc=$?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench_r2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 3 --warmup 1 --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_r2.log 2>&1; echo prof_rc=$?
