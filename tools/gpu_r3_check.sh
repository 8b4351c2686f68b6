set -o pipefail
# Round-3 GPU validation: GPU tests, then the 1-GPU headline bench.
# usage: gpurun -- bash tools/gpu_r3_check.sh <tag>
tag=${1:-v1}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3/pytest_gpu_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/r3/bench_$tag.json 2> gpurun_out/r3/bench_$tag.err
rc=$?; echo bench_rc=$rc
exit $rc
