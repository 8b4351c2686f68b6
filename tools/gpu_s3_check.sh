set -o pipefail
# Session-3 GPU check: GPU suite, smoke, graph-mode step time of the four
# models, then the headline bench. usage: gpurun -- bash tools/gpu_s3_check.sh <tag> [bench=1] ["prof models"]
tag=${1:-v1}; bench=${2:-1}
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/s3/pytest_gpu_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/s3/pytest_gpu_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke_$tag.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/s3/smoke_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 20 --warmup 3 \
  > gpurun_out/s3/models_$tag.jsonl 2>&1
rc=$?; echo models_rc=$rc; grep -v amdgpu.ids gpurun_out/s3/models_$tag.jsonl; [ $rc -eq 0 ] || exit $rc
if [ "$bench" = 1 ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/s3/bench_$tag.json 2> gpurun_out/s3/bench_$tag.err
  rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/s3/bench_$tag.json; [ $rc -eq 0 ] || exit $rc
fi
# optional: graph-step kernel stats of the listed models
if [ -n "$3" ]; then bash tools/prof_graph.sh $3; exit $?; fi
exit 0
