set -o pipefail
# Session-2 GPU check: focused tests (-k), then the GPU suite, then graph-mode
# model step times. usage: gpurun -- bash tools/gpu_s2_check.sh <tag> "<-k expr>" "<models>"
tag=${1:-v1}; kexpr=${2:-batchnorm or bn_ or resnet}; models=${3:-resnet50}
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr" \
  > gpurun_out/s2/focus_$tag.log 2>&1
rc=$?; echo focus_rc=$rc; tail -3 gpurun_out/s2/focus_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/s2/pytest_gpu_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/s2/pytest_gpu_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_models.py --models $models --graph --steps 20 --warmup 3 \
  > gpurun_out/s2/models_$tag.jsonl 2>&1
rc=$?; echo models_rc=$rc; cat gpurun_out/s2/models_$tag.jsonl | grep -v amdgpu.ids; exit $rc
