set -o pipefail
# Session-3 full check: focused tests first, then the GPU suite, the four
# models' graph steps, optional graph profiles
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.
mkdir -p gpurun_out/s3
tag=${1:-v}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${2:-colsum}" > gpurun_out/s3/focus_$tag.log 2>&1
rc=$?; echo focus_rc=$rc; tail -2 gpurun_out/s3/focus_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/pytest_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/s3/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 20 --warmup 3 > gpurun_out/s3/models_$tag.jsonl 2>&1
rc=$?; grep -v amdgpu gpurun_out/s3/models_$tag.jsonl | cut -c1-150 | grep model; [ $rc -eq 0 ] || exit $rc
if [ -n "$3" ]; then bash tools/prof_graph.sh $3; exit $?; fi
