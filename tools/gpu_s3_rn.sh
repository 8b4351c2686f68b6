set -o pipefail
# Session-3 ResNet-50 BN iteration: BN / conv GPU tests, model step, graph profile
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.
mkdir -p gpurun_out/s3
tag=${1:-v}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or batchnorm or resnet or colsum or bias" > gpurun_out/s3/focus_$tag.log 2>&1
rc=$?; echo focus_rc=$rc; tail -2 gpurun_out/s3/focus_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_models.py --models ${2:-resnet50} --graph --steps 20 --warmup 3 > gpurun_out/s3/models_$tag.jsonl 2>&1
rc=$?; grep -v amdgpu gpurun_out/s3/models_$tag.jsonl | cut -c1-150 | grep model; [ $rc -eq 0 ] || exit $rc
bash tools/prof_graph.sh ${3:-resnet50}
