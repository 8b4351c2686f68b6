set -o pipefail
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.; mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/pytest_wip.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/s3/pytest_wip.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/ab_vgg_c64.py 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python -u tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 20 --warmup 3 > gpurun_out/s3/models_wip.jsonl 2>&1
rc=$?; grep model gpurun_out/s3/models_wip.jsonl | cut -c1-130; exit $rc
