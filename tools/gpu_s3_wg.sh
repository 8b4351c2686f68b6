set -o pipefail
# conv / GEMM / LN / Transformer GPU tests, then the four models' graph steps
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.; mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or wgrad or resnet or vgg or gemm or colsum or layernorm or transformer" > gpurun_out/s3/focus_wg.log 2>&1
rc=$?; echo focus_rc=$rc; tail -2 gpurun_out/s3/focus_wg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 20 --warmup 3 > gpurun_out/s3/models_wg.jsonl 2>&1
rc=$?; grep model gpurun_out/s3/models_wg.jsonl | cut -c1-140; exit $rc
