set -o pipefail
# Session-3: GPU suite, ResNet-50 step, colsum A/B, Transformer op budget, graph profiles
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/pytest_bn.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/s3/pytest_bn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_models.py --models resnet50,vgg16,transformer,gnmt --graph --steps 20 --warmup 3 > gpurun_out/s3/models_bn1.jsonl 2>&1
rc=$?; grep -v amdgpu gpurun_out/s3/models_bn1.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ab_colsum.py --out gpurun_out/s3/ab_colsum.json > gpurun_out/s3/ab_colsum.log 2>&1
rc=$?; cat gpurun_out/s3/ab_colsum.log | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
bash tools/ab_gemm_split.sh > gpurun_out/s3/ab_gemm_split.txt 2>&1
rc=$?; cat gpurun_out/s3/ab_gemm_split.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/trace_ops.py --model transformer --top 40 --out gpurun_out/s3/ops_tr.json > gpurun_out/s3/ops_tr.log 2>&1
rc=$?; tail -45 gpurun_out/s3/ops_tr.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_graph.sh resnet50 transformer
