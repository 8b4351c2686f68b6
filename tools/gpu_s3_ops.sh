set -o pipefail
# per-op budget of one eager step (tools/trace_ops.py) for the listed models
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.; mkdir -p gpurun_out/s3
for m in ${1:-resnet50}; do
  timeout -k 10 300 python -u tools/trace_ops.py --model $m --top 60 --out gpurun_out/s3/ops_$m.json > gpurun_out/s3/ops_$m.log 2>&1
  rc=$?; grep "^#" gpurun_out/s3/ops_$m.log | head -14; [ $rc -eq 0 ] || exit $rc
done
