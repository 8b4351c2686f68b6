set -o pipefail
# Eager (the DDP gang compute path: no hipGraph, no weight-grad side stream,
# no branch streams) vs hipGraph step time per model on one MI355X.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
export PYTHONPATH=.
timeout -k 10 300 python -u tools/bench_models.py --steps 20 --warmup 3 --overlap 0 --branches 0 \
  > gpurun_out/r3/models_eager_gangpath.jsonl 2>&1
rc=$?; echo eager_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_models.py --steps 20 --warmup 3 --graph \
  > gpurun_out/r3/models_graph.jsonl 2>&1
rc=$?; echo graph_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_models.py --steps 20 --warmup 3 \
  > gpurun_out/r3/models_eager_default.jsonl 2>&1
rc=$?; echo eager2_rc=$rc; exit $rc
