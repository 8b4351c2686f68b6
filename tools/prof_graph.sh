#!/bin/bash
# per-model kernel stats under hipGraph replay: bash tools/prof_graph.sh model [model...]
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
for m in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profg_$m -o run -- python3 tools/bench_models.py --models $m --graph --steps 20 --warmup 3 > gpurun_out/profg_$m.log 2>&1 || { tail -20 gpurun_out/profg_$m.log; exit 1; }
  find gpurun_out/profg_$m -type f ! -name "*_stats.csv" -delete
  head -1 gpurun_out/profg_$m.log
done
