#!/bin/bash
# rocprofv3 kernel statistics of one headline trace replay (1 GPU).
# Run on the GPU box from the repo root:  bash tools/prof_bench.sh
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-baseline --no-exclusive-ref > gpurun_out/log_prof_bench.txt 2>&1 \
  || { tail -20 gpurun_out/log_prof_bench.txt; exit 1; }
find gpurun_out/prof_bench -type f ! -name "*_stats.csv" -delete
grep -h metric gpurun_out/log_prof_bench.txt | cut -c 1-200
