#!/bin/bash
# Per-model rocprofv3 kernel statistics (one run per model, eager steps).
# Run on the GPU box from the repo root:  bash tools/prof_models.sh [models...]
set -o pipefail
export TMPDIR=/tmp
models="${*:-resnet50 vgg16 transformer gnmt}"
for m in $models; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o run -- \
    python3 tools/bench_models.py --models $m --steps 5 --warmup 2 > gpurun_out/log_prof_$m.txt 2>&1 || { tail -20 gpurun_out/log_prof_$m.txt; exit 1; }
done
# keep only the summaries (the full traces exceed what gpurun copies back)
find gpurun_out -path "*/prof_*" -type f ! -name "*_stats.csv" -delete
find gpurun_out -name "*kernel_stats.csv"
