#!/bin/bash
# Per-model rocprofv3 kernel stats (one run per model; trace CSVs deleted).
# usage: tools/prof_models.sh <outdir-name> [models...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=$1; shift
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  out="$ROOT/gpurun_out/$name/$m"
  mkdir -p "$out"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 "$ROOT/tools/bench_models.py" --models "$m" --steps 10 --warmup 3 > "$out/log.txt" 2>&1
  rc=$?
  find "$out" -type f -name "*trace*.csv" -delete
  if [ $rc -ne 0 ]; then echo "model $m rc=$rc"; exit $rc; fi
done
