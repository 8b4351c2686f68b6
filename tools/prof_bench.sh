#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench replay; keeps only the summary
# CSVs (the per-dispatch trace is deleted so gpurun_out stays < 64 MiB).
# usage: tools/prof_bench.sh <outdir-name> [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=$1; shift
out="$ROOT/gpurun_out/$name"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 "$ROOT/bench.py" "$@" > "$out/bench.log" 2>&1
rc=$?
find "$out" -type f -name "*trace*.csv" -delete
find "$out" -type f -size +8M -printf "%s %p (deleted)\n" -delete >> "$out/bench.log"
find "$out" -type f -printf "%s %p\n" >> "$out/bench.log"
exit $rc
