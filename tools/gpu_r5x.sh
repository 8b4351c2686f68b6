#!/bin/bash
# round-5 GPU (x): headline N=1 bench, exclusive GPUs (default) vs GPU
# sharing when full (--share), same box, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
for rep in 1 2; do
  for v in excl share; do
    extra=""; [ $v = share ] && extra="--share"
    timeout -k 10 400 python bench.py $extra > gpurun_out/x_${v}_$rep.out 2> gpurun_out/x_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/x_${v}_$rep.err; exit $rc; }
    echo "$v $rep $(grep '^{"metric"' gpurun_out/x_${v}_$rep.out | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("makespan_s"), d.get("baseline_avg_jct_s"))')"
  done
done
