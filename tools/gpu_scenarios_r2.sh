#!/bin/bash
# BASELINE configs 2-4 as bench scenarios on one GPU (placement / gang effects need N >= 4)
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
for sc in resnet4 skew seq; do
  timeout -k 10 300 python -u bench.py --scenario $sc --steps 2 --warmup 1 > gpurun_out/sc_$sc.json 2> gpurun_out/sc_$sc.err || { tail -20 gpurun_out/sc_$sc.err; exit 1; }
  grep "\[bench\]" gpurun_out/sc_$sc.err | tail -2
  python3 -c "import json; d=json.load(open('gpurun_out/sc_$sc.json')); print('$sc', {k: d.get(k) for k in ['value','vs_baseline','makespan_s','baseline_makespan_s','preemptions','finished_jobs']})"
done
