#!/bin/bash
# seq scenario (Gittins + HBM-pressure spills) vs FIFO, with and without an HBM budget
cd $GRAFT_REPO_ROOT
for B in ${BUDGETS:-12 0}; do
  extra=""; [ "$B" != "0" ] && extra="--hbm-budget-gb $B"
  timeout -k 10 300 python -u bench.py --scenario seq --steps 3 --warmup 1 $extra > gpurun_out/seq_b$B.json 2> gpurun_out/seq_b$B.err || { tail -20 gpurun_out/seq_b$B.err; exit 1; }
  grep "\[bench\]" gpurun_out/seq_b$B.err
  python3 -c "import json; d=json.load(open('gpurun_out/seq_b$B.json')); print({k: d.get(k) for k in ['value','vs_baseline','baseline_avg_jct_s','makespan_s','baseline_makespan_s','pressure_spills','pool_evictions','restore_prefetches','spilled_gb','preemptions','runtime_breakdown_s']})"
done
