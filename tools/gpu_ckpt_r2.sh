#!/bin/bash
# round-2 preemption-state check: async spill test, then the seq scenario
# (Gittins + HBM-pressure spills on a 16-job Transformer/GNMT trace) vs FIFO
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "ckpt or spill" --timeout 120 --timeout-method thread > gpurun_out/ckpt_test.log 2>&1 || { tail -30 gpurun_out/ckpt_test.log; exit 1; }
tail -1 gpurun_out/ckpt_test.log
timeout -k 10 300 python -u bench.py --scenario seq --steps 2 --warmup 1 --hbm-budget-gb 12 > gpurun_out/seq_pressure.json 2> gpurun_out/seq_pressure.err || { tail -20 gpurun_out/seq_pressure.err; exit 1; }
grep "\[bench\]" gpurun_out/seq_pressure.err
python3 -c "import json; d=json.load(open('gpurun_out/seq_pressure.json')); print({k: d[k] for k in ['value','vs_baseline','baseline_avg_jct_s','pressure_spills','spilled_gb','finished_jobs','preemptions']})"
