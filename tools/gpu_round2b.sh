#!/bin/bash
# full GPU suite + GNMT branch-stream A/B + headline bench (1 GPU)
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for br in 0 1; do
  timeout -k 10 200 python -u tools/bench_models.py --models gnmt --graph --steps 20 --warmup 3 --branches $br > gpurun_out/gnmt_br$br.json 2> gpurun_out/gnmt_br$br.err || { tail -20 gpurun_out/gnmt_br$br.err; exit 1; }
  head -1 gpurun_out/gnmt_br$br.json
done
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
