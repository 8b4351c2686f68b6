#!/bin/bash
# persistent LSTM recurrence: numerics, then GNMT step time (hipGraph) + a kernel profile
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "persistent or lstm" > gpurun_out/lstm_test.log 2>&1 || { tail -40 gpurun_out/lstm_test.log; exit 1; }
tail -3 gpurun_out/lstm_test.log
timeout -k 10 240 python -u tools/bench_models.py --models gnmt --graph --steps 20 --warmup 3 > gpurun_out/lstm_bench.json 2> gpurun_out/lstm_bench.err || { tail -20 gpurun_out/lstm_bench.err; exit 1; }
cat gpurun_out/lstm_bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gnmt_persist -o run -- python3 tools/bench_models.py --models gnmt --steps 5 --warmup 2 > gpurun_out/prof_gnmt_persist.log 2>&1 || { tail -20 gpurun_out/prof_gnmt_persist.log; exit 1; }
find gpurun_out/prof_gnmt_persist -type f ! -name "*_stats.csv" -delete
head -12 $(find gpurun_out/prof_gnmt_persist -name "*kernel_stats.csv")
