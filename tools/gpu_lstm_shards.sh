cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "persistent or lstm" > gpurun_out/lstm_test.log 2>&1 || { tail -40 gpurun_out/lstm_test.log; exit 1; }
tail -2 gpurun_out/lstm_test.log
timeout -k 10 300 python -u tools/ab_lstm_shards.py 1,2,4 > gpurun_out/lstm_shards.json 2> gpurun_out/lstm_shards.err || { tail -20 gpurun_out/lstm_shards.err; exit 1; }
cat gpurun_out/lstm_shards.json
