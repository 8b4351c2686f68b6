cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread -k "batchnorm or conv or resnet or graph_capture or wgrad_stream or dgrad_epilogue" > gpurun_out/rn_test.log 2>&1 || { tail -40 gpurun_out/rn_test.log; exit 1; }
tail -2 gpurun_out/rn_test.log
timeout -k 10 200 python -u tools/bench_models.py --models resnet50 --graph --steps 20 --warmup 3 2>/dev/null | head -1 | cut -c1-150
timeout -k 10 200 python -u tools/bench_models.py --models resnet50 --graph --steps 20 --warmup 3 2>/dev/null | head -1 | cut -c1-150
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o run -- python3 tools/bench_models.py --models resnet50 --steps 5 --warmup 2 > gpurun_out/prof_rn50.log 2>&1 || { tail -20 gpurun_out/prof_rn50.log; exit 1; }
find gpurun_out/prof_rn50 -type f ! -name "*_stats.csv" -delete
