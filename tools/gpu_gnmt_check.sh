cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread -k "gnmt or lstm or persistent" > gpurun_out/gnmt_test.log 2>&1 || { tail -40 gpurun_out/gnmt_test.log; exit 1; }
tail -2 gpurun_out/gnmt_test.log
timeout -k 10 240 python -u tools/bench_models.py --models gnmt --graph --steps 20 --warmup 3 2> gpurun_out/gnmt_bench.err | head -1
