cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or transformer or vgg or linear" > gpurun_out/mask_test.log 2>&1 || { tail -40 gpurun_out/mask_test.log; exit 1; }
tail -2 gpurun_out/mask_test.log
timeout -k 10 240 python -u tools/bench_models.py --models transformer,vgg16 --graph --steps 20 --warmup 3 2> /dev/null | grep -v "^[0-9]" | head -3 | cut -c1-160
timeout -k 10 240 python -u tools/bench_models.py --models transformer --graph --steps 20 --warmup 3 2> /dev/null | grep "4096 2048 512\|4096 512 2048" 
