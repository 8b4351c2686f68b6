#!/bin/bash
# round-2 GEMM check: gemm8p numerics, GEMM bench, model steps with / without hipBLASLt
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/p8_test.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/p8_test.log; exit 1; }
tail -2 gpurun_out/p8_test.log
timeout -k 10 300 python -u tools/bench_gemm8p.py --out gpurun_out/p8_bench3.json > gpurun_out/p8_bench3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/p8_bench3.log
for lib in -1 0; do
  timeout -k 10 300 python -u tools/bench_models.py --graph --lib $lib --out gpurun_out/models_lib$lib.json > gpurun_out/models_lib$lib.log 2>&1 || { tail -20 gpurun_out/models_lib$lib.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/models_lib$lib.log | grep -v "^ " | head -8
done
