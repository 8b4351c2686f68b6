# round-4 GPU check: multi-rank tests, skinny GEMM numerics + route bench, BN bench, grouped-GEMM PMC passes
set -o pipefail; R=$GRAFT_REPO_ROOT; O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or gemm_layouts" > $O/pytest_skinny.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_gemm_routes.py --out $O/routes.json > $O/routes.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multigpu.py tests/test_models_gpu.py::test_persist_barrier_timeout_is_loud_and_falls_back tests/test_models_gpu.py::test_optimizer_guard_is_per_job > $O/pytest.log 2>&1; echo rc=$? >> $O/pytest.log
timeout -k 10 120 python -u tools/bench_bn.py --out $O/bn.json > $O/bn.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do tag=$(echo $pass | cut -d" " -f1); PYTHONPATH=$R timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --stats --output-format csv -d $R/$O/pmc_$tag -o run -- python3 $R/tools/bench_grouped.py --only grouped --reps 5 > $R/$O/pmc_$tag.log 2>&1 || exit 1; done
