set -o pipefail
# patch-staged wgrad + igemm fp32 epilogue: tests, full-size numerics, A/Bs
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.; mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "c64 or wgrad or conv_fwd_dgrad or vgg or gemm or colsum" > gpurun_out/s3/focus_c64b.log 2>&1
rc=$?; tail -3 gpurun_out/s3/focus_c64b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/check_wgrad_c64_scale.py 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python -u tools/sweep_wgrad.py --c64_ab --out gpurun_out/s3/ab_c64b.json 2>&1 | grep -v amdgpu || exit 1
bash tools/ab_fp32_epilogue.sh > gpurun_out/s3/ab_fp32ep.jsonl 2>&1; rc=$?; cat gpurun_out/s3/ab_fp32ep.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_vgg_c64.py 2>&1 | grep -v amdgpu
