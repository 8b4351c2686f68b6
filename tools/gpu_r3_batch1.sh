set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_gemm.sh && bash tools/gpu_r3_scen.sh
