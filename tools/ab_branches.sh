# interleaved A/B of model branch streams: bash tools/ab_branches.sh <model> [rounds]
cd ${GRAFT_REPO_ROOT:-.}
M=$1; R=${2:-2}
for i in $(seq $R); do
for v in 0 1; do
timeout -k 10 300 python tools/bench_models.py --models $M --graph --steps 30 --warmup 5 --branches $v > gpurun_out/abb_$v.log 2>&1 || exit $?
echo "branches=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abb_$v.log)"
done; done
