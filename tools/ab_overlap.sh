# interleaved A/B of the weight-gradient side stream on one model: bash tools/ab_overlap.sh <model> [rounds]
cd ${GRAFT_REPO_ROOT:-.}
M=$1; R=${2:-2}
for i in $(seq $R); do
for v in 0 1; do
timeout -k 10 300 python tools/bench_models.py --models $M --graph --steps 30 --warmup 5 --overlap $v > gpurun_out/abo_$v.log 2>&1 || exit $?
echo "overlap=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abo_$v.log)"
done; done
