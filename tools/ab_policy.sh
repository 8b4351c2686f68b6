# usage: bash tools/ab_policy.sh <models> <policy_name> <a> <b> [rounds]
# interleaved in-box A/B of one torch.ops.tam policy switch on the graph steps
cd ${GRAFT_REPO_ROOT:-.}
M=$1; P=$2; A=$3; B=$4; R=${5:-2}
for i in $(seq $R); do
for v in $A $B; do
timeout -k 10 300 python tools/bench_models.py --models $M --graph --steps 30 --warmup 5 --policy $P=$v > gpurun_out/ab_$v.log 2>&1 || exit $?
echo "$P=$v $(grep -o '"model": "[a-z0-9]*"\|"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log | tr '\n' ' ')"
done; done
