# rocprofv3 kernel stats of the hipGraph train steps: bash tools/prof_steps.sh [models...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in ${@:-resnet50 gnmt}; do
  mkdir -p $R/gpurun_out/prof_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$m -o $m -- python3 $R/tools/bench_models.py --models $m --graph --steps 20 --warmup 5 > $R/gpurun_out/prof_$m.log 2>&1 || exit $?
done
