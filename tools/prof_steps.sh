cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_rn $R/gpurun_out/prof_gn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o rn -- python3 $R/tools/bench_models.py --models resnet50 --graph --steps 20 --warmup 5 > $R/gpurun_out/prof_rn.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gn -o gn -- python3 $R/tools/bench_models.py --models gnmt --graph --steps 20 --warmup 5 > $R/gpurun_out/prof_gn.log 2>&1
