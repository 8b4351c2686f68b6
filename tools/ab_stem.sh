cd $GRAFT_REPO_ROOT
for i in 1 2; do
for pol in 1 0; do
timeout -k 10 200 python tools/bench_models.py --models resnet50 --graph --steps 30 --warmup 5 --policy conv_stem_policy=$pol > gpurun_out/ab_$pol.log 2>&1 || exit $?
echo "stem=$pol $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$pol.log)"
done; done
