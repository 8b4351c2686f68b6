# conv split-K numerics + ResNet-50 A/B (split on/off) + rocprof of the split step; stream-K vs split-K sweep
set -o pipefail; R=$GRAFT_REPO_ROOT; O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/pytest.log 2>&1 || exit 1
for sp in 1 0 1 0; do timeout -k 10 200 python -u tools/bench_models.py --graph --models resnet50 --steps 30 --warmup 5 --conv_split $sp >> $O/rn50_ab.log 2>&1 || exit 1; done
timeout -k 10 300 python -u tools/bench_streamk.py --out $O/streamk.json > $O/streamk.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_rn50 -o run -- python3 $R/tools/bench_models.py --graph --models resnet50 --steps 20 --warmup 5 > $R/$O/prof_rn50.log 2>&1 || exit 1
