set -o pipefail
# Where does a no-warm-pool replay's extra JCT come from? pool vs no-pool,
# with and without hipGraph capture of 1-GPU jobs (short runs, no baseline).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
for v in "pool:" "nopool:--no-pool" "nopool_nograph:--no-pool --no-graph" "pool_nograph:--no-graph"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 3 --warmup 1 --no-baseline --no-nopool-replay $args \
    > gpurun_out/r3/np_$tag.json 2> gpurun_out/r3/np_$tag.err
  rc=$?; echo ${tag}_rc=$rc; [ $rc -eq 0 ] || exit $rc
done
