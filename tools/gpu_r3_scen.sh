set -o pipefail
# BASELINE configs 2-4 at N=1 with statistical weight (>= 10 timed replays).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
for sc in seq skew resnet4; do
  timeout -k 10 300 python -u bench.py --gpus 1 --scenario $sc --steps 10 --warmup 1 --no-nopool-replay \
    --budget-s 280 > gpurun_out/r3/scen_$sc.json 2> gpurun_out/r3/scen_$sc.err
  rc=$?; echo ${sc}_rc=$rc; [ $rc -eq 0 ] || exit $rc
done
