#!/bin/bash
# Job-submission API end to end on one MI355X: the live cluster serves a spool
# directory; jobs are submitted while it runs, their status polled, then the
# cluster is shut down once drained. Outputs land in gpurun_out/live_api/.
#   bash tools/live_api_demo.sh
set -o pipefail
SPOOL=$(mktemp -d /tmp/tam_spool.XXXX)
OUT=$PWD/gpurun_out/live_api
mkdir -p $OUT
timeout -k 10 240 python -u -m tiresias_amd.cli.run_cluster --spool $SPOOL --schedule dlas-gpu \
    --scheme tiresias --quantum 0.1 --log_path $OUT > $OUT/cluster.log 2>&1 &
CL=$!
sleep 2
python -m tiresias_amd.cli.submit --spool $SPOOL --model resnet50 --gpus 1 --iterations 300 --job-id r50
python -m tiresias_amd.cli.submit --spool $SPOOL --model transformer --gpus 1 --iterations 200 --job-id tfm
sleep 3
python -m tiresias_amd.cli.submit --spool $SPOOL --model vgg16 --gpus 1 --iterations 60 --job-id vgg
python -m tiresias_amd.cli.submit --spool $SPOOL --model gnmt --gpus 4 --iterations 10 --job-id too_big
for i in 1 2 3 4 5 6; do
  sleep 2
  python -m tiresias_amd.cli.submit --spool $SPOOL --status | tee -a $OUT/status.log | head -c 600
  echo
done
python -m tiresias_amd.cli.submit --spool $SPOOL --shutdown
wait $CL
rc=$?
echo "cluster exit $rc"
for d in accepted rejected; do
  echo "== $d"; for f in $SPOOL/$d/*; do [ -f "$f" ] && { echo "$(basename $f): $(head -c 300 $f)"; }; done
done | tee $OUT/spool_outcome.txt
tail -5 $OUT/cluster.log
exit $rc
