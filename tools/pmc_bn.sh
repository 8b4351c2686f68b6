#!/bin/bash
# HBM bytes of ResNet-50's BatchNorm passes (tools/bench_bn.py shapes): one
# rocprofv3 PMC pass for FETCH_SIZE and one for WRITE_SIZE (TCC block limit:
# 4 counters per pass), each under its own SIGKILL limit; per-dispatch bytes
# joined by dispatch order and divided by the dispatch duration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/pmc_bn
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/$c -o run -- python3 tools/bench_bn.py --reps 3 > $OUT/$c.log 2>&1
  rc=$?
  echo "pass $c rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/$c.log; exit $rc; }
done
python3 tools/pmc_bn_summary.py $OUT > $OUT/summary.txt
find $OUT -name "*.db" -delete
cat $OUT/summary.txt
