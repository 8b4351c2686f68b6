#!/bin/bash
# PMC passes over the persistent LSTM forward / backward (GNMT shapes,
# tools/bench_lstm_pair.py --one): L2 hits vs misses and bytes fetched beyond
# L2, and where the waves wait. One counter group per pass, each under its
# own SIGKILL limit; a failing pass ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/pmc_lstm
mkdir -p $OUT
P1="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P2="FETCH_SIZE"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"
P4="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA"
i=0
for pass in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $OUT/p$i -o run -- python3 tools/bench_lstm_pair.py --one > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT lstm_persist > $OUT/summary.txt
find $OUT -name "*.db" -delete
cat $OUT/summary.txt
