#!/bin/bash
# SQ instruction-mix PMC passes over every kernel of each model's eager train
# step (where VALU, LDS or waits dominate): bash tools/pmc_models.sh [models...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
for m in ${@:-resnet50 vgg16 transformer gnmt}; do
  OUT=gpurun_out/pmcm_$m
  mkdir -p $OUT
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $pass -d $OUT/p$i -o run -- python3 tools/bench_models.py --models $m --steps 2 --warmup 1 > $OUT/p$i.log 2>&1
    rc=$?
    echo "$m pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
  done
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
  find $OUT -name "*.db" -delete
done
