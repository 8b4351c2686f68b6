#!/bin/bash
# PMC passes over the grouped weight-gradient launch (Transformer-base problem
# set, tools/bench_grouped.py) and, for comparison, the 128^2 gemm8p on a
# K-major 4096^3 GEMM. One counter group per pass (<= 8 SQ counters each);
# every pass under its own SIGKILL time limit; a failing pass ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/pmc_grouped
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL"
P3="SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
i=0
for pass in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  for what in grouped gemm; do
    if [ $what = grouped ]; then cmd="tools/bench_grouped.py --reps 3 --only grouped"; else cmd="tools/gemm_one.py 4096 4096 4096 MN 5 128"; fi
    timeout -s KILL 90 rocprofv3 --pmc $pass -d $OUT/p${i}_$what -o run -- python3 $cmd > $OUT/p${i}_$what.log 2>&1
    rc=$?
    echo "pass $i $what rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $OUT/p${i}_$what.log; exit $rc; }
  done
done
python3 tools/pmc_summary.py $OUT grouped > $OUT/summary_grouped.txt
python3 tools/pmc_summary.py $OUT gemm8p > $OUT/summary_gemm8p.txt
find $OUT -name "*.db" -delete
cat $OUT/summary_grouped.txt $OUT/summary_gemm8p.txt
