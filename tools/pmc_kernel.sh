#!/bin/bash
# PMC passes over one kernel family of any program:
#   bash tools/pmc_kernel.sh <name> <kernel-substring> <python args...>
# e.g. bash tools/pmc_kernel.sh halo conv_halo tools/bench_models.py --models vgg16 --graph --steps 3 --warmup 1
# L2 hits / misses, bytes beyond L2, where the waves wait, instruction mix.
# One counter group per pass, each under its own SIGKILL limit; a failing
# pass ends the script. Medians per dispatch in gpurun_out/pmc_<name>/summary.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
NAME=$1; MATCH=$2; shift 2
OUT=gpurun_out/pmc_$NAME
mkdir -p $OUT
P1="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
P4="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P5="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
i=0
for pass in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/p$i -o run -- python3 "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT "$MATCH" > $OUT/summary.txt
find $OUT -name "*.db" -delete
cat $OUT/summary.txt
