set -o pipefail
# PMC passes on the p8 GEMM: K-major (KK) vs transposed-read (MN) operands at 4096^3
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3/pmc
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/r3/pmc/avail.txt 2>&1; echo list_rc=$?
for lay in KK MN KN; do
  for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM"; do
    tag=$(echo $pass | cut -d' ' -f1)
    PYTHONPATH=$R timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-trace --stats -d $R/gpurun_out/r3/pmc/${lay}_$tag -o run \
      -- python3 $R/tools/gemm_one.py 4096 4096 4096 $lay 20 > $R/gpurun_out/r3/pmc/${lay}_$tag.log 2>&1
    echo ${lay}_${tag}_rc=$?
  done
done
