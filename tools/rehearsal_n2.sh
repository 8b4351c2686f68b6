#!/bin/bash
# N=2 rehearsal of the multi-rank runtime on the ONE-GPU box (both ranks on
# cuda:0, communicators over gloo): fill mode on / off, plus the N=1 bench at
# two scheduling quanta. Each GPU step has its own time limit; a failing step
# ends the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
run() {  # run <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 3 "gpurun_out/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
N2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-nopool-replay"
for mode in "$@"; do
  case $mode in
    n2fill) run n2_fill 400 env TAM_SHARED_GPU=1 TAM_FILL=1 $N2 ;;
    n2nofill) run n2_nofill 400 env TAM_SHARED_GPU=1 TAM_FILL=0 $N2 ;;
    n1q20) run n1_q20 300 python bench.py --steps 5 --warmup 2 --quantum 0.02 --no-nopool-replay ;;
    n1q10) run n1_q10 300 python bench.py --steps 5 --warmup 2 --quantum 0.01 --no-nopool-replay ;;
  esac
done
