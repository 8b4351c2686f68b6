#!/bin/bash
# round-5 GPU (g): N=2 shared-GPU rehearsal with finishing rounds (fill mode),
# then the N=1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
run() {
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== [$name] rc=$rc"; grep '^\[bench\]' "gpurun_out/$name.out" | tail -n 6; tail -n 3 "gpurun_out/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
run n2 400 env TAM_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-nopool-replay
run n1 300 python bench.py --steps 5 --warmup 2 --no-nopool-replay
