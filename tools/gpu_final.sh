#!/bin/bash
# full GPU checkpoint: the GPU suite (as the driver runs it), smoke, the N=1
# headline bench (driver defaults) and the N=2 shared-GPU rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
run() {
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 3 "gpurun_out/$name.out"; tail -n 3 "gpurun_out/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
run suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench1 400 python bench.py
run n2 400 env TAM_SHARED_GPU=1 TAM_STACK_DUMP_S=45 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-nopool-replay
