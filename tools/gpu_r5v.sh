#!/bin/bash
# round-5 GPU (v): final checkpoint with the re-tuned routing -- step traces
# of the four models, smoke, N=2 shared-GPU rehearsal (suite and N=1 bench
# ran in gpu_r5t.sh on the same code)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TRACE_MODELS="resnet50 transformer gnmt vgg16" bash tools/gpu_trace3.sh || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/v_smoke.out 2>&1
rc=$?; tail -2 gpurun_out/v_smoke.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env TAM_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-nopool-replay > gpurun_out/v_n2.out 2> gpurun_out/v_n2.err
rc=$?; grep '^{"metric"' gpurun_out/v_n2.out | tail -1 | cut -c1-300; exit $rc
