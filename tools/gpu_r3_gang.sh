set -o pipefail
# Round-3 gang-lifecycle checks on one MI355X: RCCL GangPG / PGCache
# lifecycle (warm, abort, re-create), then the 2-rank shared-GPU rehearsal of
# the multi-rank bench path (canonical comm pre-creation, pair-PG state moves,
# move agreement) -- gloo gang transport because RCCL refuses two ranks/GPU.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
PYTHONPATH=. timeout -k 10 120 python -u tools/gpu_rccl_smoke.py > gpurun_out/r3/rccl_smoke.log 2>&1
rc=$?; echo rccl_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k persist_barrier > gpurun_out/r3/persist_timeout.log 2>&1
rc=$?; echo persist_rc=$rc; [ $rc -eq 0 ] || exit $rc
TAM_SHARED_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 1 --warmup 1 --jobs-per-gpu 12 \
  > gpurun_out/r3/shared2.json 2> gpurun_out/r3/shared2.err
rc=$?; echo shared2_rc=$rc
exit $rc
