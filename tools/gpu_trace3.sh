#!/bin/bash
# per-call kernel traces of the ResNet-50 / Transformer / GNMT graph steps
# (layer attribution; summaries by tools/trace_step.py --first xent_kernel)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for m in ${TRACE_MODELS:-resnet50 transformer gnmt}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$m -o run -- \
    python3 tools/bench_models.py --models $m --graph --steps 3 --warmup 2 > gpurun_out/trace_$m.log 2>&1
  rc=$?; echo "$m trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/trace_$m.log; exit $rc; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/trace_$m.log
  find gpurun_out/trace_$m -name "*.db" -delete
  python3 tools/trace_step.py gpurun_out/trace_$m/run_kernel_trace.csv --first xent_kernel > gpurun_out/trace_$m.summary.txt
  head -30 gpurun_out/trace_$m.summary.txt
done
