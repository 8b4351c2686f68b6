#!/bin/bash
# GPU smoke/numerics/bench driver for gpurun. Each GPU step has its own time
# limit; a fault / abort / timeout stops the script (no further GPU steps).
# usage: tools/gpu_check.sh "<pytest args>" "<extra python cmd>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout> <cmd...>
  local name=$1; local lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after rc=$rc (fault/abort/timeout)"; exit $rc
  fi
  return 0
}
for spec in "$@"; do
  name=${spec%%::*}; rest=${spec#*::}; lim=${rest%%::*}; cmd=${rest#*::}
  step "$name" "$lim" bash -c "$cmd" || exit $?
done
