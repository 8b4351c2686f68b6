#!/bin/bash
# Host sanitizers over the native control-plane code.
#  * ASan + UBSan: the event core (csrc/sched_core) replayed for every policy.
#  * The checkpoint engine's pinned host pool (tam/pinned_pool.h) hammered by
#    concurrent threads under ASan + UBSan and under ThreadSanitizer.
#  * The checkpoint engine's host code (csrc/ckpt) is compiled with host-only
#    ASan/UBSan (-Xarch_host) as a build check; it needs a GPU to run.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/tam_sanitize}"
mkdir -p "$OUT"
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all \
  "$ROOT/csrc/sched_core/sanitize_main.cpp" -o "$OUT/sched_core_asan"
ASAN_OPTIONS=detect_leaks=1:verify_asan_link_order=0 UBSAN_OPTIONS=print_stacktrace=1 \
  "$OUT/sched_core_asan" "${N_JOBS:-400}"
# checkpoint engine's pinned pool (host-only header): ASan+UBSan, then TSan
g++ -O1 -g -std=c++17 -pthread -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all \
  -I"$ROOT/csrc/include" "$ROOT/csrc/sanitize/pool_sanitize_main.cpp" -o "$OUT/pool_asan"
ASAN_OPTIONS=detect_leaks=1 "$OUT/pool_asan" 4 2000
g++ -O1 -g -std=c++17 -pthread -fsanitize=thread -fno-omit-frame-pointer \
  -I"$ROOT/csrc/include" "$ROOT/csrc/sanitize/pool_sanitize_main.cpp" -o "$OUT/pool_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/pool_tsan" 4 2000
if [ "${SKIP_HIP:-0}" != "1" ] && command -v /opt/rocm/bin/hipcc >/dev/null; then
  TORCH_INC=$(python3 -c "import torch.utils.cpp_extension as c; print(' '.join('-I'+p for p in c.include_paths()))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O1 -g -fPIC -Xarch_host -fsanitize=address \
    -Xarch_host -fsanitize=undefined $TORCH_INC -I"$ROOT/csrc/include" \
    -c "$ROOT/csrc/ckpt/ckpt_engine.cpp" -o "$OUT/ckpt_engine_asan.o"
  echo "ckpt engine host-ASan/UBSan build OK"
fi
