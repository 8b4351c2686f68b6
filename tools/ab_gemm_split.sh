set -o pipefail
# cross-build A/B: base = the one-TU build (tiresias_amd/_C_base.so), split =
# one production gemm8p variant per TU (the in-tree _C.so); 3 alternating rounds
cd $GRAFT_REPO_ROOT; export PYTHONPATH=.
mkdir -p gpurun_out/s3
for r in 1 2 3; do
  for v in base split; do
    if [ $v = base ]; then export TAM_LIB_PATH=$PWD/tiresias_amd/_C_base.so; else unset TAM_LIB_PATH; fi
    timeout -k 10 120 python -u tools/gemm_shapes_tf.py $v >> gpurun_out/s3/ab_gemm_split.jsonl 2>/dev/null || exit 1
  done
done
unset TAM_LIB_PATH
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/s3/ab_gemm_split.jsonl"):
    r = json.loads(l); d[(r["shape"], r["lib"])].append(r["tflops"])
for (sh, lib), v in sorted(d.items()):
    print(f"{sh:22s} {lib:6s} max {max(v):7.1f} all {v}")
PY
