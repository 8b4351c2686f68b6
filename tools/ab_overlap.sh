cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
for m in transformer resnet50 gnmt; do
  for ov in 0 1 0 1; do
    timeout -k 10 120 python -u tools/bench_models.py --models $m --graph --steps 20 --warmup 3 --overlap $ov 2>/dev/null | head -1 | cut -c1-140 >> gpurun_out/ab_overlap.txt || exit 1
  done
done
for mm in 1048576 131072 1048576 131072; do
  TAM_DGRAD64_MIN_M=$mm timeout -k 10 120 python -u tools/bench_models.py --models resnet50 --graph --steps 20 --warmup 3 2>/dev/null | head -1 | cut -c1-120 | sed "s/^/dg64=$mm /" >> gpurun_out/ab_overlap.txt || exit 1
done
