cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD TMPDIR=/tmp
for i in 1 2; do
for v in base new; do
  if [ $v = base ]; then export TAM_LIB_PATH=$PWD/tiresias_amd/_C_base.so; else unset TAM_LIB_PATH; fi
  timeout -k 10 120 python -u tools/bench_models.py --models gnmt --graph --steps 20 --warmup 3 2>/dev/null | head -1 | sed "s/^/$v /" >> gpurun_out/ab_lstm.txt || exit 1
done
done
