# round-4 GPU check: stream-K / skinny numerics, re-tuned routing vs hipBLASLt, skinny sweep, 4096^3 protocols, model steps
set -o pipefail; O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "streamk or skinny or gemm8p_slab or test_gemm8p" > $O/pytest.log 2>&1 || exit 1
TAM_GEMM_ROUTES=0 timeout -k 10 400 python -u tools/bench_gemm_routes.py --out $O/routes.json --save $O/routes_new.txt > $O/routes.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_skinny.py --out $O/skinny.json > $O/skinny.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gemm_4096_protocols.py --out $O/gemm4096.json > $O/gemm4096.log 2>&1 || exit 1
TAM_GEMM_ROUTES=$O/routes_new.txt timeout -k 10 400 python -u tools/bench_models.py --graph --models vgg16,gnmt,transformer,resnet50 --steps 20 --warmup 5 --out $O/models.json > $O/models.log 2>&1 || exit 1
