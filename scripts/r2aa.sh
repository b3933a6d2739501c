export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_k 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread &&
$S bench_rn 300 python bench.py --steps 30 --warmup 5 &&
$S bench_rn2 300 python bench.py --steps 30 --warmup 5
