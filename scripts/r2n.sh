export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_gemm 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread &&
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5 &&
$S bench_resnet50b 300 python bench.py --steps 20 --warmup 5
