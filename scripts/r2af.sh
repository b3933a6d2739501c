export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_ln 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_deterministic_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread &&
$S bench_bert 300 python bench.py --model bert --steps 30 --warmup 5 &&
$S bench_bert2 300 python bench.py --model bert --steps 30 --warmup 5
