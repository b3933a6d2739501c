export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5 &&
$S test_conv 300 python -u -m pytest tests/test_ops_differential_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or resnet"
