export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S diag_bs2_bf16 180 python -u scripts/diag_smoke.py 2 bf16 &&
$S layers_fused 240 python -u scripts/diag_layers.py 2 fused &&
$S layers_unfused 240 env HETU_FUSE=0 python -u scripts/diag_layers.py 2 &&
$S test_bn_models 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread &&
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5
