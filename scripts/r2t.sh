export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_det 300 python -u -m pytest tests/test_deterministic_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
