export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_gemm 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread &&
$S conv_shapes 400 python -u scripts/bench_conv_resnet.py 256 gpurun_out/conv_shapes_r2h.txt
