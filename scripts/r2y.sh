export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S bench_bn 300 python -u scripts/bench_bn.py gpurun_out/bench_bn_r2y.txt &&
$S test_conv 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k conv &&
$S bench_rn 300 python bench.py --steps 30 --warmup 5
