export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_gemm 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread &&
$S bench_tiles 400 python -u scripts/bench_tiles.py gpurun_out/bench_tiles_r2i.txt
