export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S test_g 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
$S bench_bert 300 python bench.py --model bert --steps 30 --warmup 5 &&
$S bench_rn 300 python bench.py --steps 30 --warmup 5 &&
$S diag_bert 300 python -u scripts/diag_torch_ops.py 0 bert
