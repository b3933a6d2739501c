#!/bin/bash
# Single-stage 128x128 tile (tile 3, 4 blocks per CU): GEMM/conv numerics, then the
# ResNet-50 / BERT bench lines with the per-shape autotune decisions.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_ops_differential_gpu.py > gpurun_out/t3_tests.txt 2>&1 \
  || { tail -30 gpurun_out/t3_tests.txt; exit 1; }
tail -2 gpurun_out/t3_tests.txt
for m in resnet50 bert; do
  HETU_AUTOTUNE_DUMP=gpurun_out/at3_${m}.txt timeout -k 10 240 \
    python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/t3_${m}.json 2>/dev/null || exit $?
  echo "$m $(sed 's/.*"value": \([0-9.]*\).*/\1/' gpurun_out/t3_${m}.json) hand=$(grep -c -- '-> hip' gpurun_out/at3_${m}.txt) lo=$(grep -c -- '-> hip_lo' gpurun_out/at3_${m}.txt) lib=$(grep -vc -- '-> hip' gpurun_out/at3_${m}.txt)"
done
