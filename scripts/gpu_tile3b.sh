#!/bin/bash
# tile-3 rolling-prefetch rerun + loss-label / matmul-cast census check for MoE
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_tile3.sh || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_tensor_ops_gpu.py tests/test_moe_gpu.py tests/test_native_dispatch_gpu.py > gpurun_out/t3b_tests.txt 2>&1 \
  || { tail -30 gpurun_out/t3b_tests.txt; exit 1; }
tail -1 gpurun_out/t3b_tests.txt
timeout -k 10 240 python scripts/find_torch_kernels.py --model moe > gpurun_out/census_moe.txt 2>&1 || exit $?
grep -A12 "kernel classes" gpurun_out/census_moe.txt
