#!/bin/bash
# New conv kernels: numerics tests, then the per-shape sweep of the shapes they target.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_stem_gpu.py tests/test_gemm_gpu.py} > gpurun_out/conv_tests.txt 2>&1 \
  || { tail -40 gpurun_out/conv_tests.txt; exit 1; }
tail -2 gpurun_out/conv_tests.txt
CONV_ONLY=${CONV_ONLY:-"3,224,64,7,2;64,56,64,1,1;64,56,64,3,1"} timeout -k 10 300 python scripts/bench_conv_resnet.py 256 gpurun_out/conv_sweep.txt > gpurun_out/conv_sweep.log 2>&1 || { tail -30 gpurun_out/conv_sweep.log; exit 1; }
cat gpurun_out/conv_sweep.txt
