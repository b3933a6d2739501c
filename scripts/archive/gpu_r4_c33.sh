#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py -k "conv3x3 or conv_passes" > gpurun_out/c33_tests.txt 2>&1 \
  || { tail -40 gpurun_out/c33_tests.txt; exit 1; }
tail -2 gpurun_out/c33_tests.txt
CONV_ONLY="64,56,64,3,1;128,28,128,3,1;256,14,256,3,1;512,7,512,3,1" timeout -k 10 300 python scripts/bench_conv_resnet.py 256 gpurun_out/c33_sweep.txt > gpurun_out/c33_sweep.log 2>&1 || { tail -30 gpurun_out/c33_sweep.log; exit 1; }
cat gpurun_out/c33_sweep.txt
