#!/bin/bash
# GEMM kernel check + microbench on one GPU box (libraries built in-tree beforehand):
# correctness tests of the MFMA GEMM / conv kernels, then scripts/bench_tiles.py
# (hand-written tiles vs hipBLASLt / MIOpen on the BERT and ResNet-50 shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
echo "== gemm/conv tests"
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py ${EXTRA_TESTS:-} -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gemm_tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
echo "== bench_tiles"
timeout -k 10 400 python -u scripts/bench_tiles.py gpurun_out/bench_tiles.txt > gpurun_out/bench_tiles.log 2>&1
rc=$?; tail -30 gpurun_out/bench_tiles.log
exit $rc
