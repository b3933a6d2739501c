#!/bin/bash
# GEMM/conv kernel validation + microbench on one GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
df -h /dev/shm; free -g | head -2
echo "== build"; make -C csrc -j16 > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== gemm tests"
  timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_tests.log 2>&1
  rc=$?; tail -30 gpurun_out/gemm_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
echo "== gemm bench"
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1
rc=$?; tail -40 gpurun_out/bench_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== diag conv"
timeout -k 10 200 python scripts/diag_conv.py > gpurun_out/diag_conv.log 2>&1
rc=$?; tail -5 gpurun_out/diag_conv.log; exit $rc
