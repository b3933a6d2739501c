#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_rng_gpu.py tests/test_rccl_gpu.py tests/test_ipc_allreduce_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py \
  tests/test_gemm_splitk_gpu.py tests/test_torch_free_launch_gpu.py > gpurun_out/r6b_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r6b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err
rc=$?; tail -2 gpurun_out/r6b_bench.json; exit $rc
