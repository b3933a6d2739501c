#!/bin/bash
# Round 6: watchdog / IPC / RNG / graph-replay tests, smoke, then the driver bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6b_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r6b_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_rng_gpu.py tests/test_rccl_gpu.py tests/test_ipc_allreduce_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py \
  > gpurun_out/r6b_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r6b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err
rc=$?; tail -2 gpurun_out/r6b_bench.json; exit $rc
