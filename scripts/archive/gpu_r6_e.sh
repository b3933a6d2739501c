#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py tests/test_ps_dense_overlap_gpu.py tests/test_models_gpu.py > gpurun_out/r6e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6e_tests.log; [ $rc -eq 0 ] || exit $rc
HETU_BENCH_PYPROF=gpurun_out/r6e_wdl_pyprof.txt timeout -k 10 200 python3 bench.py --model wdl --steps 200 --warmup 20 \
  > gpurun_out/r6e_wdl.json 2> gpurun_out/r6e_wdl.err
rc=$?; tail -c 700 gpurun_out/r6e_wdl.json; [ $rc -eq 0 ] || exit $rc
MODEL=resnet50 bash scripts/gpu_prof_model.sh || exit $?
MODEL=bert bash scripts/gpu_prof_model.sh || exit $?
