#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py tests/test_ps_dense_overlap_gpu.py tests/test_models_gpu.py \
  > gpurun_out/r6f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --model wdl --steps 200 --warmup 20 > gpurun_out/r6f_wdl.json 2> gpurun_out/r6f_wdl.err
rc=$?; tail -c 500 gpurun_out/r6f_wdl.json; [ $rc -eq 0 ] || exit $rc
