#!/bin/bash
# dedup_rows replica A/B: the new GPU test, then BERT kernel profiles old vs new.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest tests/test_gemm_splitk_gpu.py tests/test_gemm_gpu.py tests/test_models_gpu.py -x -q --capture=sys \
  --timeout 120 --timeout-method thread > gpurun_out/dedup_tests.log 2>&1 || { tail -30 gpurun_out/dedup_tests.log; exit 1; }
tail -2 gpurun_out/dedup_tests.log
bash scripts/r2_ln_prof.sh
