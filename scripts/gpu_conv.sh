#!/bin/bash
# conv/GEMM numerics tests, then the diagnostic bench (autotune table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_diag.sh
