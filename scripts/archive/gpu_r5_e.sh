#!/bin/bash
# Round-5: targeted re-check of the last failures, then the benches (gpu_r5_d.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 900 --timeout-method thread"
echo "== targeted tests"
timeout -k 10 900 $T --maxfail=5 tests/test_models_gpu.py tests/test_bn_fusion_gpu.py::test_hipgraph_replays_fused_bn_backward_like_eager \
    tests/test_deterministic_gpu.py tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py > gpurun_out/r5e_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r5e_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
bash scripts/gpu_r5_d.sh
