#!/bin/bash
# Round-5 GPU check: new tests first (hipGraph + fused BN, kernel census at bench
# shapes), then the MoE top-2 / DTS benches, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q -p no:cacheprovider --timeout 900 --timeout-method thread"
echo "== transformer kernel census"
timeout -k 10 200 python3 scripts/diag_torch_kernels_transformer.py > gpurun_out/r5a_diag_tr.txt 2>&1
tail -12 gpurun_out/r5a_diag_tr.txt
echo "== new tests"
timeout -k 10 900 $T --deselect tests/test_flash_attn_gpu.py::test_transformer_step_launches_no_torch_kernels tests/test_flash_attn_gpu.py tests/test_bn_fusion_gpu.py::test_hipgraph_replays_fused_bn_backward_like_eager \
    tests/test_native_dispatch_gpu.py > gpurun_out/r5a_new.log 2>&1
rc=$?; tail -15 gpurun_out/r5a_new.log
echo "== gpu suite"
timeout -k 10 1000 $T tests/ -m gpu > gpurun_out/r5a_suite.log 2>&1
rc=$?; tail -25 gpurun_out/r5a_suite.log; exit $rc
