#!/bin/bash
# Round-5 GPU check: new tests first (hipGraph + fused BN, kernel census at bench
# shapes), then the MoE top-2 / DTS benches, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q -p no:cacheprovider --timeout 900 --timeout-method thread"
echo "== new tests"
timeout -k 10 900 $T tests/test_flash_attn_gpu.py tests/test_bn_fusion_gpu.py::test_hipgraph_replays_fused_bn_backward_like_eager \
    tests/test_native_dispatch_gpu.py > gpurun_out/r5a_new.log 2>&1
rc=$?; tail -15 gpurun_out/r5a_new.log; [ $rc -eq 0 ] || exit $rc
echo "== moe benches"
timeout -k 10 300 python3 bench.py --model moe --steps 10 --warmup 3 > gpurun_out/r5a_moe_topk.json 2> gpurun_out/r5a_moe_topk.err
rc=$?; tail -2 gpurun_out/r5a_moe_topk.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5a_moe_topk.err; exit $rc; }
timeout -k 10 300 python3 bench.py --model moe --moe-gate dts --steps 10 --warmup 3 > gpurun_out/r5a_moe_dts.json 2> gpurun_out/r5a_moe_dts.err
rc=$?; tail -2 gpurun_out/r5a_moe_dts.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5a_moe_dts.err; exit $rc; }
echo "== gpu suite"
timeout -k 10 1000 $T tests/ -m gpu > gpurun_out/r5a_suite.log 2>&1
rc=$?; tail -25 gpurun_out/r5a_suite.log; exit $rc
