#!/bin/bash
# Round-5 GPU check (2): pipelined flash kernels (tests, then A/B timing against the
# previous revision's library), Transformer census, hipGraph BN update test, native
# dispatch censuses, then the whole GPU suite (up to 5 failures reported).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 900 --timeout-method thread"
echo "== flash tests"
timeout -k 10 600 $T --maxfail=3 tests/test_flash_attn_gpu.py tests/test_ring_attention_gpu.py > gpurun_out/r5c_flash.log 2>&1
rc=$?; tail -8 gpurun_out/r5c_flash.log
case $rc in 0|1) ;; *) exit $rc ;; esac
echo "== attention timing"
ALT_FLASH_LIB=csrc/build/libfa_old.so timeout -k 10 300 python3 scripts/bench_attn.py > gpurun_out/r5c_attn.txt 2>&1
rc=$?; cat gpurun_out/r5c_attn.txt | tail -24; [ $rc -eq 0 ] || exit $rc
echo "== new tests"
timeout -k 10 1000 $T --maxfail=3 tests/test_bn_fusion_gpu.py::test_hipgraph_replays_fused_bn_backward_like_eager \
    tests/test_native_dispatch_gpu.py > gpurun_out/r5c_new.log 2>&1
rc=$?; tail -15 gpurun_out/r5c_new.log
case $rc in 0|1) ;; *) exit $rc ;; esac
echo "== gpu suite"
timeout -k 10 1100 $T --maxfail=5 tests/ -m gpu > gpurun_out/r5c_suite.log 2>&1
rc=$?; tail -30 gpurun_out/r5c_suite.log; exit $rc
