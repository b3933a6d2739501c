#!/bin/bash
# Round-5: attention (fused + flash) tests and timing after the softmax rework, the fp32
# model tests, the hipGraph BN test; then the BERT bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 900 --timeout-method thread"
echo "== tests"
timeout -k 10 900 $T --maxfail=5 tests/test_fused_gpu.py tests/test_flash_attn_gpu.py tests/test_ring_attention_gpu.py \
    tests/test_models_gpu.py tests/test_bn_fusion_gpu.py::test_hipgraph_replays_fused_bn_backward_like_eager \
    tests/test_native_dispatch_gpu.py::test_bert_base_bench_step_launches_no_torch_kernels tests/test_ps_dense_overlap_gpu.py tests/test_ipc_allreduce_gpu.py tests/test_gemm_gpu.py::test_matmul_pre_stores_activation_and_pre_activation \
    > gpurun_out/r5g_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r5g_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
echo "== attention timing"
ALT_FLASH_LIB=csrc/build/libfa_old.so timeout -k 10 300 python3 scripts/bench_attn.py > gpurun_out/r5g_attn.txt 2>&1
rc=$?; tail -24 gpurun_out/r5g_attn.txt; [ $rc -eq 0 ] || exit $rc
echo "== bert"
timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5g_bert.json 2> gpurun_out/r5g_bert.err
rc=$?; tail -1 gpurun_out/r5g_bert.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== wdl"
HETU_BENCH_PYPROF=gpurun_out/r5g_wdl_pyprof.txt timeout -k 10 400 python3 bench.py --model wdl --steps 60 --warmup 10 > gpurun_out/r5g_wdl.json 2> gpurun_out/r5g_wdl.err
rc=$?; tail -1 gpurun_out/r5g_wdl.json | cut -c1-1200; exit $rc
