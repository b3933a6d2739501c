#!/bin/bash
# Round-5: fused expert GEMM (ReLU + dropout epilogue), locations scan, dropout kernel:
# tests, MoE copy attribution, MoE top-k / DTS benches and a MoE kernel profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 700 $T --maxfail=5 tests/test_moe_gpu.py tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py \
    tests/test_native_dispatch_gpu.py::test_moe_bench_step_launches_no_torch_kernels > gpurun_out/r5j_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r5j_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python3 scripts/diag_moe_copies.py > gpurun_out/r5j_moe_copies.txt 2>&1
rc=$?; cat gpurun_out/r5j_moe_copies.txt | tail -15; [ $rc -eq 0 ] || exit $rc
for g in topk dts; do
  timeout -k 10 300 python3 bench.py --model moe --moe-gate $g --steps 10 --warmup 3 > gpurun_out/r5j_moe_$g.json 2> gpurun_out/r5j_moe_$g.err
  rc=$?; tail -1 gpurun_out/r5j_moe_$g.json | cut -c1-220; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5j_moe_$g.err; exit $rc; }
done
MODEL=moe bash scripts/gpu_prof_model.sh
