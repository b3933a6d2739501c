#!/bin/bash
# Round-4: GEMM harness on the weight-gradient (TN) layouts, BN-fusion kernel tests with
# per-wave replicated statistics (HETU_CS_DIRECT=1), ResNet-50 A/B of that tail, and a
# steady-state ResNet-50 kernel trace at the defaults.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
if [ -n "${GEMM:-1}" ]; then
  TILES=013 bash $S gemm_tn 150 csrc/build/gemm_bench 4096 4096 4096 1 0  4096 4096 4096 0 0  4096 4096 4096 0 1 \
    4096 4096 4096 1 1  768 3072 8192 1 0  3072 3072 8192 1 0 || exit $?
fi
HETU_CS_DIRECT=1 bash $S tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_bn_fusion_gpu.py tests/test_gemm_gpu.py tests/test_stem_gpu.py || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed|[0-9]+ error" gpurun_out/tests.log || { echo "TESTS FAILED"; exit 1; }
for d in ${CSD:-1 0}; do
  HETU_CS_DIRECT=$d bash $S b_resnet50_csd$d 300 python bench.py --model resnet50 --steps 20 --warmup 5 || exit $?
done
if [ -n "${PROF:-1}" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run --output-format csv \
    -- python3 $R/bench.py --model resnet50 --steps 5 --warmup 3 > $R/gpurun_out/prof_r4.log 2>&1
  rc=$?; cd $R; tail -2 gpurun_out/prof_r4.log
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_r4 -name "*kernel_trace.csv" | head -1)
  python scripts/prof_steps.py "$f" --last 3 > gpurun_out/prof_r4_steady.txt 2>&1; head -30 gpurun_out/prof_r4_steady.txt
  python scripts/prof_shapes.py "$f" --top 80 > gpurun_out/prof_r4_shapes.txt 2>&1
fi
