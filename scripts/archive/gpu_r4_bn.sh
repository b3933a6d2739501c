#!/bin/bash
# Round-4: kernel tests (incl. the BN-reduction epilogues), then ResNet-50 A/B of the
# BatchNorm fusions (backward reduction in the dgrad epilogue; forward statistics in the
# conv epilogue), BERT bench, steady-state ResNet-50 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S tests ${TESTS_TIMEOUT:-500} python -u -m pytest -x -q --timeout ${PYTEST_TIMEOUT:-120} --timeout-method thread -m gpu \
  ${TESTS:-tests/test_bn_fusion_gpu.py tests/test_runtime_gpu.py tests/test_gemm_gpu.py tests/test_stem_gpu.py tests/test_native_dispatch_gpu.py tests/test_rccl_gpu.py} || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed|[0-9]+ error" gpurun_out/tests.log || { echo "TESTS FAILED"; exit 1; }
for v in ${VARIANTS:-1_1 1_0 0_0}; do   # <bwd fusion>_<fwd stats fusion>
  a=${v%_*}; b=${v#*_}
  HETU_FUSE_BN_BWD=$a HETU_FUSE_BN_STATS=$b HETU_AUTOTUNE_DUMP=gpurun_out/at_resnet50_bn$a$b.txt \
    bash $S b_resnet50_bn$a$b 300 python bench.py --model resnet50 --steps 20 --warmup 5 || exit $?
done
if [ -n "${BERT:-1}" ]; then
  HETU_AUTOTUNE_DUMP=gpurun_out/at_bert_r4.txt bash $S b_bert 300 python bench.py --model bert --steps 20 --warmup 5 || exit $?
fi
if [ -n "${PROF:-resnet50}" ]; then
  cd /tmp && HETU_FUSE_BN_STATS=${PROF_STATS:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run --output-format csv \
    -- python3 $R/bench.py --model ${PROF:-resnet50} --steps 5 --warmup 3 > $R/gpurun_out/prof_r4.log 2>&1
  rc=$?; cd $R; tail -2 gpurun_out/prof_r4.log
  [ $rc -eq 0 ] || exit $rc
  f=$(ls gpurun_out/prof_r4/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find gpurun_out/prof_r4 -name "*kernel_trace.csv" | head -1)
  python scripts/prof_steps.py "$f" --last 3 > gpurun_out/prof_r4_steady.txt 2>&1; head -45 gpurun_out/prof_r4_steady.txt
fi
