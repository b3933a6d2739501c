#!/bin/bash
# Round-4 checkpoint: kernel tests + census, ResNet-50 / BERT benches with the default
# hand-written-only dispatch (autotune decisions dumped), and a steady-state
# rocprofv3 kernel trace of ResNet-50 summarised per step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_runtime_gpu.py tests/test_gemm_gpu.py tests/test_stem_gpu.py tests/test_native_dispatch_gpu.py tests/test_rccl_gpu.py} || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "failed|error" gpurun_out/tests.log || { echo "TESTS FAILED"; exit 1; }
CONV_ONLY="64,56,64,3,1;128,28,128,3,1;256,14,256,3,1;512,7,512,3,1" bash $S conv_sweep 300 \
  python scripts/bench_conv_resnet.py 256 gpurun_out/conv_sweep_r4.txt || exit $?
cat gpurun_out/conv_sweep_r4.txt
for m in ${MODELS:-resnet50 bert}; do
  HETU_AUTOTUNE_DUMP=gpurun_out/at_${m}_r4.txt bash $S b_$m 300 python bench.py --model $m --steps 20 --warmup 5 || exit $?
done
if [ -n "${PROF:-resnet50}" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run --output-format csv \
    -- python3 $R/bench.py --model ${PROF:-resnet50} --steps 5 --warmup 3 > $R/gpurun_out/prof_r4.log 2>&1
  rc=$?; cd $R; tail -2 gpurun_out/prof_r4.log
  [ $rc -eq 0 ] || exit $rc
  f=$(ls gpurun_out/prof_r4/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find gpurun_out/prof_r4 -name "*kernel_trace.csv" | head -1)
  python scripts/prof_steps.py "$f" --last 3 > gpurun_out/prof_r4_steady.txt 2>&1; head -45 gpurun_out/prof_r4_steady.txt
fi
