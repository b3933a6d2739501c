#!/bin/bash
# Round-5: LayerNorm backward two rows per iteration + wider column-reduce grid: LN tests,
# memops kernel times (rocprofv3 csv), BERT bench, MoE profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_fused_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py > gpurun_out/r5p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5p_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_memops_p -o memops -- python3 $R/scripts/bench_memops.py --ln-blocks 256,512,1024 > $R/gpurun_out/r5p_memops.log 2>&1
rc=$?; cd $R; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5p_bert$i.json 2> gpurun_out/r5p_bert.err
  rc=$?; tail -1 gpurun_out/r5p_bert$i.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5p_bert.err; exit $rc; }
done
MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -24 gpurun_out/prof_moe_steady.txt
