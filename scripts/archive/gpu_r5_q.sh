#!/bin/bash
# Round-5: segmented MoE locations scan; LN backward back to one row per iteration with the
# wider column reduce: MoE / LN tests, MoE top-k + DTS and BERT benches, MoE profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_moe_gpu.py tests/test_fused_gpu.py tests/test_native_dispatch_gpu.py > gpurun_out/r5q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5q_tests.log; [ $rc -eq 0 ] || exit $rc
for m in "moe --moe-gate topk" "moe --moe-gate dts" "bert"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5q_$tag.json 2> gpurun_out/r5q_$tag.err
  rc=$?; tail -1 gpurun_out/r5q_$tag.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5q_$tag.err; exit $rc; }
done
MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -16 gpurun_out/prof_moe_steady.txt
