#!/bin/bash
# MoE: fused combine backward (HETU_MOE_FUSED_COMBINE_BWD) -- tests, kernel traces, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py tests/test_misc_ops_gpu.py tests/test_models_gpu.py \
  tests/test_autotune_candidates_gpu.py tests/test_native_dispatch_gpu.py > $O/cb_tests.txt 2>&1
rc=$?; tail -3 $O/cb_tests.txt; [ $rc = 0 ] || exit $rc
for f in 0 1; do
  HETU_MOE_FUSED_COMBINE_BWD=$f MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null || exit $?
  mv $O/prof_moe_shapes.txt $O/cb${f}_shapes.txt && mv $O/prof_moe_steady.txt $O/cb${f}_steady.txt && rm -rf $O/prof_moe
  head -1 $O/cb${f}_shapes.txt
done
for i in 1 2; do
  for f in 0 1; do
    HETU_MOE_FUSED_COMBINE_BWD=$f timeout -k 10 300 python -u bench.py --model moe --steps 20 --warmup 5 > $O/cb_moe_$f$i.json 2> $O/cb_moe_$f$i.err || exit $?
    echo "fused=$f $i $(python3 -c "import json;d=json.loads(open('$O/cb_moe_$f$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config'].get('aten_kernels_per_step'), d['config'].get('kernels_per_step'))")"
  done
done
