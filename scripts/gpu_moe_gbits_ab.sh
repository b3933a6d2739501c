#!/bin/bash
# MoE: keep-bit gradient mask (HETU_GMASK_BITS) -- tests, then bench A/B interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py \
  tests/test_gemm_gpu.py -k "keep_bits or relu_mask or act_dropout or moe" > $O/gb_tests.txt 2>&1
rc=$?; tail -3 $O/gb_tests.txt; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for b in 0 1; do
    HETU_GMASK_BITS=$b timeout -k 10 300 python -u bench.py --model moe --steps 20 --warmup 5 > $O/gb_moe_$b$i.json 2> $O/gb_moe_$b$i.err || exit $?
    echo "gbits=$b $i $(python3 -c "import json;d=json.loads(open('$O/gb_moe_$b$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config'].get('aten_kernels_per_step'), d['config'].get('kernels_per_step'))")"
  done
done
