#!/bin/bash
# MoE: row-block expert outputs (no concatenation copy) -- tests, then bench A/B interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py \
  tests/test_autotune_candidates_gpu.py > $O/r6m_tests.txt 2>&1
rc=$?; tail -3 $O/r6m_tests.txt; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for rc in 0 1; do
    HETU_MOE_ROW_CONCAT=$rc timeout -k 10 300 python -u bench.py --model moe --steps 20 --warmup 5 > $O/r6m_moe_$rc$i.json 2> $O/r6m_moe_$rc$i.err || exit $?
    echo "rowconcat=$rc $i $(python3 -c "import json;d=json.loads(open('$O/r6m_moe_$rc$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config'].get('aten_kernels_per_step'), d['config'].get('kernels_per_step'))")"
  done
done
HETU_MOE_ROW_CONCAT=1 timeout -k 10 300 python -u bench.py --model moe --moe-gate dts --steps 20 --warmup 5 > $O/r6m_dts.json 2> $O/r6m_dts.err || exit $?
tail -1 $O/r6m_dts.json | cut -c1-300
