#!/bin/bash
# deferred embedding-gradient push (ps/table.py): PS tests, then WDL 1 worker A/B interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_piecewise_graph_gpu.py \
  tests/test_ps_dense_overlap_gpu.py > $O/r6u_tests.txt 2>&1
rc=$?; grep -v "^\[test-start\]" $O/r6u_tests.txt | grep -E "passed|failed|Error|error|Traceback|File " | tail -20; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for d in 0 1; do
    HETU_PS_DEFER_PUSH=$d timeout -k 10 300 python -u bench.py --model wdl --steps 200 --warmup 20 > $O/r6u_wdl_$d$i.json 2> $O/r6u_wdl_$d$i.err || { tail -20 $O/r6u_wdl_$d$i.err; exit 1; }
    echo "defer=$d $i $(python3 -c "import json;d=json.loads(open('$O/r6u_wdl_$d$i.json').read().strip().splitlines()[-1]);c=d['config'];print(d['value'], d['ms_per_step'], c.get('step_breakdown_ms'), c.get('cache_hit_rate'), c.get('prefetch_hits'))")"
  done
done
STEPS=100 WARMUP=20 bash scripts/gpu_wdl8_one_gpu.sh > /dev/null 2>&1; tail -1 $O/wdl8.json | cut -c1-240
