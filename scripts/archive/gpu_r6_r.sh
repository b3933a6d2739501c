#!/bin/bash
# piecewise hipGraph replay of the PS step: tests, then WDL 1 worker eager vs piecewise
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_piecewise_graph_gpu.py \
  tests/test_ps_dense_overlap_gpu.py > $O/r6r_tests.txt 2>&1
rc=$?; grep -v "^\[test-start\]" $O/r6r_tests.txt | grep -E "passed|failed|Error|error|piecewise|Traceback|File " | tail -30; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for pw in 0 1; do
    HETU_PIECEWISE_GRAPH=$pw timeout -k 10 300 python -u bench.py --model wdl --steps 200 --warmup 20 > $O/r6r_wdl_$pw$i.json 2> $O/r6r_wdl_$pw$i.err || { tail -20 $O/r6r_wdl_$pw$i.err; exit 1; }
    echo "piecewise=$pw $i $(python3 -c "import json;d=json.loads(open('$O/r6r_wdl_$pw$i.json').read().strip().splitlines()[-1]);c=d['config'];print(d['value'], d['ms_per_step'], c.get('step_breakdown_ms'), c.get('aten_kernels_per_step'), c.get('cache_hit_rate'))")"
  done
done
grep -h "piecewise" $O/r6r_wdl_*.err | head -5
