#!/bin/bash
# vector last-axis reduction: kernel tests, MoE top-2 bench (its loss reduces [65536, 2048])
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $O/r6n_tests.txt 2>&1
rc=$?; tail -3 $O/r6n_tests.txt; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model moe --steps 20 --warmup 5 > $O/r6n_moe$i.json 2> $O/r6n_moe$i.err || exit $?
  echo "moe $i $(python3 -c "import json;d=json.loads(open('$O/r6n_moe$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config'].get('aten_kernels_per_step'))")"
done
MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null 2>&1; head -14 $O/prof_moe_steady.txt
