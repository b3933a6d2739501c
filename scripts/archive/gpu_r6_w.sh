#!/bin/bash
# replica-row LayerNorm backward: tests, memops sweep, kernel trace A/B, BERT A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py > $O/r6w_tests.txt 2>&1
rc=$?; tail -2 $O/r6w_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u scripts/bench_memops.py --ln-blocks 512 > $O/r6w_memops.txt 2>&1 || exit $?
grep ln_bwd $O/r6w_memops.txt
for i in 1 2; do
  for r in 0 32; do
    HETU_LN_BWD_REP=$r timeout -k 10 300 python -u bench.py --model bert --steps 30 --warmup 5 > $O/r6w_bert_$r$i.json 2> $O/r6w_bert_$r$i.err || exit $?
    echo "rep=$r $i $(python3 -c "import json;d=json.loads(open('$O/r6w_bert_$r$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
