#!/bin/bash
# LayerNorm-backward forms: tests, the memops sweep, BERT-base A/B (row vs half) interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py > $O/r6j_tests.txt 2>&1
rc=$?; tail -3 $O/r6j_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u scripts/bench_memops.py --ln-blocks 256,512,1024,2048 > $O/r6j_memops.txt 2>&1 || exit $?
cat $O/r6j_memops.txt
for i in 1 2; do
  for f in row half; do
    HETU_LN_BWD_FORM=$f timeout -k 10 300 python -u bench.py --model bert --steps 30 --warmup 5 > $O/r6j_bert_$f$i.json 2> $O/r6j_bert_$f$i.err || exit $?
    echo "$f $i $(python3 -c "import json;d=json.loads(open('$O/r6j_bert_$f$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
