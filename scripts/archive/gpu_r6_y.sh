#!/bin/bash
# masked-position MLM head: tests, BERT A/B (HETU_BERT_MAX_PRED=0 scores every position)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlm_gather_gpu.py \
  tests/test_native_dispatch_gpu.py tests/test_torch_free_launch_gpu.py > $O/r6y_tests.txt 2>&1
rc=$?; tail -3 $O/r6y_tests.txt; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for m in 0 20; do
    HETU_BERT_MAX_PRED=$m timeout -k 10 300 python -u bench.py --model bert --steps 30 --warmup 5 > $O/r6y_bert_$m$i.json 2> $O/r6y_bert_$m$i.err || { tail -8 $O/r6y_bert_$m$i.err; exit 1; }
    echo "maxpred=$m $i $(python3 -c "import json;d=json.loads(open('$O/r6y_bert_$m$i.json').read().strip().splitlines()[-1]);c=d['config'];print(d['value'], d['ms_per_step'], c.get('aten_kernels_per_step'), c.get('vendor_kernels_per_step'), c.get('mlm_head'))")"
  done
done
