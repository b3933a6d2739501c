#!/bin/bash
# BERT-base attention backward form A/B (split vs w8, interleaved), then the step-delimited
# steady-state PMC passes of BERT and ResNet-50
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for m in split w8; do
    HETU_ATTN_BWD=$m timeout -k 10 300 python -u bench.py --model bert --steps 30 --warmup 5 > $O/r6h_bert_$m$i.json 2> $O/r6h_bert_$m$i.err || exit $?
    echo "$m $i $(python3 -c "import json;d=json.loads(open('$O/r6h_bert_$m$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config'].get('aten_kernels_per_step'))")"
  done
done
PMC_MODEL=bert bash scripts/gpu_pmc_steady.sh && PMC_MODEL=resnet50 bash scripts/gpu_pmc_steady.sh
