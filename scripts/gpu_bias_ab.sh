#!/bin/bash
# A/B of the autotune tie-break toward hand-written kernels (HETU_AUTOTUNE_NATIVE_BIAS):
# ResNet-50 and BERT bench lines plus the per-shape decisions (hand-written vs library).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in resnet50 bert; do
  for b in 0 0.03; do
    HETU_AUTOTUNE_NATIVE_BIAS=$b HETU_AUTOTUNE_DUMP=gpurun_out/at_${m}_$b.txt timeout -k 10 240 \
      python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/ab_${m}_$b.json 2>/dev/null || exit $?
    echo "$m bias=$b $(cut -c1-120 gpurun_out/ab_${m}_$b.json | sed 's/.*"value": \([0-9.]*\).*/\1/') hand=$(grep -c -- '-> hip' gpurun_out/at_${m}_$b.txt) lib=$(grep -vc -- '-> hip' gpurun_out/at_${m}_$b.txt)"
  done
done
