#!/bin/bash
# What the vendor libraries still buy: ResNet-50 and BERT bench lines with the default
# per-shape choice (hand-written vs vendor) and with HETU_GEMM=hip HETU_CONV=hip
# (hand-written only wherever a kernel exists).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$R
for m in resnet50 bert; do
  for mode in auto hip; do
    HETU_GEMM=$mode HETU_CONV=$mode timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 \
      > gpurun_out/cost_${m}_$mode.json 2> gpurun_out/cost_${m}_$mode.err
    rc=$?; echo "$m $mode rc=$rc $(cat gpurun_out/cost_${m}_$mode.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
