#!/bin/bash
# Round-4 baseline: ResNet-50 and BERT with the per-shape autotune (auto) and with the
# hand-written kernels only (hip), autotune decisions dumped for each.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODELS:-resnet50 bert}; do
  for mode in ${MODES:-auto hip}; do
    HETU_GEMM=$mode HETU_CONV=$mode HETU_AUTOTUNE_DUMP=gpurun_out/at_${m}_${mode}.txt \
      timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/b_${m}_${mode}.json 2> gpurun_out/b_${m}_${mode}.err \
      || { tail -20 gpurun_out/b_${m}_${mode}.err; exit 1; }
    echo "$m $mode: $(cut -c1-160 gpurun_out/b_${m}_${mode}.json)"
  done
done
