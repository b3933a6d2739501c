#!/bin/bash
# A/B of BN statistics fused into the conv epilogue (HETU_FUSE_BN_STATS), ResNet-50, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for f in 0 1; do
    HETU_FUSE_BN_STATS=$f timeout -k 10 240 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bns_$f.json 2>/dev/null || exit $?
    echo "rep=$rep fuse=$f $(sed 's/.*"value": \([0-9.]*\).*/\1/' gpurun_out/bns_$f.json)"
  done
done
