#!/bin/bash
# Round-5: allocator A/B on ResNet-50 (BFC pool default vs torch's caching allocator hook),
# interleaved runs.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in bfc torch bfc torch; do
  HETU_ALLOCATOR=$a timeout -k 10 400 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5ac_$a.json 2> gpurun_out/r5ac.err
  rc=$?; echo "$a $(tail -1 gpurun_out/r5ac_$a.json | cut -c1-120)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5ac.err; exit $rc; }
done
