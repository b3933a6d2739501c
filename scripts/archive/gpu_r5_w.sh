#!/bin/bash
# Round-5 closing benches: every bench.py model once at its defaults (plus the DTS gate),
# for the record in profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in "resnet50" "bert" "moe" "moe --moe-gate dts" "wdl" "logreg"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 500 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5w_$tag.json 2> gpurun_out/r5w_$tag.err
  rc=$?; echo "$tag $(tail -1 gpurun_out/r5w_$tag.json | cut -c1-150)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5w_$tag.err; exit $rc; }
done
