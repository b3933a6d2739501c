#!/bin/bash
# ResNet-50: BN partial-statistics block target A/B (HETU_BN_TUNE), interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 0 1024 2048; do
    if [ $v = 0 ]; then unset HETU_BN_TUNE; else export HETU_BN_TUNE=$v,0,0; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r6z_$v$i.json 2> $O/r6z_$v$i.err || { tail -5 $O/r6z_$v$i.err; exit 1; }
    echo "bn_chunks=$v $i $(python3 -c "import json;d=json.loads(open('$O/r6z_$v$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
