#!/bin/bash
# ResNet-50 knob A/B, interleaved: default / every eligible BN-backward fusion / more autotune reps
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in base bnall tune; do
    case $v in base) E="";; bnall) E="HETU_FUSE_BN_BWD=all";; tune) E="HETU_AUTOTUNE_REPS=10 HETU_AUTOTUNE_ROUNDS=5";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r6x_$v$i.json 2> $O/r6x_$v$i.err || { tail -5 $O/r6x_$v$i.err; exit 1; }
    echo "$v $i $(python3 -c "import json;d=json.loads(open('$O/r6x_$v$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
