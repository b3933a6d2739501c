#!/bin/bash
# MoE bench A/B of the default kernel library against an alternate build (ALT_LIB=path),
# interleaved on one box
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
ALT=${ALT_LIB:?ALT_LIB=path of the alternate libhetu_kernels.so}
TAG=${TAG:-alt}
for i in 1 2; do
  for v in def $TAG; do
    if [ $v = def ]; then L=; else L=$ALT; fi
    HETU_KERNELS_LIB=$L timeout -k 10 300 python -u bench.py --model ${MODEL:-moe} --steps 20 --warmup 5 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || exit $?
    echo "$v $i $(python3 -c "import json;d=json.loads(open('$O/ab_${v}_$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
