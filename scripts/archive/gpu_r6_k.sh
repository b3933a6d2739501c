#!/bin/bash
# current numbers for every bench config at HEAD (1 GPU): ResNet-50 (driver default), MoE
# top-2 and DTS at the reference batch, WDL 1 worker, logreg on the CPU
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {   # name, args...
  n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/r6k_$n.json 2> $O/r6k_$n.err || { echo "$n failed"; tail -5 $O/r6k_$n.err; return 1; }
  echo "$n $(tail -1 $O/r6k_$n.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print(d['value'], d['unit'], d['ms_per_step'], 'aten', c.get('aten_kernels_per_step'), 'vendor', c.get('vendor_kernels_per_step'), 'graph', c.get('hipgraph'))")"
}
run resnet50_a --steps 20 --warmup 5 && run moe_top2 --model moe --steps 20 --warmup 5 \
  && run resnet50_b --steps 20 --warmup 5 && run moe_top2_b --model moe --steps 20 --warmup 5 \
  && run moe_dts --model moe --moe-gate dts --steps 20 --warmup 5 \
  && run wdl --model wdl --steps 200 --warmup 20 && run logreg --model logreg --steps 200 --warmup 20
