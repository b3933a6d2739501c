#!/bin/bash
# (1) WDL: 1 PS server + 8 workers on the one GPU (JSON now reports n_gpus = devices, workers = 8)
# (2) DTS gate, 16 local experts, slower temperature decay (intermediate budgets)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
STEPS=100 WARMUP=20 bash scripts/gpu_wdl8_one_gpu.sh || exit $?
timeout -k 10 600 python3 bench.py --model moe --moe-gate dts --moe-local-experts 16 --dts-schedule 2.0,0.985,0.05 \
  --steps 260 --warmup 2 > $O/dts16_slow.json 2> $O/dts16_slow.err || { tail -5 $O/dts16_slow.err; exit 1; }
tail -1 $O/dts16_slow.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['dts'])"
