#!/bin/bash
# Round-5: DTS bench with the smaller budgets pre-tuned in the first warmup step (x2).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 500 python3 bench.py --model moe --moe-gate dts --steps 20 --warmup 5 > gpurun_out/r5ab_dts$i.json 2> gpurun_out/r5ab_dts.err
  rc=$?; echo "$(tail -1 gpurun_out/r5ab_dts$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["dts"])')"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5ab_dts.err; exit $rc; }
done
