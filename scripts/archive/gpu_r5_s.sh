#!/bin/bash
# Round-5: gmask model test (seeded builds); DTS gate over 20 + 5 steps with the segmented
# locations scan on / off (sparsification point), MoE top-k bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_models_gpu.py -k "moe" > gpurun_out/r5s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5s_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for env in "HETU_MOE_LOC_SEGMENTED=1" "HETU_MOE_LOC_SEGMENTED=0"; do
  tag=$(echo $env | tr '=' '_')
  env $env timeout -k 10 400 python3 bench.py --model moe --moe-gate dts --steps 20 --warmup 5 > gpurun_out/r5s_dts_$tag.json 2> gpurun_out/r5s_dts.err
  rc=$?; echo "$env $(tail -1 gpurun_out/r5s_dts_$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["dts"])')"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5s_dts.err; exit $rc; }
done
