#!/bin/bash
# Round-5: unrolled non-temporal flat optimizer: tests, memops kernel times with it on / off,
# BERT bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "optimizer" tests/test_deterministic_gpu.py > gpurun_out/r5v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5v_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  cd /tmp && HETU_OPT_V2=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_opt_v$v -o memops -- python3 $R/scripts/bench_memops.py --ln-blocks 512 > $R/gpurun_out/r5v_memops_v$v.log 2>&1
  rc=$?; cd $R; [ $rc -eq 0 ] || exit $rc
  grep -h "adam" gpurun_out/r5v_memops_v$v.log | tail -1
done
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5v_bert$i.json 2> gpurun_out/r5v_bert.err
  rc=$?; tail -1 gpurun_out/r5v_bert$i.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5v_bert.err; exit $rc; }
done
