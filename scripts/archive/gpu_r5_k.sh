#!/bin/bash
# Round-5: memory-bound BERT kernels (LN fwd/bwd, GELU-grad colsum, flat Adam) bandwidth,
# LN-backward block sweep, and the hipGraph dropout-guard test.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_models_gpu.py -k hipgraph > gpurun_out/r5k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/bench_memops.py --out gpurun_out/r5k_memops.jsonl > gpurun_out/r5k_memops.log 2>&1
rc=$?; cat gpurun_out/r5k_memops.log | tail -12; [ $rc -eq 0 ] || exit $rc
