#!/bin/bash
# Round-5: MoE locations with a pool workspace: MoE tests, the candidate test, MoE bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 700 $T tests/test_moe_gpu.py tests/test_models_gpu.py -k "moe or locations or gate" tests/test_autotune_candidates_gpu.py > gpurun_out/r5x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --model moe --steps 20 --warmup 5 > gpurun_out/r5x_moe.json 2> gpurun_out/r5x_moe.err
rc=$?; tail -1 gpurun_out/r5x_moe.json | cut -c1-160; exit $rc
