#!/bin/bash
# Round-5 last check with non-temporal BN loads on by default: BN / kernel tests, smoke,
# default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_bn_fusion_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_native_dispatch_gpu.py > gpurun_out/r5ae_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5ae_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ae_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r5ae_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/r5ae_bench.json 2> gpurun_out/r5ae_bench.err
rc=$?; tail -1 gpurun_out/r5ae_bench.json | cut -c1-160; exit $rc
