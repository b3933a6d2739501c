#!/bin/bash
# Whole GPU test suite as the driver runs it (pytest -m gpu), without -x so every failure is
# listed, each test under a thread timeout; then smoke() and a 1-GPU default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-full}
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc2=$?; tail -3 gpurun_out/${TAG}_smoke.log; [ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc3=$?; tail -1 gpurun_out/${TAG}_bench.json | cut -c1-200; [ $rc3 -eq 0 ] || exit $rc3
exit $rc
