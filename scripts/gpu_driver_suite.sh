#!/bin/bash
# Reproduce the driver's round-end GPU tier exactly: smoke(), then
# `pytest tests/ -x -q -m gpu` without a PYTHONPATH, without a rebuild.
# Usage (from the container): gpurun --timeout 1100 -- bash scripts/gpu_driver_suite.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
echo "== pytest -m gpu (driver form)"
timeout -k 10 ${TEST_TIMEOUT:-900} python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_driver.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_driver.log
echo "pytest rc=$rc"
exit $rc
