#!/bin/bash
# One GPU-box session: kernel/model tests, a bench run and a rocprofv3 kernel profile.
# Stops at the first crash / timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
df -h /dev/shm; free -g | head -2
export TMPDIR=/tmp
STEPS=${STEPS:-20}
echo "== build" ; make -C csrc -j16 > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
fi
echo "== bench"
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then echo "bench rc=$rc"; exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3"
  cd /tmp && timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  rc=$?
  cd $GRAFT_REPO_ROOT
  tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
  exit $rc
fi
