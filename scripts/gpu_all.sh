#!/bin/bash
# One GPU-box session: build, GPU tests, then every bench config (one JSON each).
# Stops at the first crash / timeout.  BENCHES="resnet50 bert moe wdl" selects configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
echo "== build"; make -C csrc -j16 > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-480} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -60; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
fi
for m in ${BENCHES-resnet50 bert moe wdl}; do
  echo "== bench $m"
  extra=""
  [ "$m" = "wdl" ] && extra="${WDL_ARGS:-}"
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --model $m --steps ${STEPS:-20} --warmup 5 $extra > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err
  rc=$?
  cat gpurun_out/bench_$m.json; tail -3 gpurun_out/bench_$m.err
  if [ $rc -ne 0 ]; then echo "bench $m rc=$rc"; [ $rc -ge 124 ] && exit $rc; fi
done
if [ -n "${PROFILE_MODEL:-}" ]; then
  echo "== rocprofv3 $PROFILE_MODEL"
  cd /tmp && timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$PROFILE_MODEL -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model $PROFILE_MODEL --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$PROFILE_MODEL.log 2>&1
  rc=$?
  cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/prof_$PROFILE_MODEL.log
  exit $rc
fi
