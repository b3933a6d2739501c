#!/bin/bash
# Diagnostic bench: autotune decisions (hip vs vendor per conv shape), per-op-type
# GPU times and channels-last layout misses.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
make -C csrc -j16 > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
HETU_AUTOTUNE_DUMP=gpurun_out/autotune.txt HETU_CHECK_LAYOUT=1 timeout -k 10 ${BENCH_TIMEOUT:-300} \
  python bench.py --steps ${STEPS:-10} --warmup 3 --op-profile gpurun_out/ops.txt ${BENCH_ARGS:-} > gpurun_out/diag.json 2> gpurun_out/diag.err
rc=$?
cat gpurun_out/diag.json; tail -8 gpurun_out/diag.err
exit $rc
