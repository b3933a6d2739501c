#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_k.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/pytest_gpu_k.log; tail -2 gpurun_out/pytest_gpu_k.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model moe --moe-gate dts --steps 20 --warmup 5 > gpurun_out/bench_moe_dts_k.json 2> gpurun_out/bench_moe_dts_k.err || exit $?
cat gpurun_out/bench_moe_dts_k.json
timeout -k 10 300 python bench.py --model moe --steps 20 --warmup 5 > gpurun_out/bench_moe_k.json 2> gpurun_out/bench_moe_k.err || exit $?
cat gpurun_out/bench_moe_k.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_moe_dts_k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model moe --moe-gate dts --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_moe_dts_k.log 2>&1
echo prof rc=$?
