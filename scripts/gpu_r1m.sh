#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn or batch" > gpurun_out/pytest_bn_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bn_m.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model wdl --steps 60 --warmup 10 > gpurun_out/bench_wdl_m.json 2> gpurun_out/bench_wdl_m.err || exit $?
cat gpurun_out/bench_wdl_m.json
timeout -k 10 300 python bench.py --model wdl --steps 60 --warmup 10 --no-prefetch > gpurun_out/bench_wdl_nopf_m.json 2> gpurun_out/bench_wdl_nopf_m.err || exit $?
cat gpurun_out/bench_wdl_nopf_m.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_rn_m.json 2> gpurun_out/bench_rn_m.err || exit $?
cat gpurun_out/bench_rn_m.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rn_m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn_m.log 2>&1
echo prof rc=$?
