#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gemm_splitk_gpu.py tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_j.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/pytest_gpu_j.log; grep -E "FAILED|ERROR|Error" gpurun_out/pytest_gpu_j.log | head; tail -2 gpurun_out/pytest_gpu_j.log
[ $rc -ne 0 ] && exit $rc
HETU_AUTOTUNE_DUMP=gpurun_out/autotune_bert_j.txt timeout -k 10 300 python bench.py --model bert --steps 20 --warmup 5 > gpurun_out/bench_bert_j.json 2> gpurun_out/bench_bert_j.err || exit $?
cat gpurun_out/bench_bert_j.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_moe_dts -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model moe --moe-gate dts --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_moe_dts.log 2>&1
echo prof rc=$?
