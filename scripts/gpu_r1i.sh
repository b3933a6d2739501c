#!/bin/bash
# GPU session: build, targeted GPU tests, BERT/MoE benches (topk + dts), BERT profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_fused_gpu.py tests/test_ops_differential_gpu.py tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_i.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/pytest_gpu_i.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_i.log | head; tail -2 gpurun_out/pytest_gpu_i.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --model bert --steps 20 --warmup 5 > gpurun_out/bench_bert_i.json 2> gpurun_out/bench_bert_i.err || exit $?
cat gpurun_out/bench_bert_i.json
timeout -k 10 300 python bench.py --model moe --moe-gate dts --steps 20 --warmup 5 > gpurun_out/bench_moe_dts_i.json 2> gpurun_out/bench_moe_dts_i.err || exit $?
tail -1 gpurun_out/bench_moe_dts_i.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert_i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert_i.log 2>&1
echo prof rc=$?
