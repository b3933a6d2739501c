#!/bin/bash
# Experiment run: GEMM/conv tests, autotuned ResNet-50 bench + profile, WDL (PS + HET cache) bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
echo "== build"; make -C csrc -j16 > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
echo "== gemm tests"
timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
echo "== bench auto"
HETU_AUTOTUNE_DUMP=gpurun_out/autotune.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err || { tail -20 gpurun_out/bench_auto.err; exit 1; }
cat gpurun_out/bench_auto.json
echo "== wdl small"
timeout -k 10 300 python bench.py --model wdl --criteo-rows 2000000 --steps 50 --warmup 10 > gpurun_out/bench_wdl_small.json 2> gpurun_out/bench_wdl_small.err || { tail -30 gpurun_out/bench_wdl_small.err; exit 1; }
cat gpurun_out/bench_wdl_small.json
echo "== rocprofv3 auto"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_auto -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_auto.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/prof_auto.log; exit $rc
