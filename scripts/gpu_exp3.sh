#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
echo "== build"; make -C csrc -j16 > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
echo "== gemm tests"
timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
echo "== gemm bench"
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || { tail -20 gpurun_out/bench_gemm.log; exit 1; }
tail -12 gpurun_out/bench_gemm.log
echo "== diag vendor"
timeout -k 10 200 python scripts/diag_conv.py > gpurun_out/diag_conv.log 2>&1 || { tail -20 gpurun_out/diag_conv.log; exit 1; }
echo "== bench auto"
HETU_AUTOTUNE_DUMP=gpurun_out/autotune.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err || { tail -20 gpurun_out/bench_auto.err; exit 1; }
cat gpurun_out/bench_auto.json
echo "== rocprofv3 auto"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_auto -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_auto.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; exit $rc
