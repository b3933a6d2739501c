#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench.py --model wdl --steps 60 --warmup 10 > gpurun_out/bench_wdl_l.json 2> gpurun_out/bench_wdl_l.err || exit $?
cat gpurun_out/bench_wdl_l.json
timeout -k 10 300 python bench.py --model wdl --steps 60 --warmup 10 --no-prefetch > gpurun_out/bench_wdl_nopf_l.json 2> gpurun_out/bench_wdl_nopf_l.err || exit $?
cat gpurun_out/bench_wdl_nopf_l.json
timeout -k 10 300 python bench.py --model wdl --steps 60 --warmup 10 --op-profile gpurun_out/wdl_ops_l.txt > /dev/null 2>&1 || exit $?
cat gpurun_out/wdl_ops_l.txt
