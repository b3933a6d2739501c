#!/bin/bash
# Round-5 closing check: optimizer / softmax-CE kernel tests, BERT bench x2 + profile, then the
# whole GPU suite, smoke and the default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "optimizer or softmax or ce" > gpurun_out/r5aa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5aa_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5aa_bert$i.json 2> gpurun_out/r5aa_bert.err
  rc=$?; tail -1 gpurun_out/r5aa_bert$i.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5aa_bert.err; exit $rc; }
done
MODEL=bert bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
grep "opt_flat\|sce_sparse" gpurun_out/prof_bert_steady.txt
TAG=r5aa bash scripts/gpu_full_suite.sh
