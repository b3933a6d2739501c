#!/bin/bash
# Round-5: sparse softmax-CE ignored rows: kernel tests, BERT bench x2, BERT profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_models_gpu.py -k "softmax or ce or bert" > gpurun_out/r5z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5z_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r5z_bert$i.json 2> gpurun_out/r5z_bert.err
  rc=$?; tail -1 gpurun_out/r5z_bert$i.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5z_bert.err; exit $rc; }
done
MODEL=bert bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -24 gpurun_out/prof_bert_steady.txt
