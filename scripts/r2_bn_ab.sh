#!/bin/bash
# Same-box A/B of BatchNorm kernel changes: ab_old = previous build, . = working tree.
# BN GPU tests first, then the BN bandwidth sweep and alternating ResNet-50 runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --capture=sys --timeout 120 --timeout-method thread \
  -k "bn or batch_norm or batchnorm or resnet" > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
(cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python scripts/bench_bn.py > ../gpurun_out/ab_bn_old.txt 2>&1) || exit 1
PYTHONPATH=$PWD timeout -k 10 200 python scripts/bench_bn.py > gpurun_out/ab_bn_new.txt 2>&1 || exit 1
for i in 1 2; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 20 --warmup 5 > ../gpurun_out/ab_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  grep -h value gpurun_out/ab_old_$i.log gpurun_out/ab_new_$i.log | cut -c1-110
done
