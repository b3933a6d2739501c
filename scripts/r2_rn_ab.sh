#!/bin/bash
# split-K sum tests, then alternating ResNet-50 benches: ab_old (previous commit) vs working tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest tests/test_gemm_splitk_gpu.py tests/test_models_gpu.py -x -q --capture=sys \
  --timeout 120 --timeout-method thread > gpurun_out/rn_tests.log 2>&1 || { tail -30 gpurun_out/rn_tests.log; exit 1; }
tail -2 gpurun_out/rn_tests.log
for i in 1 2; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 20 --warmup 5 > ../gpurun_out/rn_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/rn_new_$i.log 2>&1 || exit 1
  grep -ho '"value": [0-9.]*' gpurun_out/rn_old_$i.log gpurun_out/rn_new_$i.log
done
