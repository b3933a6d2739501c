#!/bin/bash
# Same-box A/B for the LayerNorm-backward linear-bias fusion (BERT-base):
# new-kernel GPU tests first, then alternating old/new BERT benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -x -q --capture=sys \
  --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -2 gpurun_out/ln_tests.log
for i in 1 2 3 4; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 60 --warmup 10 > ../gpurun_out/ln_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 60 --warmup 10 > gpurun_out/ln_new_$i.log 2>&1 || exit 1
  grep -ho '"value": [0-9.]*' gpurun_out/ln_old_$i.log gpurun_out/ln_new_$i.log
done
