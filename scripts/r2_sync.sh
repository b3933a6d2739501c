#!/bin/bash
# Sync-free small-table dedup: GPU tests, then alternating BERT benches (old/new) and profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_deterministic_gpu.py -x -q \
  --capture=sys --timeout 120 --timeout-method thread > gpurun_out/sync_tests.log 2>&1 || { tail -30 gpurun_out/sync_tests.log; exit 1; }
tail -2 gpurun_out/sync_tests.log
for i in 1 2 3; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 40 --warmup 5 > ../gpurun_out/sync_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 40 --warmup 5 > gpurun_out/sync_new_$i.log 2>&1 || exit 1
  grep -ho '"value": [0-9.]*' gpurun_out/sync_old_$i.log gpurun_out/sync_new_$i.log
done
bash scripts/r2_ln_prof.sh
