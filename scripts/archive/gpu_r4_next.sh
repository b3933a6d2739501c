#!/bin/bash
# Round-4: BFC-as-device-allocator + native hipGraph capture tests, ResNet-50 allocator
# A/B, Wide&Deep PS bench lines, steady-state PMC passes (scripts/gpu_r4_wdl_pmc.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S tests_next 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_memory_pool_gpu.py tests/test_models_gpu.py::test_hipgraph_mlp_matches_eager tests/test_bn_fusion_gpu.py} || exit $?
grep -q " passed" gpurun_out/tests_next.log && ! grep -q -E "[0-9]+ failed|[0-9]+ error" gpurun_out/tests_next.log || { echo "TESTS FAILED"; exit 1; }
if [ -n "${AB:-1}" ]; then
  for a in bfc torch; do
    HETU_ALLOCATOR=$a bash $S b_resnet50_alloc_$a 300 python bench.py --model resnet50 --steps 20 --warmup 5 || exit $?
  done
fi
bash scripts/gpu_r4_wdl_pmc.sh
