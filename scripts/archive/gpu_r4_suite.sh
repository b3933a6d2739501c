#!/bin/bash
# Round-4: the driver's round-end GPU tier (smoke + pytest -m gpu), then a same-box
# allocator A/B on ResNet-50 (BFC pool as the device allocator vs torch's caching
# allocator, alternating).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_driver_suite.sh || exit $?
S=scripts/gpu_step.sh
if [ -n "${AB:-1}" ]; then
  for a in bfc torch bfc torch; do
    HETU_ALLOCATOR=$a bash $S b_resnet50_ab_$a 300 python bench.py --model resnet50 --steps 20 --warmup 5 || exit $?
    cp gpurun_out/b_resnet50_ab_$a.log gpurun_out/b_resnet50_ab_${a}_$(date +%s).log
  done
fi
