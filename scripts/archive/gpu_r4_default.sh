#!/bin/bash
# Round-4: the driver's round-end tier at HEAD defaults (BFC device allocator, hand-written
# kernels only, BN epilogue fusion): smoke + pytest -m gpu, then every bench model once.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_driver_suite.sh || exit $?
S=scripts/gpu_step.sh
for m in ${MODELS:-resnet50 bert moe wdl}; do
  bash $S b_def_$m 300 python bench.py --model $m --steps 20 --warmup 5 || exit $?
done
