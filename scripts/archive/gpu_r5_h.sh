#!/bin/bash
# Round-5 steady-state kernel traces (rocprofv3 --kernel-trace --stats) of BERT, ResNet-50, MoE.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for m in bert resnet50 moe; do
  echo "== prof $m"
  MODEL=$m bash scripts/gpu_prof_model.sh || exit $?
done
