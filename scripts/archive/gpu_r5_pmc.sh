#!/bin/bash
# Round-5 PMC at HEAD: BERT-base and ResNet-50 steady steps, three counter passes each
# (gpu_pmc.sh), summarised per kernel family.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in bert resnet50; do
  PMC_MODEL=$m PMC_TIMEOUT=240 bash scripts/gpu_pmc.sh || exit $?
  cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_mem gpurun_out/pmc_wr > gpurun_out/pmc_${m}_r5.txt 2>&1
  head -14 gpurun_out/pmc_${m}_r5.txt
  rm -rf gpurun_out/pmc_sq gpurun_out/pmc_mem gpurun_out/pmc_wr
done
