#!/bin/bash
# Round-4: Wide&Deep PS-mode bench lines (uniform and zipf ids, Hybrid for contrast),
# then steady-state PMC passes (rocprofv3 --pmc only) over ResNet-50 and BERT.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
if [ "${WDL:-1}" != "0" ]; then
  for ids in zipf uniform; do
    bash $S wdl_ps_$ids 300 python bench.py --model wdl --comm PS --ids $ids --steps 40 --warmup 10 || exit $?
  done
  bash $S wdl_hybrid_zipf 300 python bench.py --model wdl --comm Hybrid --ids zipf --steps 40 --warmup 10 || exit $?
fi
pass() {
  model=$1; name=$2; shift 2
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc4_${model}_$name -o run --output-format csv \
    -- python3 $R/bench.py --model $model --steps 4 --warmup 2 > $R/gpurun_out/pmc4_${model}_$name.log 2>&1
  rc=$?; cd $R
  echo "pass $model $name rc=$rc"; tail -2 gpurun_out/pmc4_${model}_$name.log
  return $rc
}
for m in ${PMC_MODELS:-resnet50 bert}; do
  pass $m sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit $?
  pass $m mem FETCH_SIZE SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit $?
  pass $m wr WRITE_SIZE GRBM_GUI_ACTIVE || exit $?
done
for m in ${PMC_MODELS:-resnet50 bert}; do   # MFMA op counts (bf16 MOPs: 512 flops each)
  pass $m mops SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE || exit $?
done
