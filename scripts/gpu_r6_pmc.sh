#!/bin/bash
# Steady-state PMC passes: eager steps (HETU_HIPGRAPH=0, so every
# dispatch is visible), no census step, the last STEPS steps' dispatches only
# (pmc_summary.py --last N --steps S): per-family MFMA busy fraction, waits, LDS bank
# conflicts, HBM read/write rates, TF/s from MFMA op counts, HBM bytes per step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp HETU_HIPGRAPH=0 HETU_BENCH_CENSUS=0
cd /tmp
M=${PMC_MODEL:-bert}
pass() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc6_${M}_$name -o run --output-format csv \
    -- python3 $R/bench.py --model $M --steps 3 --warmup 2 > $R/gpurun_out/pmc6_${M}_$name.log 2>&1
  rc=$?
  echo "pass $M $name rc=$rc"
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  && pass mem FETCH_SIZE SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  && pass wr WRITE_SIZE GRBM_GUI_ACTIVE \
  && pass mops SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE
