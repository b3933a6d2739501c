#!/bin/bash
# Steady-state PMC passes: eager steps (HETU_HIPGRAPH=0, so every
# dispatch is visible), no census step, the kernels a plain run's autotune chose, the last 3
# steps' dispatches only (pmc_summary.py --marker opt_flat2_k --steps 3): per-family MFMA busy fraction, waits, LDS bank
# conflicts, HBM read/write rates, TF/s from MFMA op counts, HBM bytes per step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp HETU_HIPGRAPH=0 HETU_BENCH_CENSUS=0
cd /tmp
M=${PMC_MODEL:-bert}
# the kernels a plain run chooses: tune once without the profiler, then every PMC pass takes
# those decisions (serialised PMC dispatches would time the candidates differently)
export HETU_AUTOTUNE_CACHE=/tmp/pmc6_tune_$M.json
HETU_AUTOTUNE_SAVE=$HETU_AUTOTUNE_CACHE timeout -k 10 300 python3 $R/bench.py --model $M --steps 10 --warmup 3 \
  > $R/gpurun_out/pmc6_${M}_plain.json 2>&1 || exit $?
tail -1 $R/gpurun_out/pmc6_${M}_plain.json | cut -c1-200
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
rc=$?
# summarise on the box (the raw per-dispatch CSVs exceed gpurun's copy-back cap)
# window = the last 3 steps, delimited by the once-per-step optimizer launch
D=$R/gpurun_out/pmc6_$M
python3 $R/scripts/pmc_summary.py --marker opt_flat2_k --steps 3 ${D}_sq ${D}_mem ${D}_wr ${D}_mops > $R/gpurun_out/pmc6_${M}_summary.txt 2>&1
echo "summary rc=$?"; head -30 $R/gpurun_out/pmc6_${M}_summary.txt
tail -3 $R/gpurun_out/pmc6_${M}_sq.log
rm -rf ${D}_sq ${D}_mem ${D}_wr ${D}_mops
exit $rc
