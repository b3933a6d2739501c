#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --pmc only, no tracing domains)
# over a short ResNet-50 bench run.  Output: gpurun_out/pmc_<pass>/run_counter_collection.csv
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
MODEL=${PMC_MODEL:-resnet50}
pass() {
  name=$1; shift
  timeout -s KILL ${PMC_TIMEOUT:-300} rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$name -o run --output-format csv \
    -- python3 $R/bench.py --model $MODEL --steps 2 --warmup 1 > $R/gpurun_out/pmc_$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"; tail -2 $R/gpurun_out/pmc_$name.log
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  && pass mem FETCH_SIZE SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  && pass wr WRITE_SIZE GRBM_GUI_ACTIVE
