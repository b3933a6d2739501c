#!/bin/bash
# Benchmarks + GEMM counter passes on one GPU box:
#   ResNet-50 and BERT bench lines, then rocprofv3 --pmc passes over
#   scripts/gemm_prof_driver.py (one counter set per run).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$R
for m in ${BENCH_MODELS:-resnet50 bert}; do
  timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/perf_$m.json 2> gpurun_out/perf_$m.err
  rc=$?; echo "bench $m rc=$rc"; cat gpurun_out/perf_$m.json; tail -2 gpurun_out/perf_$m.err
  [ $rc -eq 0 ] || exit $rc
done
[ "${PMC:-1}" = "1" ] || exit 0
cd /tmp
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/gpmc_$name -o run --output-format csv \
    -- python3 $R/scripts/gemm_prof_driver.py 10 > $R/gpurun_out/gpmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  && pass lds SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE
