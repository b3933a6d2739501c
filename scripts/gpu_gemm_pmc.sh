#!/bin/bash
# GEMM kernel A/B on the GPU box: the same-process tile-vs-hipBLASLt timing table
# (csrc/build/gemm_bench, built in the container with `make -C csrc bench`), then
# PMC passes over one shape (GEMM_SHAPE, default 8192^3 NT) for every variant.
#   gpurun -- bash scripts/gpu_gemm_pmc.sh
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
B=$R/csrc/build/gemm_bench
timeout -k 10 180 $B ${GEMM_SHAPES:-} > $R/gpurun_out/gemm_bench.txt 2>&1
rc=$?; cat $R/gpurun_out/gemm_bench.txt
[ $rc -eq 0 ] || exit $rc
[ "${PMC:-1}" = "1" ] || exit 0
SHAPE=${GEMM_SHAPE:-8192 8192 8192 0 1}
cd /tmp
pass() {
  name=$1; shift
  ROUNDS=1 REPS=3 timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/gpurun_out/gpmc_$name -o run --output-format csv \
    -- $B $SHAPE > $R/gpurun_out/gpmc_$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  && pass mem FETCH_SIZE SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  && pass l2 TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  && cd $R && python3 scripts/pmc_summary.py gpurun_out/gpmc_sq gpurun_out/gpmc_mem gpurun_out/gpmc_l2 > gpurun_out/gemm_pmc.txt 2>&1
rc=$?; cat $R/gpurun_out/gemm_pmc.txt 2>/dev/null | head -30
exit $rc
