#!/bin/bash
# Same-process GEMM A/B (hand-written tiles incl. split-K vs hipBLASLt) on BERT-base's
# GEMM shapes.  The harness binary is built on the CPU side (make -C csrc bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=csrc/build/gemm_bench
OUT=${OUT:-gpurun_out/gemm_r5.txt}
: > "$OUT"
FWD="8192 2304 768 0 0  8192 768 768 0 0  8192 3072 768 0 0  8192 768 3072 0 0  8192 768 2304 0 1  8192 768 3072 0 1  8192 3072 768 0 1  4096 4096 4096 0 0"
WG="768 2304 8192 1 0  768 768 8192 1 0  768 3072 8192 1 0  3072 768 8192 1 0"
echo "== fwd/dgrad" | tee -a "$OUT"
VARS=${FVARS:-0:1,1:1,3:1,5:1} timeout -k 10 240 $B $FWD >> "$OUT" 2>&1 || exit $?
echo "== wgrad (fp32 out)" | tee -a "$OUT"
WGRAD_F32=1 VARS=${WVARS:-0:4,0:7,3:4,3:7,3:8,1:4,1:7,1:8} timeout -k 10 240 $B $WG >> "$OUT" 2>&1 || exit $?
cat "$OUT"
