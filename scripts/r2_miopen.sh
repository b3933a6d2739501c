#!/bin/bash
# A/B of the MIOpen solver selection behind the vendor convolution candidates
# (ResNet-50 bench): immediate-mode default vs the GTC NHWC assembly solvers
# (which zero-fill their outputs first) disabled.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
run() {
  tag=$1; shift
  echo "== $tag"
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/miopen_$tag.json 2> gpurun_out/miopen_$tag.err
  rc=$?; cat gpurun_out/miopen_$tag.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/miopen_$tag.err; exit $rc; }
  return 0
}
NOGTC="MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0"
run base HETU_X=0 &&

run nogtc $NOGTC &&

run base2 HETU_X=0
