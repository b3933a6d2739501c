#!/bin/bash
# Round-5: gradient-mask GEMM epilogue (MoE expert ReLU/dropout backward) tests + benches, and
# the DTS gate's sparsification with the segmented locations scan on / off.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_gemm_gpu.py -k "relu_mask or act_dropout or matmul_pre" tests/test_models_gpu.py -k "moe" tests/test_moe_gpu.py > gpurun_out/r5r_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5r_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for env in "HETU_MOE_LOC_SEGMENTED=1" "HETU_MOE_LOC_SEGMENTED=0" "HETU_GMASK_EPILOGUE=0"; do
  tag=$(echo $env | tr '=' '_')
  env $env timeout -k 10 400 python3 bench.py --model moe --moe-gate dts --steps 10 --warmup 3 > gpurun_out/r5r_dts_$tag.json 2> gpurun_out/r5r_dts.err
  rc=$?; echo "$env $(tail -1 gpurun_out/r5r_dts_$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["dts"])')"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5r_dts.err; exit $rc; }
done
for g in topk; do
  timeout -k 10 400 python3 bench.py --model moe --moe-gate $g --steps 20 --warmup 5 > gpurun_out/r5r_moe_$g.json 2> gpurun_out/r5r_moe.err
  rc=$?; tail -1 gpurun_out/r5r_moe_$g.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5r_moe.err; exit $rc; }
done
MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -16 gpurun_out/prof_moe_steady.txt
