#!/bin/bash
# Round-5: asm fragment reads only in the double-buffered K loops (ST 2 / 3); harness,
# BERT / ResNet-50 (c64 wgrad asm A/B) / MoE benches, BERT + ResNet kernel profiles, memops.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py tests/test_fused_gpu.py > gpurun_out/r5m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5m_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
OUT=gpurun_out/gemm_r5m.txt FVARS=0:1,1:1,3:1,5:1,6:1,7:1 WVARS=0:4,0:7,3:4,3:7,6:4,6:7,1:4,1:7 bash scripts/gpu_r5_gemm.sh > /dev/null 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
for m in bert moe; do
  timeout -k 10 400 python3 bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r5m_$m.json 2> gpurun_out/r5m_$m.err
  rc=$?; tail -1 gpurun_out/r5m_$m.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5m_$m.err; exit $rc; }
done
for a in 0 1 0 1; do
  HETU_C64_WGRAD_ASM=$a timeout -k 10 400 python3 bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/r5m_resnet_asm$a.json 2> gpurun_out/r5m_resnet.err
  rc=$?; echo "asm=$a $(tail -1 gpurun_out/r5m_resnet_asm$a.json | cut -c1-140)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5m_resnet.err; exit $rc; }
done
MODEL=bert bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
MODEL=resnet50 bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_memops -o memops -- python3 $R/scripts/bench_memops.py > $R/gpurun_out/r5m_memops.log 2>&1
rc=$?; cd $R; find gpurun_out/prof_memops -name "*kernel_stats.csv" | head -1 | xargs -r cp -t gpurun_out/ ; exit $rc
