#!/bin/bash
# Round-5: ds_read_tr as inline asm (no vmcnt(0) before MN-major fragment reads) and the
# two-ahead K loop (tiles 6 / 7): GEMM / conv tests, BERT-shape harness, memops kernel
# profile, BERT / ResNet-50 / MoE benches.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 700 $T tests/test_gemm_gpu.py tests/test_gemm_splitk_gpu.py tests/test_stem_gpu.py tests/test_fused_gpu.py tests/test_bn_fusion_gpu.py > gpurun_out/r5l_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5l_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
OUT=gpurun_out/gemm_r5l.txt FVARS=0:1,1:1,3:1,5:1,6:1,7:1 WVARS=0:4,3:4,3:7,6:4,6:7,1:4,1:7 bash scripts/gpu_r5_gemm.sh > /dev/null 2>&1
rc=$?; cat gpurun_out/gemm_r5l.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for m in bert resnet50 moe; do
  timeout -k 10 400 python3 bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r5l_$m.json 2> gpurun_out/r5l_$m.err
  rc=$?; tail -1 gpurun_out/r5l_$m.json | cut -c1-200; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5l_$m.err; exit $rc; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_memops -o memops -- python3 scripts/bench_memops.py > gpurun_out/r5l_memops.log 2>&1
rc=$?; find gpurun_out/prof_memops -name "*kernel_stats.csv" | head -1 | xargs -r head -20 | cut -c1-160; exit $rc
