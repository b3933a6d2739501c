#!/bin/bash
# Round-5: pre-activation and dropout epilogues as separate builds (no SGPR/VGPR spill in
# the 4-blocks-per-CU GELU tile); LN backward back at 4 waves; tests, BERT / MoE benches
# and the BERT kernel profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_gemm_gpu.py tests/test_fused_gpu.py tests/test_moe_gpu.py tests/test_models_gpu.py > gpurun_out/r5n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5n_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for m in bert moe bert; do
  timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5n_$m.json 2> gpurun_out/r5n_$m.err
  rc=$?; tail -1 gpurun_out/r5n_$m.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5n_$m.err; exit $rc; }
done
MODEL=bert bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -14 gpurun_out/prof_bert_steady.txt
