#!/bin/bash
# Round-5: every autotune candidate agrees (MoE dts / top-k, BERT steps); narrow-output
# tiles; gmask epilogue prefetch; MoE bench + profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 800 $T tests/test_autotune_candidates_gpu.py tests/test_gemm_gpu.py -k "candidates or narrow or relu_mask" > gpurun_out/r5t_tests.log 2>&1
rc=$?; grep -E "passed|failed|^E .*\(|AssertionError" gpurun_out/r5t_tests.log | head -30; case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python3 bench.py --model moe --steps 20 --warmup 5 > gpurun_out/r5t_moe.json 2> gpurun_out/r5t_moe.err
rc=$?; tail -1 gpurun_out/r5t_moe.json | cut -c1-160; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5t_moe.err; exit $rc; }
MODEL=moe bash scripts/gpu_prof_model.sh > /dev/null 2>&1 || exit $?
head -8 gpurun_out/prof_moe_steady.txt
