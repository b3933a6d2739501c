#!/bin/bash
# Round 6: per-shape ResNet-50 conv table, the 8-worker Wide&Deep PS run on the one GPU,
# the 16-expert dense-to-sparse schedule, BERT / WDL / MoE bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bench_conv_resnet.py 256 gpurun_out/r6c_conv_shapes.txt > gpurun_out/r6c_conv.log 2>&1
rc=$?; tail -2 gpurun_out/r6c_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --model wdl --steps 100 --warmup 20 > gpurun_out/r6c_wdl1.json 2> gpurun_out/r6c_wdl1.err
rc=$?; tail -1 gpurun_out/r6c_wdl1.json; [ $rc -eq 0 ] || exit $rc
STEPS=100 WARMUP=20 bash scripts/gpu_wdl8_one_gpu.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --model moe --moe-gate dts --moe-local-experts 16 --dts-schedule 2.0,0.97,0.05 \
  --steps 150 --warmup 2 > gpurun_out/r6c_dts16.json 2> gpurun_out/r6c_dts16.err
rc=$?; tail -c 1500 gpurun_out/r6c_dts16.json; [ $rc -eq 0 ] || exit $rc
