#!/bin/bash
# Round 6: WDL stray-kernel census + host profile, BERT / MoE bench lines (hipGraph default),
# steady-state rocprofv3 traces of ResNet-50 and BERT.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/find_torch_kernels.py --model wdl > gpurun_out/r6d_wdl_kernels.txt 2>&1
rc=$?; tail -15 gpurun_out/r6d_wdl_kernels.txt; [ $rc -eq 0 ] || exit $rc
HETU_BENCH_PYPROF=gpurun_out/r6d_wdl_pyprof.txt timeout -k 10 200 python3 bench.py --model wdl --steps 100 --warmup 20 \
  > gpurun_out/r6d_wdl.json 2> gpurun_out/r6d_wdl.err
rc=$?; tail -c 600 gpurun_out/r6d_wdl.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r6d_bert.json 2> gpurun_out/r6d_bert.err
rc=$?; tail -c 400 gpurun_out/r6d_bert.json; [ $rc -eq 0 ] || exit $rc
HETU_HIPGRAPH=0 timeout -k 10 300 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/r6d_bert_eager.json 2> gpurun_out/r6d_bert_eager.err
rc=$?; tail -c 300 gpurun_out/r6d_bert_eager.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model moe --steps 20 --warmup 5 > gpurun_out/r6d_moe.json 2> gpurun_out/r6d_moe.err
rc=$?; tail -c 300 gpurun_out/r6d_moe.json; [ $rc -eq 0 ] || exit $rc
MODEL=resnet50 bash scripts/gpu_prof_model.sh || exit $?
MODEL=bert bash scripts/gpu_prof_model.sh || exit $?
