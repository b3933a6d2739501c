#!/bin/bash
# Round-5 perf pass: attention kernels (fused vs flash), BERT / ResNet-50 / MoE benches
# (eager vs hipGraph replay), WDL PS bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== attention kernels"
timeout -k 10 300 python3 scripts/bench_attn.py > gpurun_out/r5b_attn.txt 2>&1
rc=$?; cat gpurun_out/r5b_attn.txt | tail -20; [ $rc -eq 0 ] || exit $rc
for m in bert resnet50; do
  echo "== bench $m"
  timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5b_$m.json 2> gpurun_out/r5b_$m.err
  rc=$?; tail -1 gpurun_out/r5b_$m.json | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5b_$m.err; exit $rc; }
  echo "== bench $m hipgraph"
  HETU_HIPGRAPH=1 timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5b_${m}_graph.json 2> gpurun_out/r5b_${m}_graph.err
  rc=$?; tail -1 gpurun_out/r5b_${m}_graph.json | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5b_${m}_graph.err; exit $rc; }
done
echo "== moe benches"
timeout -k 10 300 python3 bench.py --model moe --steps 10 --warmup 3 > gpurun_out/r5b_moe_topk.json 2> gpurun_out/r5b_moe_topk.err
rc=$?; tail -1 gpurun_out/r5b_moe_topk.json | cut -c1-500; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5b_moe_topk.err; exit $rc; }
timeout -k 10 300 python3 bench.py --model moe --moe-gate dts --steps 10 --warmup 3 > gpurun_out/r5b_moe_dts.json 2> gpurun_out/r5b_moe_dts.err
rc=$?; tail -1 gpurun_out/r5b_moe_dts.json | cut -c1-800; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5b_moe_dts.err; exit $rc; }
echo "== bench wdl"
timeout -k 10 400 python3 bench.py --model wdl --steps 60 --warmup 10 > gpurun_out/r5b_wdl.json 2> gpurun_out/r5b_wdl.err
rc=$?; tail -1 gpurun_out/r5b_wdl.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5b_wdl.err; exit $rc; }
