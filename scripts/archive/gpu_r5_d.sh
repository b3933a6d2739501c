#!/bin/bash
# Round-5 benches: driver-form default runs of every BASELINE config, hipGraph A/B for
# ResNet-50 / BERT, MoE top-2 and DTS, WDL PS (with a host profile of extra steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  echo "== $n"
  timeout -k 10 $t python3 bench.py "$@" > gpurun_out/r5d_$n.json 2> gpurun_out/r5d_$n.err
  local rc=$?
  tail -1 gpurun_out/r5d_$n.json | cut -c1-700
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/r5d_$n.err; exit $rc; fi
}
run resnet50 400 --model resnet50 --steps 20 --warmup 5
run bert 400 --model bert --steps 20 --warmup 5
HETU_HIPGRAPH=1 run resnet50_graph 400 --model resnet50 --steps 20 --warmup 5
HETU_HIPGRAPH=1 run bert_graph 400 --model bert --steps 20 --warmup 5
run moe_topk 400 --model moe --steps 10 --warmup 3
run moe_dts 400 --model moe --moe-gate dts --steps 10 --warmup 3
HETU_BENCH_PYPROF=gpurun_out/r5d_wdl_pyprof.txt run wdl 400 --model wdl --steps 60 --warmup 10
run logreg 200 --model logreg --steps 200 --warmup 20
