#!/bin/bash
# End-of-round evidence: BERT-base steady-state rocprofv3 trace, MoE and Wide&Deep bench lines.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in bert moe wdl; do
  timeout -k 10 240 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/end_$m.json 2> gpurun_out/end_$m.err || { tail -20 gpurun_out/end_$m.err; exit 1; }
  cut -c1-200 gpurun_out/end_$m.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bert -o run --output-format csv -- python3 $R/bench.py --model bert --steps 5 --warmup 3 > $R/gpurun_out/prof_bert.log 2>&1
rc=$?; cd $R; tail -2 gpurun_out/prof_bert.log; exit $rc
