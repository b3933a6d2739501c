#!/bin/bash
# Steady-state kernel trace of one bench model at the defaults: per-family summary
# (prof_steps.py) and per-(kernel, grid) table (prof_shapes.py).  MODEL=bert|resnet50|...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
M=${MODEL:-bert}
cd /tmp && HETU_HIPGRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$M -o run --output-format csv \
  -- python3 $R/bench.py --model $M --steps 5 --warmup 3 > $R/gpurun_out/prof_$M.log 2>&1
rc=$?; cd $R; tail -2 gpurun_out/prof_$M.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$M -name "*kernel_trace.csv" | head -1)
python scripts/prof_steps.py "$f" --last 3 > gpurun_out/prof_${M}_steady.txt 2>&1; head -30 gpurun_out/prof_${M}_steady.txt
python scripts/prof_shapes.py "$f" --top 100 > gpurun_out/prof_${M}_shapes.txt 2>&1
