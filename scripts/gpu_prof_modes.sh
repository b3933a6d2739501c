#!/bin/bash
# Steady-state kernel breakdown of one model under two dispatch modes
# (HETU_GEMM/HETU_CONV = auto vs hip): rocprofv3 kernel traces summarised by
# scripts/prof_steps.py into gpurun_out/steady_<model>_<mode>.txt.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONPATH=$R
M=${MODEL:-bert}
for mode in ${MODES:-auto hip}; do
  (cd /tmp && HETU_GEMM=$mode HETU_CONV=$mode timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/ptrace_${M}_$mode \
     -o run --output-format csv -- python3 $R/bench.py --model $M --steps 6 --warmup 4 \
     > $R/gpurun_out/ptrace_${M}_$mode.log 2>&1)
  rc=$?; echo "trace $M $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ptrace_${M}_$mode.log; exit $rc; }
  f=$(ls gpurun_out/ptrace_${M}_$mode/*/run_kernel_trace.csv gpurun_out/ptrace_${M}_$mode/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/prof_steps.py $f --last 3 --top 45 ${CONTEXT:-} > gpurun_out/steady_${M}_$mode.txt
  head -30 gpurun_out/steady_${M}_$mode.txt
  rm -f $f
done
