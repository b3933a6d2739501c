#!/bin/bash
# Kernel-time A/B (BERT-base): rocprofv3 kernel traces of ab_old and the working tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
cd /tmp
for v in old new; do
  if [ $v = old ]; then B=$R/ab_old; else B=$R; fi
  PYTHONPATH=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lnprof_$v -o run --output-format csv \
    -- python3 $B/bench.py --model bert --steps 5 --warmup 3 > $R/gpurun_out/lnprof_$v.log 2>&1 || { tail -5 $R/gpurun_out/lnprof_$v.log; exit 1; }
  echo "$v done"
done
