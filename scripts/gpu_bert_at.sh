#!/bin/bash
# BERT-base bench line with the per-shape autotune decisions
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
HETU_AUTOTUNE_DUMP=gpurun_out/at_bert.txt timeout -k 10 240 python bench.py --model bert --steps 20 --warmup 5 > gpurun_out/bert.json 2>/dev/null || exit $?
cut -c1-200 gpurun_out/bert.json
grep -v -- '-> hip' gpurun_out/at_bert.txt | cut -c1-200
echo "hand=$(grep -c -- '-> hip' gpurun_out/at_bert.txt) lib=$(grep -vc -- '-> hip' gpurun_out/at_bert.txt)"
