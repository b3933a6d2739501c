#!/bin/bash
# Parallel-equivalence suite (reference examples/runner/parallel/all_mlp_tests.sh):
# baseline, pipeline (GPipe, 1F1B), data+pipeline, model-parallel splits; every
# layout must reproduce the baseline losses.  HETU_CPU=1 rehearses it on CPU (gloo).
set -e
cd "$(dirname "$0")"
R=../../../bin/heturun
S=mlp_parallel.py
rm -rf results
python $S --mode base ${HETU_CPU:+--cpu}
$R -w 2 python $S --mode pp --schedule gpipe
$R -w 4 python $S --mode pp --schedule pipedream
$R -w 4 python $S --mode dp_pp --replicas 2 --schedule gpipe
for s in left right middle; do $R -w 2 python $S --mode mp --split $s; done
$R -w 4 python complex_pipeline_mlp.py
$R -w 2 -s 1 python $S --mode pp --schedule hetpipe
$R -w 4 -s 1 python $S --mode dp_pp --replicas 2 --schedule hetpipe
python validate_results.py
