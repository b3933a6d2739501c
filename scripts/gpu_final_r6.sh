#!/bin/bash
# Round-6 closing check: the driver-form GPU tier (smoke + pytest -m gpu), then the default
# bench line and the MoE / BERT / Wide&Deep bench lines at HEAD
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
cd $R
PYTEST_ARGS="--timeout 300 --timeout-method thread" TEST_TIMEOUT=600 bash scripts/gpu_driver_suite.sh || exit $?
timeout -k 10 300 python -u bench.py > $O/fin_resnet.json 2> $O/fin_resnet.err || exit $?
tail -1 $O/fin_resnet.json | cut -c1-200
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model moe --steps 20 --warmup 5 > $O/fin_moe_$i.json 2> $O/fin_moe_$i.err || exit $?
  tail -1 $O/fin_moe_$i.json | cut -c1-160
done
timeout -k 10 300 python -u bench.py --model bert --steps 20 --warmup 5 > $O/fin_bert.json 2> $O/fin_bert.err || exit $?
tail -1 $O/fin_bert.json | cut -c1-160
timeout -k 10 300 python -u bench.py --model wdl --steps 200 --warmup 20 > $O/fin_wdl.json 2> $O/fin_wdl.err || exit $?
tail -1 $O/fin_wdl.json | cut -c1-160
