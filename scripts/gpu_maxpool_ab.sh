#!/bin/bash
# ResNet-50 max-pool backward: one block per input row vs the flat form (HETU_MAXPOOL_FLAT=1)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py > $O/mp_tests.txt 2>&1
rc=$?; tail -1 $O/mp_tests.txt; [ $rc = 0 ] || exit $rc
for f in 1 0; do
  if [ $f = 1 ]; then export HETU_MAXPOOL_FLAT=1; else unset HETU_MAXPOOL_FLAT; fi
  MODEL=resnet50 bash scripts/gpu_prof_model.sh > /dev/null || exit $?
  echo "flat=$f $(grep -E 'kernel time' $O/prof_resnet50_shapes.txt) $(grep -E 'maxpool_bwd' $O/prof_resnet50_shapes.txt)"
  mv $O/prof_resnet50_shapes.txt $O/mp_shapes_flat$f.txt; rm -rf $O/prof_resnet50
done
for i in 1 2; do
  for f in 1 0; do
    if [ $f = 1 ]; then export HETU_MAXPOOL_FLAT=1; else unset HETU_MAXPOOL_FLAT; fi
    timeout -k 10 300 python -u bench.py > $O/mp_rn_$f$i.json 2>/dev/null || exit $?
    echo "flat=$f $i $(python3 -c "import json;d=json.loads(open('$O/mp_rn_$f$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
