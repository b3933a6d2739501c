#!/bin/bash
# ResNet-50 stem forward: 16-byte input staging vs the element-wise loop (HETU_STEM_SCALAR=1)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py tests/test_bn_fusion_gpu.py > $O/stem_tests.txt 2>&1
rc=$?; tail -1 $O/stem_tests.txt; [ $rc = 0 ] || exit $rc
for f in 1 0; do
  if [ $f = 1 ]; then export HETU_STEM_SCALAR=1; else unset HETU_STEM_SCALAR; fi
  MODEL=resnet50 bash scripts/gpu_prof_model.sh > /dev/null || exit $?
  echo "scalar=$f $(grep -E 'kernel time' $O/prof_resnet50_shapes.txt) $(grep -E 'stem_fwd_k' $O/prof_resnet50_shapes.txt)"
  mv $O/prof_resnet50_shapes.txt $O/stem_shapes_scalar$f.txt; rm -rf $O/prof_resnet50
done
for i in 1 2; do
  for f in 1 0; do
    if [ $f = 1 ]; then export HETU_STEM_SCALAR=1; else unset HETU_STEM_SCALAR; fi
    timeout -k 10 300 python -u bench.py > $O/stem_rn_$f$i.json 2>/dev/null || exit $?
    echo "scalar=$f $i $(python3 -c "import json;d=json.loads(open('$O/stem_rn_$f$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
