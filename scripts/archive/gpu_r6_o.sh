#!/bin/bash
# A/B of a kernel library built with other flags (ALT, default alt_lib/libhetu_kernels.so):
# its BN-fusion / conv tests, then ResNet-50 interleaved against the in-tree library
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
ALT=${ALT:-$R/alt_lib/libhetu_kernels.so}
HETU_KERNELS_LIB=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_bn_fusion_gpu.py tests/test_gemm_gpu.py > $O/r6o_tests.txt 2>&1
rc=$?; tail -2 $O/r6o_tests.txt; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export HETU_KERNELS_LIB=$ALT; else unset HETU_KERNELS_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r6o_$v$i.json 2> $O/r6o_$v$i.err || exit $?
    echo "$v $i $(python3 -c "import json;d=json.loads(open('$O/r6o_$v$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
