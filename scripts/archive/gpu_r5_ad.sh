#!/bin/bash
# Round-5: non-temporal input loads in the BatchNorm apply passes: BN tests with the switch on,
# ResNet-50 interleaved A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python3 -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread"
HETU_BN_NT=1 timeout -k 10 600 $T tests/test_bn_fusion_gpu.py tests/test_kernels_gpu.py -k "bn or batchnorm or norm" > gpurun_out/r5ad_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5ad_tests.log; [ $rc -eq 0 ] || exit $rc
for a in 0 1 0 1; do
  HETU_BN_NT=$a timeout -k 10 400 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5ad_nt$a.json 2> gpurun_out/r5ad.err
  rc=$?; echo "nt=$a $(tail -1 gpurun_out/r5ad_nt$a.json | cut -c1-120)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5ad.err; exit $rc; }
done
