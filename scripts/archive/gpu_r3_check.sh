#!/bin/bash
# Targeted GPU checks after a change: the named test files, then the non-hand-written
# kernel census of one ResNet-50 / BERT step.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { name=$1; lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log; return $rc; }
step tests 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py} -q -x --timeout 120 --timeout-method thread &&
TAILN=30 step tk_resnet 200 python scripts/find_torch_kernels.py --model resnet50 --batch 32 &&
TAILN=30 step tk_bert 200 python scripts/find_torch_kernels.py --model bert --batch 16
