#!/bin/bash
# Targeted tests, kernel census, then the model benches (ResNet-50, BERT, MoE, WDL).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { name=$1; lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log; return $rc; }
step tests 400 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py} -q -x --timeout 120 --timeout-method thread &&
TAILN=12 step tk_resnet 200 python scripts/find_torch_kernels.py --model resnet50 --batch 32 &&
TAILN=24 step tk_bert 200 python scripts/find_torch_kernels.py --model bert --batch 16 &&
TAILN=1 step b_resnet 200 python bench.py --steps 20 --warmup 5 &&
TAILN=1 step b_bert 200 python bench.py --model bert --steps 20 --warmup 5 &&
TAILN=1 step b_moe 200 python bench.py --model moe --steps 20 --warmup 5 &&
TAILN=1 step b_wdl 300 python bench.py --model wdl --steps 60 --warmup 10
