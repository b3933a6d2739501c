#!/bin/bash
# Round-3 GPU batch: long-tail tensor-op tests, the non-hand-written kernels of one
# steady-state ResNet-50 / BERT step (scripts/find_torch_kernels.py), and the BERT bench
# with and without hipGraph replay.  Each step has its own time limit; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { name=$1; lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log; return $rc; }
step tops 120 python -u -m pytest tests/test_tensor_ops_gpu.py -q --timeout 60 --timeout-method thread &&
TAILN=40 step tk_resnet 200 python scripts/find_torch_kernels.py --model resnet50 --batch 32 &&
TAILN=40 step tk_bert 200 python scripts/find_torch_kernels.py --model bert --batch 16 &&
TAILN=2 step bert_eager 200 python bench.py --model bert --steps 20 --warmup 5 &&
HETU_HIPGRAPH=1 TAILN=2 step bert_graph 200 python bench.py --model bert --steps 20 --warmup 5
[ "${MORE:-1}" = "1" ] || exit 0
TAILN=2 step resnet_default 200 python bench.py --steps 20 --warmup 5 &&
HETU_ALLOCATOR=bfc TAILN=2 step resnet_bfc 200 python bench.py --steps 20 --warmup 5 &&
TAILN=2 step wdl 300 python bench.py --model wdl --steps 60 --warmup 10 &&
TAILN=2 step moe 200 python bench.py --model moe --steps 20 --warmup 5
