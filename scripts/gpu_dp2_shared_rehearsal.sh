#!/bin/bash
# 2-rank data-parallel ResNet-50 rehearsal on ONE MI355X (both ranks share the device, gloo
# carries the bucketed gradient all-reduce through host memory -- RCCL refuses two ranks on
# one GPU): the multi-rank bench path end to end (bucket launch during backward, max-over-
# ranks timing, one JSON line).  Not a scaling number.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp HETU_DIST_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus 2 --steps ${STEPS:-5} --warmup ${WARMUP:-3} --batch ${BATCH:-64} \
  > gpurun_out/dp2_shared.json 2> gpurun_out/dp2_shared.err
rc=$?; tail -3 gpurun_out/dp2_shared.err; tail -1 gpurun_out/dp2_shared.json | cut -c1-400; exit $rc
