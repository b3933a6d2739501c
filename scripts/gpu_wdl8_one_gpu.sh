#!/bin/bash
# BASELINE config 3 with 8 workers on the one GPU: 1 PS server + 8 worker processes (pure PS
# mode, no RCCL: gloo host group for the barriers), distinct id shards per worker.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HETU_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 8 --model wdl --steps ${STEPS:-100} --warmup ${WARMUP:-20} \
  > gpurun_out/wdl8.json 2> gpurun_out/wdl8.err
rc=$?; tail -3 gpurun_out/wdl8.err; tail -1 gpurun_out/wdl8.json; exit $rc
