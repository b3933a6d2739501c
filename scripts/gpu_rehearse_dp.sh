#!/bin/bash
# Multi-rank data-parallel rehearsal on the one-GPU box:
#   1. the RCCL communicator + forced single-rank DP tests (tests/test_rccl_gpu.py)
#   2. N ranks sharing the GPU over gloo (HETU_DIST_BACKEND=gloo), autotune off, with
#      per-rank progress lines and a stack dump of every rank silent for 60 s.
#   gpurun -- bash scripts/gpu_rehearse_dp.sh
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
[ "${SKIP_RCCL:-0}" = "1" ] || timeout -k 10 240 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/rccl_tests.log 2>&1
rc=$?; tail -8 gpurun_out/rccl_tests.log
[ $rc -eq 0 ] || exit $rc
N=${NRANK:-4}
HETU_DIST_BACKEND=gloo HETU_DETERMINISTIC=1 HETU_STALL_DUMP_S=60 timeout -k 10 ${REH_TIMEOUT:-170} \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus $N --batch ${REH_BATCH:-16} --steps 3 --warmup 2 > gpurun_out/rehearse_dp$N.json 2> gpurun_out/rehearse_dp$N.err
rc=$?
cat gpurun_out/rehearse_dp$N.json; grep "bench rank" gpurun_out/rehearse_dp$N.err | tail -12
echo "rehearsal rc=$rc"
exit $rc
