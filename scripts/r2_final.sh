#!/bin/bash
# Round-2 final-session GPU call: GPU tests, ResNet-50 / BERT benches, a two-rank
# data-parallel rehearsal on the one GPU (gloo carries the gradients, both ranks
# share cuda:0), and a steady-state rocprofv3 kernel trace of ResNet-50.
# Stops at the first crash or timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 540 python -u -m pytest tests -m gpu -x -v --capture=sys --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -20; tail -2 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for m in ${BENCHES-resnet50 bert}; do
  echo "== bench $m"
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err
  rc=$?
  cat gpurun_out/bench_$m.json; tail -2 gpurun_out/bench_$m.err
  [ $rc -ne 0 ] && { echo "bench $m rc=$rc"; exit $rc; }
done
if [ "${REHEARSE:-1}" = "1" ]; then
  echo "== 2-rank DP rehearsal (gloo, shared GPU)"
  HETU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --batch 32 \
    > gpurun_out/rehearse_dp2.json 2> gpurun_out/rehearse_dp2.err
  rc=$?
  cat gpurun_out/rehearse_dp2.json; tail -3 gpurun_out/rehearse_dp2.err
  [ $rc -ne 0 ] && { echo "rehearsal rc=$rc"; exit $rc; }
fi
if [ -n "${PROFILE_MODEL:-}" ]; then
  echo "== rocprofv3 $PROFILE_MODEL"
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$PROFILE_MODEL -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model $PROFILE_MODEL --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$PROFILE_MODEL.log 2>&1
  rc=$?
  cd $GRAFT_REPO_ROOT; tail -2 gpurun_out/prof_$PROFILE_MODEL.log
  exit $rc
fi
