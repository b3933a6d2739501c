#!/bin/bash
# Round-4: steady-state ResNet-50 kernel traces with and without the BN-backward epilogue
# fusion, per (kernel, grid) (scripts/prof_shapes.py), for a kernel-by-kernel comparison.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-1 0}; do
  cd /tmp && HETU_FUSE_BN_BWD=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_ab$v -o run --output-format csv \
    -- python3 $R/bench.py --model ${MODEL:-resnet50} --steps 5 --warmup 3 > $R/gpurun_out/prof_ab$v.log 2>&1
  rc=$?; cd $R; grep '"metric"' gpurun_out/prof_ab$v.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_ab$v -name "*kernel_trace.csv" | head -1)
  python scripts/prof_shapes.py "$f" --top 80 > gpurun_out/prof_ab${v}_shapes.txt 2>&1; head -3 gpurun_out/prof_ab${v}_shapes.txt
done
