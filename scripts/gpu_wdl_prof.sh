#!/bin/bash
# Wide&Deep (PS + HET cache) step: bench line, then a cProfile of the host side
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python bench.py --model wdl --steps 60 --warmup 10 > gpurun_out/wdl.json 2> gpurun_out/wdl.err || { tail -20 gpurun_out/wdl.err; exit 1; }
cat gpurun_out/wdl.json
timeout -k 10 300 python -m cProfile -o gpurun_out/wdl.prof bench.py --model wdl --steps 300 --warmup 10 > gpurun_out/wdl_prof.json 2>/dev/null || exit $?
cat gpurun_out/wdl_prof.json
python - <<'PY' > gpurun_out/wdl_pstats.txt
import pstats
p = pstats.Stats('gpurun_out/wdl.prof'); p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumtime').print_stats(45)
PY
head -80 gpurun_out/wdl_pstats.txt | tail -55
