export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S wdl1 300 python bench.py --model wdl --steps 60 --warmup 10 &&
$S wdl2 300 python bench.py --model wdl --steps 200 --warmup 64 &&
$S wdl_noprefetch 300 python bench.py --model wdl --steps 60 --warmup 10 --no-prefetch
