export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S ablate 300 python -u scripts/bench_big_ablate.py
