export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S prof_wdl 300 python -u scripts/prof_wdl.py
