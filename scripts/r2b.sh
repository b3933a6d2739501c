export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S layers_unfused 240 env HETU_FUSE=0 python -u scripts/diag_layers.py 2 &&
$S layers_fused 240 python -u scripts/diag_layers.py 2 fused &&
$S layers_unfused_vendor 240 env HETU_FUSE=0 HETU_CONV=vendor python -u scripts/diag_layers.py 2
