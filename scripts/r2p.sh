export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S rn_on1 300 python bench.py --steps 30 --warmup 5 &&
$S rn_off1 300 env HETU_FUSE_BN_STATS=0 python bench.py --steps 30 --warmup 5 &&
$S rn_on2 300 python bench.py --steps 30 --warmup 5 &&
$S rn_off2 300 env HETU_FUSE_BN_STATS=0 python bench.py --steps 30 --warmup 5
