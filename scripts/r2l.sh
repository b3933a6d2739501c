export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S rn_fwd 300 env HETU_GRAD_ORDER=forward python bench.py --steps 20 --warmup 5 &&
$S rn_rev 300 env HETU_GRAD_ORDER=reverse python bench.py --steps 20 --warmup 5 &&
$S rn_fwd2 300 env HETU_GRAD_ORDER=forward python bench.py --steps 20 --warmup 5 &&
$S wdl 300 python bench.py --model wdl --steps 60 --warmup 10 &&
$S bert 300 python bench.py --model bert --steps 20 --warmup 5
