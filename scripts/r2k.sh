export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S bench_resnet50 300 python bench.py --steps 20 --warmup 5 &&
$S bench_bert 300 python bench.py --model bert --steps 20 --warmup 5 &&
$S conv_shapes 400 python -u scripts/bench_conv_resnet.py 256 gpurun_out/conv_shapes_r2k.txt
