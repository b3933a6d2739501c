export PYTHONPATH=$PWD TMPDIR=/tmp
S=scripts/gpu_step.sh
$S bert_graph 300 env HETU_HIPGRAPH=1 python bench.py --model bert --steps 20 --warmup 5 ;
$S moe_graph 300 env HETU_HIPGRAPH=1 python bench.py --model moe --steps 20 --warmup 5 ;
$S rn_graph 300 env HETU_HIPGRAPH=1 python bench.py --steps 20 --warmup 5
