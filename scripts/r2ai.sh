export TMPDIR=/tmp
for i in 1 2 3; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 30 --warmup 5 > ../gpurun_out/ab_old_$i.log 2>&1) || exit 1
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --model bert --steps 30 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/rn_new_$i.log 2>&1 || exit 1
done
grep -h value gpurun_out/ab_old_*.log gpurun_out/ab_new_*.log gpurun_out/rn_new_*.log | cut -c1-110
