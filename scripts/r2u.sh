export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && $GRAFT_REPO_ROOT/scripts/gpu_step.sh prof_bert 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2u -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 5 --warmup 3 &&
cd $GRAFT_REPO_ROOT && python scripts/prof_steps.py gpurun_out/prof_r2u/run_kernel_trace.csv --last 3 > gpurun_out/bert_steady_r2u.txt 2>&1
