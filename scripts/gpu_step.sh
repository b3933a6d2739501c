#!/bin/bash
# run one GPU step under its own time limit; stop the whole call on a crash /
# timeout (rc >= 124 or a signal), continue on an ordinary failure (rc 1/2).
# usage: gpu_step.sh NAME SECONDS cmd...   (output -> gpurun_out/NAME.log)
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name"
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
tail -15 "gpurun_out/$name.log"
echo "== $name rc=$rc"
if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name"; exit $rc; fi
exit 0
