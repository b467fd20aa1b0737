#!/bin/bash
# GPU box: hand-over budget below 1.5 M rays
mkdir -p gpurun_out
set -- "KEY=5,CHAIN=0" "KEY=5" "BUDGET=24" "BUDGET=28" "BUDGET=22"
timeout -k 10 200 python tools/sweep.py synthetic 1000000 15 "$@" > gpurun_out/sweep14_syn.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py parabolic 1000000 7 "$@" > gpurun_out/sweep14_par.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 1000000 5 "$@" > gpurun_out/sweep14_lens.log 2>&1
rc=$?; cat gpurun_out/sweep14_*.log | cut -c1-110; exit $rc
