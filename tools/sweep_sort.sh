#!/bin/bash
# GPU box: hand-over budget below the rays-per-triangle switch
mkdir -p gpurun_out
set -- "KEY=5,CHAIN=0" "KEY=5" "BUDGET=20" "BUDGET=28" "BUDGET=32"
timeout -k 10 200 python tools/sweep.py synthetic 1000000 11 "$@" > gpurun_out/sweep17_syn.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep17_eye.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py synthetic 4000000 5 "$@" > gpurun_out/sweep17_syn4m.log 2>&1
rc=$?; cat gpurun_out/sweep17_*.log | grep -v amdgpu | cut -c1-100; exit $rc
