#!/bin/bash
# GPU box: hand-over switch at a rays-per-triangle ratio across scenes
mkdir -p gpurun_out
set -- "KEY=5,CHAIN=0" "KEY=5" "LARGE_N=0,LARGE_PER_TRI=12" "LARGE_N=0,LARGE_PER_TRI=16" "LARGE_N=0,LARGE_PER_TRI=20"
timeout -k 10 200 python tools/sweep.py parabolic 1000000 5 "$@" > gpurun_out/sweep16_par.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py synthetic 1000000 11 "$@" > gpurun_out/sweep16_syn.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 1000000 5 "$@" > gpurun_out/sweep16_lens.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep16_eye.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py synthetic 12500000 3 "$@" > gpurun_out/sweep16_syn12m.log 2>&1
rc=$?; cat gpurun_out/sweep16_*.log | grep -v amdgpu | cut -c1-100; exit $rc
