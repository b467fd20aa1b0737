#!/bin/bash
# GPU box: hand-over switch point (population vs triangles) across scenes
mkdir -p gpurun_out
set -- "KEY=5,CHAIN=0" "KEY=5" "LARGE_N=1500000" "LARGE_PER_TRI=32" "LARGE_PER_TRI=128"
timeout -k 10 200 python tools/sweep.py synthetic 4000000 5 "$@" > gpurun_out/sweep12_syn4m.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 2000000 5 "$@" > gpurun_out/sweep12_lens.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep12_eye.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py synthetic 1000000 9 "$@" > gpurun_out/sweep12_syn.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py synthetic 12500000 3 "$@" > gpurun_out/sweep12_syn12m.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py parabolic 1000000 5 "$@" > gpurun_out/sweep12_par.log 2>&1
rc=$?; cat gpurun_out/sweep12_*.log | cut -c1-110; exit $rc
