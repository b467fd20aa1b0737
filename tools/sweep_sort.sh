#!/bin/bash
# GPU box: hand-over budget/levels for large populations across scenes
mkdir -p gpurun_out
set -- "KEY=5,CHAIN=0" "KEY=5" "BUDGET_LARGE=40,SPILL_LEVELS=1" "BUDGET_LARGE=40,SPILL_LEVELS=2" "BUDGET_LARGE=20,SPILL_LEVELS=2" "BUDGET_LARGE=64,SPILL_LEVELS=2" "BUDGET_LARGE=20"
timeout -k 10 200 python tools/sweep.py synthetic 4000000 5 "$@" > gpurun_out/sweep11_syn4m.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 2000000 5 "$@" > gpurun_out/sweep11_lens.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep11_eye.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py synthetic 1000000 9 "$@" > gpurun_out/sweep11_syn.log 2>&1
rc=$?; cat gpurun_out/sweep11_*.log | cut -c1-110; exit $rc
