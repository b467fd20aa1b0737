#!/bin/bash
# GPU box: A/B of launch-policy defaults on the synthetic, lens and eye scenes
# (tools/sweep.py; every configuration must give the identical trace).
mkdir -p gpurun_out
O=BUDGET=16,BUDGET_LARGE=16,TARGET_BLOCKS=16384,WAVE_TARGET=65536
set -- "KEY=5,CHAIN=0" "BUDGET_LARGE=96" "BUDGET_LARGE=200" "BUDGET_LARGE=1000" "BUDGET_LARGE=0" "BUDGET_LARGE=200,LARGE_N=1000000" "BUDGET_LARGE=200,LARGE_N=4000000" "BUDGET_LARGE=0,LARGE_N=1000000"
timeout -k 10 200 python tools/sweep.py synthetic 1000000 9 "$@" > gpurun_out/sweep7_syn.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 2000000 5 "$@" > gpurun_out/sweep7_lens.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep7_eye.log 2>&1
rc=$?; cat gpurun_out/sweep7_*.log | cut -c1-110; exit $rc
