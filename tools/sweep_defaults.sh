#!/bin/bash
# GPU box: A/B of launch-policy defaults on the synthetic, lens and eye scenes
# (tools/sweep.py; every configuration must give the identical trace).
mkdir -p gpurun_out
O=BUDGET=16,BUDGET_LARGE=16,TARGET_BLOCKS=16384,WAVE_TARGET=65536
set -- "KEY=5,CHAIN=0" "KEY=5" "TARGET_BLOCKS=65536" "TARGET_BLOCKS=16384" "WAVE_TARGET=262144" "WAVE_TARGET=65536" "SLIVER_WAVES=32768" "KEY=0" "KEY=3" "CHAIN=1" "ISECT_MINB=1"
timeout -k 10 200 python tools/sweep.py synthetic 1000000 9 "$@" > gpurun_out/sweep8_syn.log 2>&1 &&
timeout -k 10 200 python tools/sweep.py lens 2000000 5 "$@" > gpurun_out/sweep8_lens.log 2>&1 &&
timeout -k 10 300 python tools/sweep.py eye 500000 2 "$@" > gpurun_out/sweep8_eye.log 2>&1
rc=$?; cat gpurun_out/sweep8_*.log | cut -c1-110; exit $rc
