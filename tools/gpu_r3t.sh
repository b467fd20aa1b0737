#!/bin/bash
# round 3: packed root tests -- all GPU tests, bench, kernel trace
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3t_gpu.log 2>&1 || { tail -40 gpurun_out/r3t_gpu.log; exit 1; }
tail -1 gpurun_out/r3t_gpu.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'nogate:LPC_ROOTS_GATE=0' 'b32:LPC_BUDGET=32' 'b16:LPC_BUDGET=16' > gpurun_out/r3t_ab.log 2>&1 || { tail -20 gpurun_out/r3t_ab.log; exit 1; }
tail -1 gpurun_out/r3t_ab.log
mkdir -p gpurun_out/prof_r3t; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3t/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3t/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3t/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3t/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3t/kt 40 > gpurun_out/prof_r3t/timeline.txt
grep -E "roots_s|k_b|gather" gpurun_out/prof_r3t/timeline.txt | head -8
