#!/bin/bash
# round 3: hybrid drain (dense entries triangle-uniform) -- parity, all GPU
# tests, A/B of the threshold, kernel trace; traversal stats
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "bitexact or policies" > gpurun_out/r3q_p.log 2>&1 || { tail -40 gpurun_out/r3q_p.log; exit 1; }
tail -1 gpurun_out/r3q_p.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3q_gpu.log 2>&1 || { tail -40 gpurun_out/r3q_gpu.log; exit 1; }
tail -1 gpurun_out/r3q_gpu.log
timeout -k 10 900 python tools/ab.py 3 'base:' 'packed:LPC_DRAIN_U=65' 'u4:LPC_DRAIN_U=4' 'u16:LPC_DRAIN_U=16' > gpurun_out/r3q_ab.log 2>&1 || { tail -20 gpurun_out/r3q_ab.log; exit 1; }
tail -1 gpurun_out/r3q_ab.log
mkdir -p gpurun_out/prof_r3q; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3q/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3q/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3q/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3q/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3q/kt 40 > gpurun_out/prof_r3q/timeline.txt
for u in 8 65; do LPC_DRAIN_U=$u timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/u=$u /" >> gpurun_out/r3q_eye.log 2>&1 || exit 1; done
grep scene gpurun_out/r3q_eye.log
