#!/bin/bash
# round 3: counting sort v3 (rows move with keys; host bucket estimate) --
# parity, all GPU tests, A/B vs rocPRIM, kernel trace; traversal stats
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k counting_sort > gpurun_out/r3l_bs.log 2>&1 || { tail -40 gpurun_out/r3l_bs.log; exit 1; }
tail -1 gpurun_out/r3l_bs.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3l_gpu.log 2>&1 || { tail -40 gpurun_out/r3l_gpu.log; exit 1; }
tail -1 gpurun_out/r3l_gpu.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3l_ab.log 2>&1 || { tail -20 gpurun_out/r3l_ab.log; exit 1; }
tail -1 gpurun_out/r3l_ab.log
mkdir -p gpurun_out/prof_r3l; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3l/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3l/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3l/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3l/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3l/kt 40 > gpurun_out/prof_r3l/timeline.txt
timeout -k 10 300 python tools/trace_stats.py synthetic 1000000 > gpurun_out/r3l_stats.log 2>&1 || { tail -20 gpurun_out/r3l_stats.log; exit 1; }
cat gpurun_out/r3l_stats.log
for b in 1 0; do LPC_BSORT=$b timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 >> gpurun_out/r3l_eye.log 2>&1 || exit 1; done
grep scene gpurun_out/r3l_eye.log
