#!/bin/bash
# round 3: counting sort v7 -- parity, all GPU tests, A/B, kernel trace; then
# the re-sort experiments (tools/gpu_r3n.sh)
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "counting_sort" > gpurun_out/r3o_bs.log 2>&1 || { tail -40 gpurun_out/r3o_bs.log; exit 1; }
tail -1 gpurun_out/r3o_bs.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3o_gpu.log 2>&1 || { tail -40 gpurun_out/r3o_gpu.log; exit 1; }
tail -1 gpurun_out/r3o_gpu.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3o_ab.log 2>&1 || { tail -20 gpurun_out/r3o_ab.log; exit 1; }
tail -1 gpurun_out/r3o_ab.log
mkdir -p gpurun_out/prof_r3o; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3o/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3o/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3o/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3o/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3o/kt 40 > gpurun_out/prof_r3o/timeline.txt
grep -E "k_b|gather|roots_s" gpurun_out/prof_r3o/timeline.txt | head -8
bash tools/gpu_r3n.sh
