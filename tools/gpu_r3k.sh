#!/bin/bash
# round 3: counting sort with 10-bit hi buckets -- parity, all GPU tests, A/B,
# kernel trace of the bench; parabolic A/B; eye kernel trace (1M rays)
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k counting_sort > gpurun_out/r3k_bs.log 2>&1 || { tail -40 gpurun_out/r3k_bs.log; exit 1; }
tail -1 gpurun_out/r3k_bs.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3k_gpu.log 2>&1 || { tail -40 gpurun_out/r3k_gpu.log; exit 1; }
tail -1 gpurun_out/r3k_gpu.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3k_ab.log 2>&1 || { tail -20 gpurun_out/r3k_ab.log; exit 1; }
tail -1 gpurun_out/r3k_ab.log
for b in 1 0 1 0; do LPC_BSORT=$b timeout -k 10 120 python tools/cfg_trace.py parabolic 1000000 4 20 >> gpurun_out/r3k_para.log 2>&1 || exit 1; done
cat gpurun_out/r3k_para.log
mkdir -p gpurun_out/prof_r3k; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3k/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3k/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3k/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3k/kt | tail -4
python tools/kt_timeline.py gpurun_out/prof_r3k/kt 40 > gpurun_out/prof_r3k/timeline.txt
mkdir -p gpurun_out/prof_r3k_eye; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3k_eye/kt -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 1000000 16 1 > $R/gpurun_out/prof_r3k_eye/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3k_eye/kt.log; exit 1; }
tail -1 gpurun_out/prof_r3k_eye/kt.log
