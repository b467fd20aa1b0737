#!/bin/bash
# round 3: counting sort v4 (LDS-ordered contiguous stores) + k_roots_s records
# in LDS -- parity, all GPU tests, A/B, kernel trace
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "counting_sort or policies" > gpurun_out/r3m_bs.log 2>&1 || { tail -40 gpurun_out/r3m_bs.log; exit 1; }
tail -1 gpurun_out/r3m_bs.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3m_gpu.log 2>&1 || { tail -40 gpurun_out/r3m_gpu.log; exit 1; }
tail -1 gpurun_out/r3m_gpu.log
cat gpurun_out/sharded.jsonl
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3m_ab.log 2>&1 || { tail -20 gpurun_out/r3m_ab.log; exit 1; }
tail -1 gpurun_out/r3m_ab.log
mkdir -p gpurun_out/prof_r3m; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3m/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3m/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3m/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3m/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3m/kt 40 > gpurun_out/prof_r3m/timeline.txt
head -32 gpurun_out/prof_r3m/timeline.txt | tail -26
