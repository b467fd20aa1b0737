#!/bin/bash
# round 3: speculative device-sized iterations -- parity, A/B, kernel trace
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spec.py > gpurun_out/r3f_spec.log 2>&1 || { tail -40 gpurun_out/r3f_spec.log; exit 1; }
tail -2 gpurun_out/r3f_spec.log
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_golden.py > gpurun_out/r3f_par.log 2>&1 || { tail -40 gpurun_out/r3f_par.log; exit 1; }
tail -2 gpurun_out/r3f_par.log
LPC_HOSTPROF=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu --no-configs > gpurun_out/r3f_hp.log 2>&1 || { tail -20 gpurun_out/r3f_hp.log; exit 1; }
grep "lpc host\] n" gpurun_out/r3f_hp.log | tail -8
timeout -k 10 900 python tools/ab.py 3 'base:' 'nospec:LPC_SPEC=0' > gpurun_out/r3f_ab.log 2>&1 || { tail -20 gpurun_out/r3f_ab.log; exit 1; }
tail -1 gpurun_out/r3f_ab.log
mkdir -p gpurun_out/prof_r3f; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3f/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3f/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3f/kt.log; exit 1; }
python tools/kt_timeline.py gpurun_out/prof_r3f/kt 45 > gpurun_out/prof_r3f/timeline.txt 2>&1; tail -45 gpurun_out/prof_r3f/timeline.txt
