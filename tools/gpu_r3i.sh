#!/bin/bash
# round 3: bucket + chunk sort of the emitted rays -- parity, A/B, kernel trace
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_golden.py tests/test_ref_parity.py > gpurun_out/r3i_par.log 2>&1 || { tail -40 gpurun_out/r3i_par.log; exit 1; }
tail -2 gpurun_out/r3i_par.log
timeout -k 10 900 python tools/ab.py 4 'base:' 'nobsort:LPC_BSORT=0' > gpurun_out/r3i_ab.log 2>&1 || { tail -20 gpurun_out/r3i_ab.log; exit 1; }
tail -1 gpurun_out/r3i_ab.log
mkdir -p gpurun_out/prof_r3i; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3i/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3i/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3i/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3i/kt
python tools/kt_timeline.py gpurun_out/prof_r3i/kt 40 > gpurun_out/prof_r3i/timeline.txt
head -24 gpurun_out/prof_r3i/timeline.txt
