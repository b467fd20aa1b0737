#!/bin/bash
# round 3: A/B of speculation, emitted-key bits, sorted secondaries; kernel trace of the last
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 1000 python tools/ab.py 4 'base:' 'nospec:LPC_SPEC=0' 'kb8:LPC_KEY_BITS=8' 'csort:LPC_CHAIN_SORT=1' > gpurun_out/r3g_ab.log 2>&1 || { tail -20 gpurun_out/r3g_ab.log; exit 1; }
tail -1 gpurun_out/r3g_ab.log
mkdir -p gpurun_out/prof_r3g; (cd /tmp && export TMPDIR=/tmp && LPC_CHAIN_SORT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3g/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3g/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3g/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3g/kt
python tools/kt_timeline.py gpurun_out/prof_r3g/kt 40
