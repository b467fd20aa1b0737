#!/bin/bash
# round 3: written-slot masks (the shading reads only the slots the walk wrote) --
# every -m gpu test, smoke, the default bench line, A/B against LPC_TMASK=0,
# a kernel trace of 5 bench steps.
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r3ab_gpu.log 2>&1 || { tail -40 gpurun_out/r3ab_gpu.log; exit 1; }
tail -1 gpurun_out/r3ab_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ab_smoke.log 2>&1 || { tail -30 gpurun_out/r3ab_smoke.log; exit 1; }
tail -1 gpurun_out/r3ab_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3ab_bench.json 2> gpurun_out/r3ab_bench.err || { tail -20 gpurun_out/r3ab_bench.err; exit 1; }
cut -c1-200 gpurun_out/r3ab_bench.json
timeout -k 10 600 python tools/ab.py 3 'base:' 'notm:LPC_TMASK=0' > gpurun_out/r3ab_ab.log 2>&1 || { tail -20 gpurun_out/r3ab_ab.log; exit 1; }
tail -1 gpurun_out/r3ab_ab.log
mkdir -p gpurun_out/prof_r3ab; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3ab/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3ab/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3ab/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3ab/kt | tail -4
python tools/kt_timeline.py gpurun_out/prof_r3ab/kt 40 > gpurun_out/prof_r3ab/timeline.txt
