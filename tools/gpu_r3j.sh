#!/bin/bash
# round 3 (re-entry): counting sort of the emitted rays -- its parity test first,
# then smoke, every -m gpu test, the default bench line, A/B against rocPRIM,
# a kernel trace of 5 bench steps.
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k counting_sort > gpurun_out/r3j_bs.log 2>&1 || { tail -40 gpurun_out/r3j_bs.log; exit 1; }
tail -1 gpurun_out/r3j_bs.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j_smoke.log 2>&1 || { tail -30 gpurun_out/r3j_smoke.log; exit 1; }
tail -1 gpurun_out/r3j_smoke.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3j_gpu.log 2>&1 || { tail -40 gpurun_out/r3j_gpu.log; exit 1; }
tail -1 gpurun_out/r3j_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || { tail -20 gpurun_out/r3j_bench.err; exit 1; }
cut -c1-300 gpurun_out/r3j_bench.json
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3j_ab.log 2>&1 || { tail -20 gpurun_out/r3j_ab.log; exit 1; }
tail -1 gpurun_out/r3j_ab.log
mkdir -p gpurun_out/prof_r3j; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3j/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3j/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3j/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3j/kt
python tools/kt_timeline.py gpurun_out/prof_r3j/kt 40 > gpurun_out/prof_r3j/timeline.txt
