#!/bin/bash
# round 3: counting sort moves the rays itself (no permutation, no k_gather_aos) --
# its parity test first, smoke, every -m gpu test, the default bench line, a
# kernel trace of 5 bench steps.
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "counting_sort or resort" > gpurun_out/r3aa_bs.log 2>&1 || { tail -40 gpurun_out/r3aa_bs.log; exit 1; }
tail -1 gpurun_out/r3aa_bs.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3aa_smoke.log 2>&1 || { tail -30 gpurun_out/r3aa_smoke.log; exit 1; }
tail -1 gpurun_out/r3aa_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3aa_bench.json 2> gpurun_out/r3aa_bench.err || { tail -20 gpurun_out/r3aa_bench.err; exit 1; }
cut -c1-200 gpurun_out/r3aa_bench.json
mkdir -p gpurun_out/prof_r3aa; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3aa/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3aa/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3aa/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3aa/kt | tail -4
python tools/kt_timeline.py gpurun_out/prof_r3aa/kt 40 > gpurun_out/prof_r3aa/timeline.txt
timeout -k 10 900 $T tests -m gpu > gpurun_out/r3aa_gpu.log 2>&1 || { tail -40 gpurun_out/r3aa_gpu.log; exit 1; }
tail -1 gpurun_out/r3aa_gpu.log
