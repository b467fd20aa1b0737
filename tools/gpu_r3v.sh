#!/bin/bash
# round 3: k_stage_move batched tile sums -- parity subset; then a re-sweep of the
# hand-over knobs after the drain change
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_spec.py -k "fused or traced_order or counting or spec or aggregate" > gpurun_out/r3v_p.log 2>&1 || { tail -40 gpurun_out/r3v_p.log; exit 1; }
tail -1 gpurun_out/r3v_p.log
timeout -k 10 900 python tools/ab.py 3 'base:' 'ps6:LPC_PAIR_SHIFT=6' 'ps4:LPC_PAIR_SHIFT=4' 'lv3:LPC_SPILL_LEVELS=3' 'b28:LPC_BUDGET=28' > gpurun_out/r3v_ab.log 2>&1 || { tail -20 gpurun_out/r3v_ab.log; exit 1; }
tail -1 gpurun_out/r3v_ab.log
mkdir -p gpurun_out/prof_r3v; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3v/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3v/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3v/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3v/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3v/kt 40 > gpurun_out/prof_r3v/timeline.txt
grep -E "stage_move" gpurun_out/prof_r3v/timeline.txt | head -4
