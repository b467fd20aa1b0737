#!/bin/bash
# round 3: hybrid drain with the next dense record prefetched -- parity of the
# drain paths, A/B of the threshold on the synthetic bench and the eye
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "bitexact or policies or trace_results" > gpurun_out/r3r_p.log 2>&1 || { tail -40 gpurun_out/r3r_p.log; exit 1; }
tail -1 gpurun_out/r3r_p.log
timeout -k 10 900 python tools/ab.py 3 'u16:LPC_DRAIN_U=16' 'packed:LPC_DRAIN_U=65' 'u24:LPC_DRAIN_U=24' 'u40:LPC_DRAIN_U=40' > gpurun_out/r3r_ab.log 2>&1 || { tail -20 gpurun_out/r3r_ab.log; exit 1; }
tail -1 gpurun_out/r3r_ab.log
for u in 8 16 24 40 65; do LPC_DRAIN_U=$u timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/u=$u /" >> gpurun_out/r3r_eye.log 2>&1 || exit 1; done
grep scene gpurun_out/r3r_eye.log | cut -c1-60,200-
for u in 16 65; do LPC_DRAIN_U=$u timeout -k 10 120 python tools/cfg_trace.py lens 10000000 8 3 | sed "s/^/u=$u /" >> gpurun_out/r3r_lens.log 2>&1 || exit 1; LPC_DRAIN_U=$u timeout -k 10 120 python tools/cfg_trace.py parabolic 1000000 4 20 | sed "s/^/u=$u /" >> gpurun_out/r3r_lens.log 2>&1 || exit 1; done
grep scene gpurun_out/r3r_lens.log | cut -c1-60,200-
