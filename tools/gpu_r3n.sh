#!/bin/bash
# round 3: re-sorting large chained populations (LPC_RESORT_MIN) on the eye,
# lens and the synthetic secondaries; one process per configuration
R=$(pwd); mkdir -p $R/gpurun_out
for r in x 500000 4000000 x 500000 4000000; do
  if [ $r = x ]; then E=""; else E="LPC_RESORT_MIN=$r"; fi
  env $E timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/resort=$r /" >> gpurun_out/r3n_eye.log 2>&1 || exit 1
done
grep scene gpurun_out/r3n_eye.log
for r in x 2000000 x 2000000; do
  if [ $r = x ]; then E=""; else E="LPC_RESORT_MIN=$r"; fi
  env $E timeout -k 10 120 python tools/cfg_trace.py lens 10000000 8 3 | sed "s/^/resort=$r /" >> gpurun_out/r3n_lens.log 2>&1 || exit 1
done
grep scene gpurun_out/r3n_lens.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'resort50k:LPC_RESORT_MIN=50000' > gpurun_out/r3n_ab.log 2>&1 || { tail -20 gpurun_out/r3n_ab.log; exit 1; }
tail -1 gpurun_out/r3n_ab.log
