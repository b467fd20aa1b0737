#!/bin/bash
# round 3: chained-population key experiment (LPC_RESORT_KEY=1: [mesh left | direction])
# -- per-iteration traversal statistics, then an A/B of the bench step.
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 200 python tools/trace_stats.py synthetic 1000000 > gpurun_out/r3z_stats_base.log 2>&1 || { tail -20 gpurun_out/r3z_stats_base.log; exit 1; }
LPC_RESORT_MIN=50000 timeout -k 10 200 python tools/trace_stats.py synthetic 1000000 > gpurun_out/r3z_stats_r50.log 2>&1 || { tail -20 gpurun_out/r3z_stats_r50.log; exit 1; }
LPC_RESORT_MIN=50000 LPC_RESORT_KEY=1 timeout -k 10 200 python tools/trace_stats.py synthetic 1000000 > gpurun_out/r3z_stats_r50k.log 2>&1 || { tail -20 gpurun_out/r3z_stats_r50k.log; exit 1; }
grep -h "it[0-9]" gpurun_out/r3z_stats_*.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'r50:LPC_RESORT_MIN=50000' 'r50k:LPC_RESORT_MIN=50000,LPC_RESORT_KEY=1' > gpurun_out/r3z_ab.log 2>&1 || { tail -20 gpurun_out/r3z_ab.log; exit 1; }
tail -1 gpurun_out/r3z_ab.log
