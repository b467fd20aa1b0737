#!/bin/bash
# round 3: traversal statistics per iteration
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python tools/trace_stats.py synthetic 1000000 > gpurun_out/r3h_stats.log 2>&1 || { tail -20 gpurun_out/r3h_stats.log; exit 1; }
cat gpurun_out/r3h_stats.log
