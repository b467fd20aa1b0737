#!/bin/bash
# quick GPU diagnostic: traversal statistics only
mkdir -p gpurun_out
timeout -k 10 300 python tools/trace_stats.py ${STATS_SCENE:-synthetic} ${STATS_RAYS:-1000000} > gpurun_out/stats.log 2>&1
