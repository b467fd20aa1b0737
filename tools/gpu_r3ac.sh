#!/bin/bash
# round 3: k_stage_move's counters in registers (no scratch) -- every -m gpu
# test, then the final evidence (tools/gpu_final.sh).
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r3ac_gpu.log 2>&1 || { tail -40 gpurun_out/r3ac_gpu.log; exit 1; }
tail -1 gpurun_out/r3ac_gpu.log
bash tools/gpu_final.sh
