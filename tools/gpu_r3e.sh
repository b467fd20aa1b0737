#!/bin/bash
# round 3: gated root tests + batched walk -- parity, host-side roots lines, A/B
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "policies or trace" > gpurun_out/r3e_tests.log 2>&1 || { tail -30 gpurun_out/r3e_tests.log; exit 1; }
tail -2 gpurun_out/r3e_tests.log
LPC_WALK_NB=4 LPC_HALF=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "trace" > gpurun_out/r3e_tests_nb.log 2>&1 || { tail -30 gpurun_out/r3e_tests_nb.log; exit 1; }
tail -2 gpurun_out/r3e_tests_nb.log
LPC_HOSTPROF=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu --no-configs > gpurun_out/r3e_hp.log 2>&1 || { tail -20 gpurun_out/r3e_hp.log; exit 1; }
grep "roots:" gpurun_out/r3e_hp.log | head -8
timeout -k 10 900 python tools/ab.py 3 'base:' 'nogate:LPC_ROOTS_GATE=0' 'nb4:LPC_WALK_NB=4' > gpurun_out/r3e_ab.log 2>&1 || { tail -20 gpurun_out/r3e_ab.log; exit 1; }
tail -1 gpurun_out/r3e_ab.log
