#!/bin/bash
# round 3: k_stage_move block-0 batch (LPC_MOVE_UB 8 / 4 / 2) A/B
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 900 python tools/ab.py 5 'ub8:' "ub4:LPC_LIB_PATH=$R/lightpycl_amd/liblpc_ub4.so" "ub2:LPC_LIB_PATH=$R/lightpycl_amd/liblpc_ub2.so" > gpurun_out/r3ae_ab.log 2>&1 || { tail -20 gpurun_out/r3ae_ab.log; exit 1; }
tail -1 gpurun_out/r3ae_ab.log
