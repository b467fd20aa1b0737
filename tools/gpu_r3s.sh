#!/bin/bash
# round 3: compile-time variants of the walk (pipelined packed drain, 5 waves/SIMD
# launch bounds) A/B on the synthetic bench and the eye; lens/parabolic at the
# new drain threshold
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for v in pipe pipe5; do
  LPC_LIB_PATH=lightpycl_amd/liblpc_$v.so timeout -k 10 300 $T tests/test_gpu_parity.py -k "bitexact and (two_levels or policies)" > gpurun_out/r3s_p_$v.log 2>&1 || { tail -30 gpurun_out/r3s_p_$v.log; exit 1; }
  tail -1 gpurun_out/r3s_p_$v.log
done
timeout -k 10 900 python tools/ab.py 3 'base:' 'pipe:LPC_LIB_PATH=lightpycl_amd/liblpc_pipe.so' 'minb5:LPC_LIB_PATH=lightpycl_amd/liblpc_minb5.so' 'pipe5:LPC_LIB_PATH=lightpycl_amd/liblpc_pipe5.so' > gpurun_out/r3s_ab.log 2>&1 || { tail -20 gpurun_out/r3s_ab.log; exit 1; }
tail -1 gpurun_out/r3s_ab.log
for v in base pipe minb5 pipe5; do
  if [ $v = base ]; then E=""; else E="LPC_LIB_PATH=lightpycl_amd/liblpc_$v.so"; fi
  env $E timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/$v /" >> gpurun_out/r3s_eye.log 2>&1 || exit 1
  env $E timeout -k 10 120 python tools/cfg_trace.py lens 10000000 8 3 | sed "s/^/$v /" >> gpurun_out/r3s_eye.log 2>&1 || exit 1
  env $E timeout -k 10 120 python tools/cfg_trace.py parabolic 1000000 4 20 | sed "s/^/$v /" >> gpurun_out/r3s_eye.log 2>&1 || exit 1
done
grep scene gpurun_out/r3s_eye.log | python -c "
import sys,json
for l in sys.stdin:
    tag,js=l.split(' ',1); d=json.loads(js); print(tag,d['scene'],round(d['ms_per_trace'],3),round(d['ray_bounces_per_s']/1e9,3))"
bash tools/pmc_probe.sh "k_shade_stage|k_roots_s|k_stage_move|k_slivers|k_bsort2|k_bscatter|k_rootwalk|k_spill" > gpurun_out/r3s_pmc.txt 2>&1 || { tail -20 gpurun_out/r3s_pmc.txt; exit 1; }
cut -c1-260 gpurun_out/r3s_pmc.txt | head -60
