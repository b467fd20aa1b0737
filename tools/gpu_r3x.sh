#!/bin/bash
# round 3: plane-side cull at the walk's leaves -- device superset test, parity,
# A/B (bench, eye, lens, parabolic), then all GPU tests
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_filter.py > gpurun_out/r3x_f.log 2>&1 || { tail -40 gpurun_out/r3x_f.log; exit 1; }
tail -1 gpurun_out/r3x_f.log
timeout -k 10 400 $T tests/test_gpu_parity.py -k "bitexact or trace_results or policies" > gpurun_out/r3x_p.log 2>&1 || { tail -40 gpurun_out/r3x_p.log; exit 1; }
tail -1 gpurun_out/r3x_p.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'noplane:LPC_PLANE=0' > gpurun_out/r3x_ab.log 2>&1 || { tail -20 gpurun_out/r3x_ab.log; exit 1; }
tail -1 gpurun_out/r3x_ab.log
for v in 1 0; do
  LPC_PLANE=$v timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/p=$v /" >> gpurun_out/r3x_cfg.log 2>&1 || exit 1
  LPC_PLANE=$v timeout -k 10 120 python tools/cfg_trace.py lens 10000000 8 3 | sed "s/^/p=$v /" >> gpurun_out/r3x_cfg.log 2>&1 || exit 1
  LPC_PLANE=$v timeout -k 10 120 python tools/cfg_trace.py parabolic 1000000 4 20 | sed "s/^/p=$v /" >> gpurun_out/r3x_cfg.log 2>&1 || exit 1
done
grep scene gpurun_out/r3x_cfg.log | python -c "
import sys,json
for l in sys.stdin:
    tag,js=l.split(' ',1); d=json.loads(js); print(tag,d['scene'],round(d['ms_per_trace'],3),round(d['ray_bounces_per_s']/1e9,3))"
timeout -k 10 400 $T tests -m gpu > gpurun_out/r3x_gpu.log 2>&1 || { tail -40 gpurun_out/r3x_gpu.log; exit 1; }
tail -1 gpurun_out/r3x_gpu.log
