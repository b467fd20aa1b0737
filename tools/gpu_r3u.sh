#!/bin/bash
# round 3: four-group walk for launches without hand-over -- parity first, then
# A/B on the configs that use it (eye, lens, parabolic) and the headline
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "group_walk or policies" > gpurun_out/r3u_p.log 2>&1 || { tail -40 gpurun_out/r3u_p.log; exit 1; }
tail -1 gpurun_out/r3u_p.log
for v in 1 0 1 0; do
  LPC_GROUP=$v timeout -k 10 120 python tools/cfg_trace.py eye 1000000 16 1 | sed "s/^/g=$v /" >> gpurun_out/r3u_cfg.log 2>&1 || exit 1
  LPC_GROUP=$v timeout -k 10 120 python tools/cfg_trace.py lens 10000000 8 3 | sed "s/^/g=$v /" >> gpurun_out/r3u_cfg.log 2>&1 || exit 1
  LPC_GROUP=$v timeout -k 10 120 python tools/cfg_trace.py parabolic 1000000 4 20 | sed "s/^/g=$v /" >> gpurun_out/r3u_cfg.log 2>&1 || exit 1
done
grep scene gpurun_out/r3u_cfg.log | python -c "
import sys,json
for l in sys.stdin:
    tag,js=l.split(' ',1); d=json.loads(js); print(tag,d['scene'],round(d['ms_per_trace'],3),round(d['ray_bounces_per_s']/1e9,3))"
timeout -k 10 300 $T tests -m gpu > gpurun_out/r3u_gpu.log 2>&1 || { tail -40 gpurun_out/r3u_gpu.log; exit 1; }
tail -1 gpurun_out/r3u_gpu.log
