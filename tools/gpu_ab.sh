#!/bin/bash
# GPU box: bench under several launch policies (one process each), then an
# optional kernel trace of the default: gpu_ab.sh 'LPC_X=1' 'LPC_Y=2 LPC_Z=0' ...
R=$(pwd); mkdir -p $R/gpurun_out
i=0
for cfg in "" "$@"; do
  ( [ -n "$cfg" ] && export $cfg; timeout -k 10 120 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu} > $R/gpurun_out/ab$i.log 2>&1 ) || { echo "cfg '$cfg' failed"; cat $R/gpurun_out/ab$i.log | tail -5; exit 1; }
  python - "$R/gpurun_out/ab$i.log" "$cfg" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(f"{sys.argv[2] or 'default':40s} {d['value']/1e6:8.1f} M/s  {d['ms_per_step']:.3f} ms/step  isect {d['roofline']['avg_launch_ms']*1e3:.1f} us")
PY
  i=$((i+1))
done
if [ -n "$KT" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/kt.log 2>&1 || { echo kt failed; exit 1; }
fi
