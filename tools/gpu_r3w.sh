#!/bin/bash
# round 3: hand-over knobs re-checked with more repetitions; the default bench
# line with the committed PMC summary current (roofline traffic / VALU filled)
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 900 python tools/ab.py 5 'base:' 'lv3:LPC_SPILL_LEVELS=3' 'ps4:LPC_PAIR_SHIFT=4' 'lv3ps4:LPC_SPILL_LEVELS=3,LPC_PAIR_SHIFT=4' > gpurun_out/r3w_ab.log 2>&1 || { tail -20 gpurun_out/r3w_ab.log; exit 1; }
tail -1 gpurun_out/r3w_ab.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err || { tail -20 gpurun_out/r3w_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3w_bench.json'));print(d['value'],d['ms_per_step'],json.dumps(d['roofline'])[:300],json.dumps(d['roofline_valu'])[:300])"
