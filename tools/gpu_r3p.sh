#!/bin/bash
# round 3: chunked second sort level; re-sort of large chained populations by
# default -- parity, all GPU tests, A/B, kernel trace, configs
R=$(pwd); mkdir -p $R/gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "counting_sort or resort" > gpurun_out/r3p_bs.log 2>&1 || { tail -40 gpurun_out/r3p_bs.log; exit 1; }
tail -1 gpurun_out/r3p_bs.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/r3p_gpu.log 2>&1 || { tail -40 gpurun_out/r3p_gpu.log; exit 1; }
tail -1 gpurun_out/r3p_gpu.log
timeout -k 10 600 python tools/ab.py 3 'base:' 'radix:LPC_BSORT=0' > gpurun_out/r3p_ab.log 2>&1 || { tail -20 gpurun_out/r3p_ab.log; exit 1; }
tail -1 gpurun_out/r3p_ab.log
mkdir -p gpurun_out/prof_r3p; (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3p/kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/prof_r3p/kt.log 2>&1) || { tail -20 gpurun_out/prof_r3p/kt.log; exit 1; }
python tools/kt_steps.py gpurun_out/prof_r3p/kt | tail -3
python tools/kt_timeline.py gpurun_out/prof_r3p/kt 40 > gpurun_out/prof_r3p/timeline.txt
grep -E "k_b|gather|roots_s" gpurun_out/prof_r3p/timeline.txt | head -8
timeout -k 10 600 python -u bench.py --steps 200 > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err || { tail -20 gpurun_out/r3p_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3p_bench.json'));print(d['value'],d['ms_per_step'],json.dumps(d['parity'].get('vs_reference_kernels')),json.dumps({k:(v['ray_bounces_per_s'],v['ms_per_trace']) for k,v in d['configs'].items()}))"
