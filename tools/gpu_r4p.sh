R=$(pwd); O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 600 python -u tools/ab_cfg.py 2 eye:2000000:16:3 t100: t50:LPC_THIN=50 t25:LPC_THIN=25 t200:LPC_THIN=200 > $O/ab_thin_k.log 2>&1 || { tail $O/ab_thin_k.log; exit 1; }
tail -1 $O/ab_thin_k.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
TAG=r4p bash tools/gpu_round.sh pmc && echo pmc ok
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs > $R/$O/kt.log 2>&1 ) || { echo kt failed; exit 1; }
python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt; tail -3 $O/steps.txt
