R=$(pwd); O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TAG=r4y bash tools/gpu_round.sh pmc && echo pmc ok
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs > $R/$O/kt.log 2>&1 ) || { echo kt failed; exit 1; }
python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt; tail -2 $O/steps.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kte -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 2000000 16 1 > $R/$O/kte.log 2>&1 ) || { echo kte failed; exit 1; }
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
