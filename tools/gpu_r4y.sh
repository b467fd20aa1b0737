R=$(pwd); O=gpurun_out/r4final3; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r4final3 bash tools/gpu_round.sh pmc && echo pmc ok
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs > $R/$O/kt.log 2>&1 ) || { echo kt failed; exit 1; }
python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt; tail -2 $O/steps.txt
