R=$(pwd); O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_results.py -x -q --timeout 120 --timeout-method thread > $O/pytest_results.log 2>&1 || { tail -30 $O/pytest_results.log; exit 1; }
tail -1 $O/pytest_results.log
timeout -k 10 300 python -u tools/results_mode.py parabolic 1000000 4 > $O/results.log 2>&1 || { tail $O/results.log; exit 1; }
tail -1 $O/results.log
LPC_HOSTPROF=1 timeout -k 10 120 python -u tools/host_gap.py 20 > $O/host_gap.log 2>&1 || { tail $O/host_gap.log; exit 1; }
tail -1 $O/host_gap.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/ktr -o kt --output-format csv -- python3 $R/tools/results_mode.py parabolic 1000000 2 > $R/$O/ktr.log 2>&1 ) || { echo ktr failed; exit 1; }
timeout -k 10 600 python -u tools/ab_cfg.py 2 parabolic:1000000:4:5,synthetic:1000000:16:5 base: nospec:LPC_SPEC=0 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 400 python -u tools/trace_stats.py eye 300000 > $O/stats_eye.log 2>&1 || { tail $O/stats_eye.log; exit 1; }
tail -30 $O/stats_eye.log
