R=$(pwd); O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u tools/ab_cfg.py 2 eye:2000000:16:3,lens:10000000:8:3,parabolic:1000000:4:5,synthetic_dense:1000000:16:3 base: nothin:LPC_THIN=0 > $O/ab_thin.log 2>&1 || { tail $O/ab_thin.log; exit 1; }
tail -1 $O/ab_thin.log
timeout -k 10 400 python -u tools/trace_stats.py eye 300000 > $O/stats_eye.log 2>&1 || { tail $O/stats_eye.log; exit 1; }
grep "exact/ray" $O/stats_eye.log | tail -12
