R=$(pwd); O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 env LPC_HOSTPROF=1 python -u tools/results_mode.py parabolic 1000000 3 > $O/results_hostprof.log 2>&1 || { tail $O/results_hostprof.log; exit 1; }
tail -1 $O/results_hostprof.log
timeout -k 10 700 python -u tools/ab.py 3 base: hsmall:LPC_HALF_SMALL=1 du16:LPC_DRAIN_U=16 du32:LPC_DRAIN_U=32 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
timeout -k 10 800 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,eye:2000000:16:1,lens:10000000:8:2 base: half1:LPC_HALF=1 lpt4:LPC_LARGE_PER_TRI=4 lpt64:LPC_LARGE_PER_TRI=64 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
