R=$(pwd); O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python -u tools/results_mode.py parabolic 1000000 4 > $O/results.log 2>&1 || { tail $O/results.log; exit 1; }
tail -1 $O/results.log
timeout -k 10 700 python -u tools/ab.py 3 base: wb4k:LPC_Q_WALK_BLOCKS=4096 wb2k:LPC_Q_WALK_BLOCKS=2048 wb1536:LPC_Q_WALK_BLOCKS=1536 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
timeout -k 10 700 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,eye:2000000:16:1,lens:10000000:8:2,parabolic:1000000:4:5 base: wb4k:LPC_Q_WALK_BLOCKS=4096 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
