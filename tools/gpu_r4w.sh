R=$(pwd); O=gpurun_out/r4w; mkdir -p $O
AB_STEPS=500 timeout -k 10 900 python -u tools/ab.py 4 base: b24:LPC_BUDGET=24 lv3:LPC_SPILL_LEVELS=3 b24lv3:LPC_BUDGET=24,LPC_SPILL_LEVELS=3 b20:LPC_BUDGET=20 > $O/ab_spill2.log 2>&1 || { tail $O/ab_spill2.log; exit 1; }
tail -1 $O/ab_spill2.log
timeout -k 10 600 python -u tools/ab_cfg.py 2 eye:2000000:16:2,lens:10000000:8:3,synthetic_dense:1000000:16:3,parabolic:1000000:4:5 base: b24lv3:LPC_BUDGET=24,LPC_SPILL_LEVELS=3 > $O/ab_spill2_cfg.log 2>&1 || { tail $O/ab_spill2_cfg.log; exit 1; }
tail -1 $O/ab_spill2_cfg.log
