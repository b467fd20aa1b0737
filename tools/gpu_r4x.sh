R=$(pwd); O=gpurun_out/r4x; mkdir -p $O
AB_STEPS=500 timeout -k 10 900 python -u tools/ab.py 4 base: b20:LPC_BUDGET=20 b20lv3:LPC_BUDGET=20,LPC_SPILL_LEVELS=3 b16:LPC_BUDGET=16 lv3:LPC_SPILL_LEVELS=3 > $O/ab_spill3.log 2>&1 || { tail $O/ab_spill3.log; exit 1; }
tail -1 $O/ab_spill3.log
