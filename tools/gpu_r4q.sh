R=$(pwd); O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 900 python -u tools/ab.py 3 base: b12:LPC_BUDGET=12 b24:LPC_BUDGET=24 lv3:LPC_SPILL_LEVELS=3 lv5:LPC_SPILL_LEVELS=5 pb2:LPC_ROOTS_PB3=2 pb4:LPC_ROOTS_PB3=4 > $O/ab_spill.log 2>&1 || { tail $O/ab_spill.log; exit 1; }
tail -1 $O/ab_spill.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kte -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 2000000 16 1 > $R/$O/kte.log 2>&1 ) || { echo kte failed; exit 1; }
head -12 $O/kte/kt_kernel_stats.csv | cut -c1-150
