R=$(pwd); O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 600 python -u tools/ab_cfg.py 2 eye:2000000:16:2,lens:10000000:8:3 base: fork0:LPC_FORK_ROOTS_MIN=0 fork2m:LPC_FORK_ROOTS_MIN=2000000 > $O/ab_fork_cfg.log 2>&1 || { tail $O/ab_fork_cfg.log; exit 1; }
tail -1 $O/ab_fork_cfg.log
AB_STEPS=500 timeout -k 10 600 python -u tools/ab.py 3 base: fork0:LPC_FORK_ROOTS_MIN=0 > $O/ab_fork.log 2>&1 || { tail $O/ab_fork.log; exit 1; }
tail -1 $O/ab_fork.log
( cd /tmp && export TMPDIR=/tmp && LPC_FORK_ROOTS_MIN=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kte -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 2000000 16 1 > $R/$O/kte.log 2>&1 ) || { echo kte failed; exit 1; }
head -6 $O/kte/kt_kernel_stats.csv | cut -c1-100
