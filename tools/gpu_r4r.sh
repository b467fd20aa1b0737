R=$(pwd); O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 900 python -u tools/ab_cfg.py 2 eye:2000000:16:2 base: rs16:LPC_ROOTS_S=16 sw64k:LPC_SLIVER_WAVES=65536 sw4k:LPC_SLIVER_WAVES=4096 > $O/ab_eye_roots.log 2>&1 || { tail $O/ab_eye_roots.log; exit 1; }
tail -1 $O/ab_eye_roots.log
( cd /tmp && export TMPDIR=/tmp && LPC_ROOTS_S=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kte -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 2000000 16 1 > $R/$O/kte.log 2>&1 ) || { echo kte failed; exit 1; }
head -6 $O/kte/kt_kernel_stats.csv | cut -c1-120
