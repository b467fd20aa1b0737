R=$(pwd); O=gpurun_out/r4l; mkdir -p $O
LPC_HOSTPROF=1 timeout -k 10 120 python -u tools/host_gap.py 20 > $O/host_gap.log 2>&1 || { tail $O/host_gap.log; exit 1; }
tail -1 $O/host_gap.log
timeout -k 10 400 python -u tools/ab.py 3 base: moveocc0:LPC_LIB_PATH=$R/lightpycl_amd/liblpc_moveocc0.so > $O/ab_move.log 2>&1 || { tail $O/ab_move.log; exit 1; }
tail -1 $O/ab_move.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/ktr -o kt --output-format csv -- python3 $R/tools/results_mode.py parabolic 1000000 2 > $R/$O/ktr.log 2>&1 ) || { echo ktr failed; exit 1; }
timeout -k 10 400 python -u tools/trace_stats.py eye 300000 > $O/stats_eye.log 2>&1 || { tail $O/stats_eye.log; exit 1; }
tail -30 $O/stats_eye.log
TAG=r4l bash tools/gpu_round.sh atomics && echo atomics ok
TAG=r4l bash tools/gpu_round.sh pmc && echo pmc ok
