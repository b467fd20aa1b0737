export TAG=r4c
mkdir -p gpurun_out/r4c
timeout -k 10 300 env LPC_HOSTPROF=1 python -u tools/results_mode.py parabolic 1000000 3 > gpurun_out/r4c/results_hostprof.log 2>&1 || { tail gpurun_out/r4c/results_hostprof.log; exit 1; }
timeout -k 10 300 env LPC_HOSTPROF=1 python -u bench.py --steps 4 --warmup 2 --no-cpu --no-configs > gpurun_out/r4c/bench_hostprof.log 2>&1 || { tail gpurun_out/r4c/bench_hostprof.log; exit 1; }
timeout -k 10 1000 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,parabolic:1000000:4:5,lens:10000000:8:3,eye:2000000:16:1,synthetic:1000000:16:5 base: r500k:LPC_RESORT_MIN=500000 r250k:LPC_RESORT_MIN=250000 > gpurun_out/r4c/ab_resort.log 2>&1 || { tail gpurun_out/r4c/ab_resort.log; exit 1; }
tail -1 gpurun_out/r4c/ab_resort.log
