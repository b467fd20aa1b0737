R=$(pwd); O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "resorted_populations" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 env LPC_HOSTPROF=1 python -u bench.py --steps 3 --warmup 2 --no-cpu --no-configs > $O/bench_hostprof.log 2>&1 || { tail $O/bench_hostprof.log; exit 1; }
timeout -k 10 1000 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,lens:10000000:8:2,eye:2000000:16:1 base: ob6:LPC_KEY_OBITS=6 ob7:LPC_KEY_OBITS=7 ob4:LPC_KEY_OBITS=4 r250k:LPC_RESORT_MIN=250000 claim:LPC_XCD_CLAIM=1 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
