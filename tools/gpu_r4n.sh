R=$(pwd); O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=$R/lightpycl_amd
timeout -k 10 600 python -u tools/ab.py 3 base: prev:LPC_LIB_PATH=$L/liblpc_prev.so minb7:LPC_LIB_PATH=$L/liblpc_minb7.so minb5:LPC_LIB_PATH=$L/liblpc_minb5.so > $O/ab_walkregs.log 2>&1 || { tail $O/ab_walkregs.log; exit 1; }
tail -1 $O/ab_walkregs.log
TAG=r4n bash tools/gpu_round.sh atomics && echo atomics ok
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_WRITE_SIZE -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs > $R/$O/pmc_WRITE_SIZE.log 2>&1 ) && echo write ok
timeout -k 10 900 python -u tools/ab_cfg.py 2 eye:2000000:16:3,lens:10000000:8:3,synthetic_dense:1000000:16:3 base: half1:LPC_HALF=1 half2:LPC_HALF=2 > $O/ab_half.log 2>&1 || { tail $O/ab_half.log; exit 1; }
tail -1 $O/ab_half.log
