mkdir -p gpurun_out/v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v/pytest.log 2>&1 || { tail -30 gpurun_out/v/pytest.log; exit 1; }
tail -1 gpurun_out/v/pytest.log
BENCH_ARGS="--steps 30 --warmup 3 --no-cpu" bash tools/gpu_ab.sh 'LPC_SHADE_CFIRST=0' 'LPC_SHADE_CFIRST=1' 'LPC_SHADE_CFIRST=0' 'LPC_SHADE_CFIRST=1' 'LPC_SHADE_CFIRST=0' 'LPC_SHADE_CFIRST=1'
