mkdir -p gpurun_out/diag
timeout -k 10 200 python tools/item_probe.py synthetic 1000000 > gpurun_out/diag/items.log 2>&1 && \
timeout -k 10 200 python tools/trace_stats.py synthetic 1000000 > gpurun_out/diag/stats.log 2>&1 && \
LPC_HOSTPROF=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/diag/hostprof.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/diag/bench20.log 2>&1
