#!/bin/bash
# round 3: rehearsal of bench.py's N=2 path on the one-GPU box (both ranks on
# GPU 0, gloo exchange) -- checks the multi-rank line prints; not a measurement.
R=$(pwd); mkdir -p $R/gpurun_out
LPC_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 2 --no-cpu \
  > gpurun_out/r3y_n2.json 2> gpurun_out/r3y_n2.err || { tail -30 gpurun_out/r3y_n2.err; exit 1; }
cut -c1-600 gpurun_out/r3y_n2.json
