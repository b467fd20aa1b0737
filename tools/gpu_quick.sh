#!/bin/bash
# quick GPU iteration: parity tests (subset via PYTEST_ARGS) + traversal stats + bench
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/trace_stats.py synthetic 1000000 > gpurun_out/stats.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1 || exit $?
