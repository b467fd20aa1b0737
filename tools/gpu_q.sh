#!/bin/bash
# GPU box: smoke -> parity subset -> bench -> kernel trace (each step time-limited,
# stop at the first failure).
mkdir -p gpurun_out
R=$(pwd)
step() { local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$log 2>&1; local rc=$?; echo "rc=$rc" >> $R/gpurun_out/$log
  tail -n 4 $R/gpurun_out/$log
  if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; exit $rc; fi; }
step 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step ${PYTEST_LIMIT:-600} pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS}
step 200 bench.log python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu}
if [ -n "$KT" ]; then
  cd /tmp && export TMPDIR=/tmp
  step 300 kt.log rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu
fi
