#!/bin/bash
# GPU-box check: smoke -> gpu parity tests -> short bench.  Each GPU step has
# its own time limit; a crash/timeout (rc >= 124) stops the script, ordinary
# test failures (rc 1) do not.
mkdir -p gpurun_out
run() {  # run <limit> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "gpurun_out/$log"
  if [ $rc -ge 124 ] || [ $rc -eq 2 ] && [ "$log" != "pytest_gpu.log" ]; then echo "stop after $log rc=$rc"; exit $rc; fi
  if [ $rc -ge 124 ]; then echo "stop after $log rc=$rc"; exit $rc; fi
  return 0
}
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run ${PYTEST_LIMIT:-600} pytest_gpu.log python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
run 300 bench.log python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}
tail -n 3 gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench.log
