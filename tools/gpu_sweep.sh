#!/bin/bash
# GPU box: optional parity subset, then tools/sweep.py A/B of launch policies on
# one or more scenes: SWEEP_SCENES="synthetic:1000000 lens:1000000" gpu_sweep.sh 'X=0' 'X=1'
R=$(pwd); mkdir -p $R/gpurun_out/sweep
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > $R/gpurun_out/sweep/pytest.log 2>&1
  rc=$?; tail -n 3 $R/gpurun_out/sweep/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for sn in ${SWEEP_SCENES:-synthetic:1000000}; do
  s=${sn%%:*}; n=${sn##*:}
  timeout -k 10 300 python -u tools/sweep.py $s $n ${SWEEP_ROUNDS:-5} "$@" > $R/gpurun_out/sweep/$s.log 2>&1 || { echo "sweep $s failed"; tail -5 $R/gpurun_out/sweep/$s.log; exit 1; }
  echo "== $s $n"; grep -v amdgpu.ids $R/gpurun_out/sweep/$s.log
done
