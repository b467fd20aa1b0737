#!/bin/bash
R=$(pwd); mkdir -p gpurun_out/r4a
timeout -k 10 60 ./tools/_valu_issue 4096 > gpurun_out/r4a/valu_issue.json 2>&1 || { echo valu failed; cat gpurun_out/r4a/valu_issue.json; exit 1; }
cat gpurun_out/r4a/valu_issue.json
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r4a/valu_pmc -o pmc --output-format csv -- $R/tools/_valu_issue 4096 > $R/gpurun_out/r4a/valu_pmc.log 2>&1 ) || { echo valu pmc failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r4a/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u tools/results_mode.py parabolic 1000000 3 > gpurun_out/r4a/results_mode.json 2>&1 || { tail gpurun_out/r4a/results_mode.json; exit 1; }
cat gpurun_out/r4a/results_mode.json
timeout -k 10 600 python -u bench.py > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || { tail -20 gpurun_out/r4a/bench.err; exit 1; }
cut -c1-600 gpurun_out/r4a/bench.json
