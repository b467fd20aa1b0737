#!/bin/bash
# PC sampling of the bench (beta): where the walk kernels' waves sit
R=$(pwd); mkdir -p $R/gpurun_out/pcs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INT:-1048576} -d $R/gpurun_out/pcs -o pcs --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-configs > $R/gpurun_out/pcs/run.log 2>&1
rc=$?
echo "rc $rc"; tail -5 $R/gpurun_out/pcs/run.log
find $R/gpurun_out/pcs -name "*.csv" | head; du -sh $R/gpurun_out/pcs
