#!/bin/bash
# round 3: hardware rsq/sqrt probe, reference-kernel parity report, sharded 2-process test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/rsq_probe gpurun_out/rsq_probe.bin > gpurun_out/probe.log 2>&1 || exit 1
rm -f gpurun_out/ref_parity.jsonl
LPC_REF_REPORT=gpurun_out/ref_parity.jsonl timeout -k 10 900 python -u -m pytest tests/test_ref_parity.py -v \
  --timeout 600 --timeout-method thread > gpurun_out/ref.log 2>&1
echo "ref rc $?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -v -x --timeout 300 --timeout-method thread \
  > gpurun_out/sharded.log 2>&1
rc=$?
echo "sharded rc $rc"
tail -5 gpurun_out/ref.log
tail -15 gpurun_out/sharded.log
exit $rc
