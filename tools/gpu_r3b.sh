#!/bin/bash
# round 3: hardware rsq/sqrt probe, then the whole -m gpu suite (reference-kernel
# parity report in gpurun_out/ref_parity.jsonl)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/rsq_probe gpurun_out/rsq_probe.bin > gpurun_out/probe.log 2>&1 || exit 1
rm -f gpurun_out/ref_parity.jsonl
LPC_REF_REPORT=gpurun_out/ref_parity.jsonl timeout -k 10 1050 python -u -m pytest tests -m gpu -v \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -40
exit $rc
