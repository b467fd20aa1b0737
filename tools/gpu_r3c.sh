#!/bin/bash
# round 3: hardware rsq/sqrt check, reference-kernel parity (report) and the
# liblpc-vs-oracle parity tests with the OpenCL-library arithmetic
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/rsq_check.py > gpurun_out/rsq_check.json 2> gpurun_out/rsq_check.err || exit 1
cat gpurun_out/rsq_check.json
rm -f gpurun_out/ref_parity.jsonl
LPC_REF_REPORT=gpurun_out/ref_parity.jsonl timeout -k 10 1000 python -u -m pytest tests/test_ref_parity.py \
  tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -40
exit $rc
