#!/bin/bash
# Parity against the reference's own kernels (oracle/_ref) on the GPU box.
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ref_parity.jsonl
LPC_REF_REPORT=gpurun_out/ref_parity.jsonl timeout -k 10 1000 python -u -m pytest tests/test_ref_parity.py -v \
  --timeout 600 --timeout-method thread -s "$@" > gpurun_out/ref.log 2>&1
rc=$?
tail -30 gpurun_out/ref.log
exit $rc
