#!/bin/bash
# round 3: golden fixtures from the reference kernels, the whole -m gpu suite, a bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/golden
timeout -k 10 300 python -u tests/golden/make_golden.py --out gpurun_out/golden > gpurun_out/golden.log 2>&1 || { tail -20 gpurun_out/golden.log; exit 1; }
rm -f gpurun_out/ref_parity.jsonl
LPC_REF_REPORT=gpurun_out/ref_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc $rc"
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -30
timeout -k 10 400 python -u bench.py --no-configs > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc $?"
tail -c 3000 gpurun_out/bench.json
timeout -k 10 400 python -u tools/ab.py 3 'base:' 'walk1536:LPC_Q_WALK_BLOCKS=1536' 'walk4096:LPC_Q_WALK_BLOCKS=4096' \
  'spill1024:LPC_SPILL_BLOCKS=1024' > gpurun_out/ab.jsonl 2>&1
tail -1 gpurun_out/ab.jsonl
exit $rc
