#!/bin/bash
# GPU box: stall breakdown of bench.py's kernels (two --pmc passes of SQ counters;
# SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, quad-cycles).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-stalls}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="--steps 1 --warmup 0 --no-cpu ${BENCH_EXTRA}"
step() { local lim=$1 name=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi; }
step 300 kt rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu
step 300 pmc_a rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_a -o pmc --output-format csv -- python3 $R/bench.py $B
step 300 pmc_b rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVES -d $OUT/pmc_b -o pmc --output-format csv -- python3 $R/bench.py $B
step 300 pmc_c rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_c -o pmc --output-format csv -- python3 $R/bench.py $B
step 300 pmc_d rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_d -o pmc --output-format csv -- python3 $R/bench.py $B
echo done
