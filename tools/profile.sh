#!/bin/bash
# GPU-box profiling of bench.py: kernel trace + stats, then PMC passes (one
# counter group per pass, --pmc never combined with trace domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="--steps ${PROF_STEPS:-3} --warmup 1 --no-cpu --no-configs ${BENCH_EXTRA}"
step() { local lim=$1 name=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi; }
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
step 300 kt rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py $B
step 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs ${BENCH_EXTRA}
step 300 pmc_write rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs ${BENCH_EXTRA}
step 300 pmc_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs ${BENCH_EXTRA}
echo done
