#!/bin/bash
# One GPU-box round of evidence (tools/gpu_round.sh [stage]): every GPU step under
# its own time limit, chained so that a failure or timeout ends the script.
R=$(pwd); O=gpurun_out/${TAG:-r4}; mkdir -p $O
run() { local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2>&1; local rc=$?
  echo "rc=$rc" >> $O/$log
  if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; tail -20 $O/$log; exit $rc; fi; }
prof() { local lim=$1 dir=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 $lim rocprofv3 "$@" ) ; }
case "${1:-all}" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -5 $O/pytest.log; [ $rc -ne 0 ] && exit $rc ;;
profile)
  # kernel trace of 3 bench steps, the dense scene's trace, per-iteration statistics
  prof 300 kt --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-strong > $O/kt.log 2>&1 || { echo kt failed; exit 1; }
  python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt
  prof 300 ktd --kernel-trace --stats -d $R/$O/ktd -o kt --output-format csv -- python3 $R/tools/cfg_trace.py synthetic_dense 1000000 16 1 > $O/ktd.log 2>&1 || { echo ktd failed; exit 1; }
  run 300 stats_dense.log python -u tools/trace_stats.py synthetic_dense 200000
  run 300 stats_synth.log python -u tools/trace_stats.py synthetic 1000000 ;;
pmc)
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -c1-10 | tr ' ' '_')
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/$O/pmc_$tag -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-strong > $R/$O/pmc_$tag.log 2>&1 ) || { echo "pmc $grp failed"; exit 1; }
  done
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/$O/valu_pmc -o pmc --output-format csv -- $R/tools/_valu_issue 4096 > $R/$O/valu_pmc.log 2>&1 ) || { echo valu pmc failed; exit 1; } ;;
atomics)
  # where the walk's writes go: memory-side atomic requests (64 B each) against
  # all write requests, per launch (one bench step: the primary and two secondaries)
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $R/$O/pmc_atomics -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-strong > $R/$O/pmc_atomics.log 2>&1 ) || { echo "pmc atomics failed"; exit 1; } ;;
eye)
  # kernel trace of one eye trace (2 M rays, 16 iterations) after two warm-up traces
  prof 300 kte --kernel-trace --stats -d $R/$O/kte -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 2000000 16 1 > $O/kte.log 2>&1 || { echo kte failed; exit 1; } ;;
all)
  # the round's evidence: GPU tests, PMC passes, kernel traces, the bench line
  for st in tests pmc profile eye bench; do bash $0 $st || exit 1; done ;;
hostgap)
  LPC_HOSTPROF=1 run 120 host_gap.log python -u tools/host_gap.py 20 ;;
results)
  run 300 results_mode.json python -u tools/results_mode.py parabolic 1000000 5 ;;
ab)
  run 900 ab.log python -u tools/ab.py ${AB_REPS:-3} $AB_CFGS ;;
bench)
  run 900 bench.json python -u bench.py ;;
esac
