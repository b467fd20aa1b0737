#!/bin/bash
# Round-5 GPU evidence stages (tools/gpu_r5.sh stage): every GPU step under its
# own time limit, chained so a failure or timeout ends the script.
R=$(pwd); O=gpurun_out/${TAG:-r5}; mkdir -p $O
run() { local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2>&1; local rc=$?
  echo "rc=$rc" >> $O/$log
  if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; tail -20 $O/$log; exit $rc; fi; }
prof() { ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 $1 rocprofv3 "${@:2}" ) ; }
for st in "$@"; do case "$st" in
pinned) run 120 pinned.log python -u tools/pinned_probe.py ;;
results) run 300 results_mode.log python -u tools/results_mode.py parabolic 1000000 6 ;;
results_var) RM_GC=0 run 300 results_nogc.log python -u tools/results_mode.py parabolic 1000000 6
             LPC_HOSTPROF=1 run 300 results_hostprof.log python -u tools/results_mode.py parabolic 1000000 4 ;;
ab) AB_STEPS=${AB_STEPS:-300} run 900 ab.log python -u tools/ab.py ${AB_REPS:-3} $AB_CFGS ;;
listpmc) ( cd /tmp && timeout -k 10 120 rocprofv3 --list-avail ) > $O/pmc_list.txt 2>&1 || { echo list failed; exit 1; } ;;
pmcwalk) for grp in "$PMC1" "$PMC2" "$PMC3"; do [ -z "$grp" ] && continue; tag=$(echo $grp | md5sum | cut -c1-6)
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/$O/pmc_$tag -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-strong > $R/$O/pmc_$tag.log 2>&1 ) || { echo "pmc $grp failed"; exit 1; }
      echo "$grp" > $O/pmc_$tag.groups; done ;;
dispatch) hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o tools/_dispatch_probe && run 60 dispatch.json tools/_dispatch_probe ;;
stats) run 300 stats_synth.log python -u tools/trace_stats.py synthetic 1000000
       run 300 stats_dense.log python -u tools/trace_stats.py synthetic_dense 200000 ;;
stats_eye) run 300 stats_eye.log python -u tools/trace_stats.py eye 300000 ;;
kt) prof 300 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-strong > $O/kt.log 2>&1 || { echo kt failed; exit 1; }
    python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt ;;
kthip) prof 300 --kernel-trace --hip-runtime-trace --output-format csv -d $R/$O/kth -o kth -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-strong > $O/kth.log 2>&1 || { echo kthip failed; exit 1; } ;;
bench) run 600 bench.json python -u bench.py ;;
quick) run 300 quick.json python -u bench.py --no-cpu --no-configs --no-strong ;;
tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
       rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc ;;
esac; done
exit 0
