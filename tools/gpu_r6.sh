#!/bin/bash
# Round-6 GPU evidence stages (tools/gpu_r6.sh stage ...): every GPU step under
# its own time limit, chained so a failure or timeout ends the script.
R=$(pwd); O=gpurun_out/${TAG:-r6}; mkdir -p $O
export LPC_TEST_OUT=$R/$O
run() { local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2>&1; local rc=$?
  echo "rc=$rc" >> $O/$log
  if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; tail -30 $O/$log; exit $rc; fi; }
prof() { ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 $1 rocprofv3 "${@:2}" ) ; }
for st in "$@"; do case "$st" in
new) run 900 pytest_new.log python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_capacity.py tests/test_gpu_fullsize.py -s ;;
cap) run 600 pytest_cap.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_capacity.py ;;
full) run 900 pytest_full.log python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -s ;;
tests) run 1100 pytest.log python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ;;
sel) run 900 pytest_sel.log python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $SEL ;;
freshab) for p in 1 2; do for m in 0 1 2; do LPC_STAGE_MODE=$m run 300 fresh_m${m}_p$p.json python -u tools/fresh_probe.py; done; done
         for m in 0 1 2; do LPC_HOSTPROF=1 LPC_STAGE_MODE=$m run 300 fresh_hp_m$m.json python -u tools/fresh_probe.py; done ;;
fresh) LPC_HOSTPROF=${HP:-0} run 300 fresh.json python -u tools/fresh_probe.py ;;
stream) run 600 pytest_stream.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream.py ;;
dispatch) run 120 dispatch.json tools/_dispatch_probe ;;
quick) run 300 quick.json python -u bench.py --no-cpu --no-configs --no-strong ;;
bench) run 900 bench.json python -u bench.py ;;
ab) AB_STEPS=${AB_STEPS:-300} run 900 ab.log python -u tools/ab.py ${AB_REPS:-3} $AB_CFGS ;;
abcfg) run 900 abcfg.log python -u tools/ab_cfg.py $ABCFG_ARGS ;;
stats) run 300 stats_synth.log python -u tools/trace_stats.py synthetic 1000000
       run 300 stats_dense.log python -u tools/trace_stats.py synthetic_dense 200000 ;;
stats_eye) run 300 stats_eye.log python -u tools/trace_stats.py eye 300000 ;;
kt) prof 300 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-strong $KT_ARGS > $O/kt.log 2>&1 || { echo kt failed; exit 1; }
    python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt ;;
ktstats) prof 300 --kernel-trace --stats -d $R/$O/kts -o kts --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu --no-configs --no-strong > $O/kts.log 2>&1 || { echo ktstats failed; exit 1; } ;;
pmcwalk) for grp in "$PMC1" "$PMC2" "$PMC3"; do [ -z "$grp" ] && continue; tag=$(echo $grp | md5sum | cut -c1-6)
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/$O/pmc_$tag -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-strong > $R/$O/pmc_$tag.log 2>&1 ) || { echo "pmc $grp failed"; exit 1; }
      echo "$grp" > $O/pmc_$tag.groups; done ;;
esac; done
exit 0
