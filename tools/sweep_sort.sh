mkdir -p gpurun_out
timeout -k 10 200 python tools/sweep.py synthetic 1000000 11 "KEY=5,CHAIN=0" "KEY=5" "ONESWEEP_MIN=50000" "SORT=2" "ONESWEEP_MIN=50000,SORT_MIN=1000000" "SORT_MIN=100000" > gpurun_out/sweep9_syn.log 2>&1; rc=$?; cat gpurun_out/sweep9_syn.log | cut -c1-200; exit $rc
