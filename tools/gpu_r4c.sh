export TAG=r4c
R=$(pwd); O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "policies or traced_order" > $O/pytest_pol.log 2>&1 || { tail -30 $O/pytest_pol.log; exit 1; }
tail -2 $O/pytest_pol.log
timeout -k 10 300 env LPC_HOSTPROF=1 python -u tools/results_mode.py parabolic 1000000 3 > $O/results_hostprof.log 2>&1 || { tail $O/results_hostprof.log; exit 1; }
timeout -k 10 300 env LPC_HOSTPROF=1 python -u bench.py --steps 4 --warmup 2 --no-cpu --no-configs > $O/bench_hostprof.log 2>&1 || { tail $O/bench_hostprof.log; exit 1; }
for cfg in "" "LPC_XCD_CLAIM=1"; do
  tag=$( [ -n "$cfg" ] && echo claim || echo base )
  ( cd /tmp && export TMPDIR=/tmp && [ -n "$cfg" ] && export $cfg; timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$O/tcc_$tag -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-configs > $R/$O/tcc_$tag.log 2>&1 ) || { echo "tcc $tag failed"; exit 1; }
  ( cd /tmp && export TMPDIR=/tmp && [ -n "$cfg" ] && export $cfg; timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$O/tccd_$tag -o pmc --output-format csv -- python3 $R/tools/cfg_trace.py synthetic_dense 200000 16 1 > $R/$O/tccd_$tag.log 2>&1 ) || { echo "tccd $tag failed"; exit 1; }
done
timeout -k 10 600 python -u tools/ab.py 3 base: claim:LPC_XCD_CLAIM=1 > $O/ab_claim.log 2>&1 || { tail $O/ab_claim.log; exit 1; }
tail -1 $O/ab_claim.log
timeout -k 10 900 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,parabolic:1000000:4:5,lens:10000000:8:3,eye:2000000:16:1 base: r250k:LPC_RESORT_MIN=250000 claim:LPC_XCD_CLAIM=1 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
