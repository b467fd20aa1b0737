R=$(pwd); O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "policies" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 800 python -u tools/ab_cfg.py 2 parabolic:1000000:4:5,synthetic:1000000:16:5 base: cap500k:LPC_DS_CAP=500000 nospec:LPC_SPEC=0 nobox:LPC_POPBOX=0 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
timeout -k 10 600 python -u tools/ab.py 3 base: x2:LPC_XCD_CLAIM=2 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
timeout -k 10 500 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,eye:2000000:16:1,lens:10000000:8:2 base: x2:LPC_XCD_CLAIM=2 > $O/ab_cfg2.log 2>&1 || { tail $O/ab_cfg2.log; exit 1; }
tail -1 $O/ab_cfg2.log
