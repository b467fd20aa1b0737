R=$(pwd); O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u tools/ab.py 3 base: nospec2:LPC_RESORT_MIN=1999999 noprof:ARGS=--no-prof nobox:LPC_POPBOX=0 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
timeout -k 10 900 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,lens:10000000:8:3,eye:2000000:16:1 base: nobox:LPC_POPBOX=0 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
