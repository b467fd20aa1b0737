R=$(pwd); O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "resorted_populations" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 1100 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,lens:10000000:8:2,eye:2000000:16:1 base: ob4:LPC_KEY_OBITS=4 m6:LPC_KEY_MODE=1,LPC_KEY_OBITS=6 m5:LPC_KEY_MODE=1,LPC_KEY_OBITS=5 dm5:LPC_KEY_MODE=2 dm4:LPC_KEY_MODE=2,LPC_KEY_OBITS=4 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
