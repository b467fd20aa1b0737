R=$(pwd); O=gpurun_out/r4s; mkdir -p $O; L=$R/lightpycl_amd
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u tools/ab_cfg.py 2 eye:2000000:16:2 base: noprio:LPC_STREAM_PRIO=0 a2:LPC_LIB_PATH=$L/liblpc_a2.so > $O/ab_eye.log 2>&1 || { tail $O/ab_eye.log; exit 1; }
tail -1 $O/ab_eye.log
AB_STEPS=500 timeout -k 10 600 python -u tools/ab.py 3 base: noprio:LPC_STREAM_PRIO=0 > $O/ab_prio.log 2>&1 || { tail $O/ab_prio.log; exit 1; }
tail -1 $O/ab_prio.log
timeout -k 10 600 python -u tools/ab_cfg.py 2 lens:10000000:8:3,parabolic:1000000:4:5,synthetic_dense:1000000:16:3 base: noprio:LPC_STREAM_PRIO=0 > $O/ab_cfg_prio.log 2>&1 || { tail $O/ab_cfg_prio.log; exit 1; }
tail -1 $O/ab_cfg_prio.log
