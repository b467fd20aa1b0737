R=$(pwd); O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-configs > $R/$O/kt.log 2>&1 ) || { echo kt failed; exit 1; }
python tools/kt_timeline.py $O/kt 60 > $O/timeline.txt; python tools/kt_steps.py $O/kt > $O/steps.txt
timeout -k 10 600 python -u tools/ab.py 3 base: rpb2048:LPC_LIB_PATH=$R/lightpycl_amd/liblpc_rpb2048.so rpb1024:LPC_LIB_PATH=$R/lightpycl_amd/liblpc_rpb1024.so > $O/ab_rpb.log 2>&1 || { tail $O/ab_rpb.log; exit 1; }
tail -1 $O/ab_rpb.log
timeout -k 10 700 python -u tools/ab_cfg.py 2 synthetic_dense:1000000:16:1,eye:2000000:16:1 base: m7:LPC_KEY_OBITS=7 m5:LPC_KEY_OBITS=5 > $O/ab_cfg.log 2>&1 || { tail $O/ab_cfg.log; exit 1; }
tail -1 $O/ab_cfg.log
