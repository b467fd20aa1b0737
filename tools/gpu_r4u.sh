R=$(pwd); O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 700 python -u tools/ab_cfg.py 2 eye:2000000:16:2,lens:10000000:8:3,synthetic_dense:1000000:16:3,parabolic:1000000:4:5 base: merge:LPC_SLIVER_MERGE=1 merge8:LPC_SLIVER_MERGE=1,LPC_SLIVER_MERGE_PPW=8 > $O/ab_merge_cfg.log 2>&1 || { tail $O/ab_merge_cfg.log; exit 1; }
tail -1 $O/ab_merge_cfg.log
AB_STEPS=500 timeout -k 10 600 python -u tools/ab.py 3 base: merge:LPC_SLIVER_MERGE=1 merge1:LPC_SLIVER_MERGE=1,LPC_SLIVER_MERGE_PPW=1 > $O/ab_merge.log 2>&1 || { tail $O/ab_merge.log; exit 1; }
tail -1 $O/ab_merge.log
