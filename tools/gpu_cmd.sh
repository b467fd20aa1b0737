mkdir -p gpurun_out/v
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 || { tail -5 gpurun_out/v/smoke.log; exit 1; }
tail -1 gpurun_out/v/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v/pytest.log 2>&1 || { tail -30 gpurun_out/v/pytest.log; exit 1; }
tail -1 gpurun_out/v/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/v/bench.log 2>&1 || { tail -5 gpurun_out/v/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/v/bench.log
