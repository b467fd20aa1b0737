mkdir -p gpurun_out/sweep
SWEEP_ASYNC=1 SWEEP_STEPS=10 timeout -k 10 300 python -u tools/sweep.py synthetic 1000000 5 FORK_LATE=1 FORK_LATE=0 FORK_LATE=1,KEY=0 EV_SYSFENCE=0 > gpurun_out/sweep/aba.log 2>&1 || { tail -5 gpurun_out/sweep/aba.log; exit 1; }
grep -v amdgpu gpurun_out/sweep/aba.log
SWEEP_ASYNC=1 SWEEP_STEPS=10 timeout -k 10 300 python -u tools/sweep.py lens 1000000 5 FORK_LATE=1 FORK_LATE=0 FORK_LATE=1,KEY=0 > gpurun_out/sweep/aba2.log 2>&1 || { tail -5 gpurun_out/sweep/aba2.log; exit 1; }
grep -v amdgpu gpurun_out/sweep/aba2.log
bash tools/kt_cfg.sh 'LPC_ROOTS_TASKS=0' 'LPC_ROOTS_TASKS=4096' 'LPC_ROOTS_S=0' > gpurun_out/sweep/kt.log 2>&1 || { tail -5 gpurun_out/sweep/kt.log; exit 1; }
