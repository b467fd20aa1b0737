#!/bin/bash
# round 3 final evidence: smoke, the default bench line, kernel trace + PMC passes
# of the bench (profiles/r03_final_*), the eye's kernel trace + SQ pass
R=$(pwd); mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -30 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -20 gpurun_out/fin_bench.err; exit 1; }
cut -c1-300 gpurun_out/fin_bench.json
PROF_TAG=r03_final PROF_STEPS=3 bash tools/profile.sh || exit 1
python tools/pmc_summary.py gpurun_out/r03_final r03_final k_rootwalk > gpurun_out/fin_pmc_summary.txt 2>&1 || { tail -20 gpurun_out/fin_pmc_summary.txt; exit 1; }
python tools/kt_timeline.py gpurun_out/r03_final/kt 60 > gpurun_out/fin_timeline.txt
python tools/kt_steps.py gpurun_out/r03_final/kt > gpurun_out/fin_steps.txt
mkdir -p gpurun_out/eye; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/eye/kt -o kt --output-format csv -- python3 $R/tools/cfg_trace.py eye 1000000 16 1 > $R/gpurun_out/eye/kt.log 2>&1 || { tail -20 $R/gpurun_out/eye/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/eye/pmc_sq -o pmc --output-format csv -- python3 $R/tools/cfg_trace.py eye 300000 16 1 > $R/gpurun_out/eye/pmc.log 2>&1 || { tail -20 $R/gpurun_out/eye/pmc.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/eye/pmc_fetch -o pmc --output-format csv -- python3 $R/tools/cfg_trace.py eye 300000 16 1 > $R/gpurun_out/eye/pmcf.log 2>&1 || { tail -20 $R/gpurun_out/eye/pmcf.log; exit 1; }
echo done
