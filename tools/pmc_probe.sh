#!/bin/bash
# GPU box: SQ counter passes over one bench step (one rocprofv3 --pmc pass per
# counter group, nothing else collected), then per-dispatch rows of the named
# kernels: pmc_probe.sh [kernel-regex]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcp; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_LEVEL_WAVES SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_IFETCH GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o pmc --output-format csv -- \
      python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-configs > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
python3 $R/tools/pmc_rows.py $OUT "${1:-k_intersect|k_spill|k_slivers}"
