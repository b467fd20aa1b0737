#!/bin/bash
# GPU box: SQ counter passes of one bench step under two launch policies
# (e.g. LPC_QUEUE=0 vs 1), then per-kernel averages: pmc_ab.sh 'CFG_A' 'CFG_B'
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE"
j=0
for cfg in "$@"; do
  k=0
  for grp in "$G1" "$G2"; do
    ( [ -n "$cfg" ] && export $cfg; timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/c$j/p$k -o pmc --output-format csv -- \
      python3 $R/bench.py --steps 1 --warmup 1 --no-cpu > $OUT/c$j.p$k.log 2>&1 ) || { echo "cfg $cfg pass $k failed"; exit 1; }
    k=$((k+1))
  done
  j=$((j+1))
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
for j, cfg in enumerate(sys.argv[2:]):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{out}/c{j}/**/pmc_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if any(k in nm for k in ("k_intersect", "k_spill", "k_trav", "k_roots")):
                per[nm][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", cfg)
    for nm, cs in per.items():
        print("  ", nm[:30], " ".join(f"{c}={sum(v)/len(v):.3g}" for c, v in sorted(cs.items())), "launches", len(next(iter(cs.values()))))
PY
