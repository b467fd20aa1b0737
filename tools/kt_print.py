"""Print per-kernel totals of the kt_cfg.sh runs (rocprofv3 kernel_stats.csv)."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p))):
    cfg = open(os.path.join(d, "cfg.txt")).read().strip()
    st = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    b = [l for l in open(os.path.join(d, "bench.log")) if l.startswith("{")]
    v = json.loads(b[-1]) if b else {}
    if not v:
        v = {"value": 0, "ms_per_step": 0}
        for l in open(os.path.join(d, "bench.log")):
            if "ms/step" in l:
                print("   " + l.strip()[:100])
    print(f"== {cfg}: {v.get('value', 0) / 1e6:.1f} M/s, {v.get('ms_per_step', 0):.3f} ms/step")
    if not st:
        continue
    rows = list(csv.DictReader(open(st[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:14]:
        print(f"   {r['Name'].split('(')[0][:44]:44s} n={int(r['Calls']):5d} avg={float(r['AverageNs']) / 1e3:8.1f} us "
              f"max={float(r['MaxNs']) / 1e3:8.1f} tot={float(r['TotalDurationNs']) / 1e6:7.2f} ms")
